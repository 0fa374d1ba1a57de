"""ADV_ISONEUTRAL: the rotated biharmonic tracer operator (step3d_t_ISO.F:253-846,
with SW_TRIADS and STABILIZE, :15-18) and its inputs -- the corrector prsgrd's
slopes dRdx/dRde (prsgrd.F:307-338, 423-453) and step3d_uv2's diff3u/diff3v/
idRz (step3d_uv2.F:572-697) -- in oracle/oracle_iso.c (two-slice recursive
form, like the reference) and ucla-roms_amd/csrc/k_iso.hip (full 3-D fields).

Parity is unpinned to reference output: the only reference case that defines
ADV_ISONEUTRAL (tests/Flux_frc) reads input_data that is not checked in.  So:
  * CPU: the oracle's slope and limiter formulas against a numpy evaluation
    of the same Fortran expressions on the oracle's own state (interior cells
    away from the edges, where the reference reads unset scratch -- see
    oracle_iso.c), and the switch changes the run;
  * GPU: whole steps against the oracle (closed basin with split EOS and KPP,
    open basin with an island, periodic Filament with the linear EOS), and a
    2x2 decomposition bitwise equal to the single domain (exchanged slopes,
    idRz, diff3u/v).
"""
import numpy as np
import pytest

import oracle

QP2, G = 0.0000172, 9.81


def iso_cfg(LLm=24, MMm=16, N=12, lmd=oracle.LMD_ICELAND, obc=0, island=0, iso=1):
    c = oracle.OrCfg()
    c.LLm, c.MMm, c.N, c.NT = LLm, MMm, N, 2
    c.ew_periodic = c.ns_periodic = 0
    c.salinity, c.nonlin_eos, c.lmd, c.surf_flux = 1, 1, lmd, 1
    c.case_id = oracle.CASE_BASIN
    c.dt, c.ndtfast = 60.0, 30
    c.theta_s, c.theta_b, c.hc, c.rho0 = 6.0, 2.0, 250.0, 1027.5
    c.rdrg, c.rdrg2, c.Zob = 0.0, 1.0e-3, 1.0e-2
    c.Akv_bak = 1.0e-4
    c.Akt_bak[0] = c.Akt_bak[1] = 1.0e-5
    c.Tcoef, c.T0, c.Scoef, c.S0 = 0.20, 1.0, 0.822, 1.0
    c.sizex, c.sizey = 3.0e3 * LLm, 3.0e3 * MMm
    c.diag_np_xi = c.diag_np_eta = 1
    c.obc, c.ubind, c.island = obc, 0.1, island
    c.adv_isoneutral = iso
    return c


def _rx(R, Q, Z, msk, axis):
    """prsgrd's elementary adiabatic difference at faces m (between m-1 and m) along axis."""
    sl = [slice(None)] * R.ndim
    lo, hi = list(sl), list(sl)
    lo[axis], hi[axis] = slice(0, -1), slice(1, None)
    lo, hi = tuple(lo), tuple(hi)
    dpth = -0.5 * (Z[hi] + Z[lo])
    out = np.zeros_like(R)
    out[hi] = (R[hi] - R[lo] + (Q[hi] - Q[lo]) * dpth * (1.0 - QP2 * dpth)) * msk[hi]
    return out


def test_oracle_iso_slopes_and_limiter_formulas():
    """or_prsgrd (corrector) and or_step3d_uv2 on a mid-run state: dRdx, dRde,
    diff3u, diff3v and idRz equal a numpy evaluation of the reference's
    expressions on the oracle's own arrays (rtol 1e-12)."""
    cfg = iso_cfg()
    o = oracle.Oracle(cfg)
    o.init()
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    o.set_tindex([iic, kstp, knew, nstp, 3, 3 - nstp])   # the corrector's indices (main.F:425)
    o.L.or_rho_eos(o.h, 3)
    o.L.or_prsgrd(o.h)
    Lm, Mm, N = cfg.LLm, cfg.MMm, cfg.N
    r0g = cfg.rho0 / G
    R, Q, Z = o.field("rho1"), o.field("qp1"), o.field("z_r")
    f2 = lambda n: o.field(n).reshape(R.shape[1:])   # 2-D fields as (ny2, nx2)
    f, pm, pn = f2("f"), f2("pm"), f2("pn")
    rx = _rx(R, Q, Z, f2("umask")[None], 2)
    ry = _rx(R, Q, Z, f2("vmask")[None], 1)
    # interior faces whose three rx are all computed by prsgrd: i = 3..Lm-1 (array index i+1)
    I, J = slice(4, Lm + 1), slice(2, Mm + 2)
    fs = f[:, 1:] + f[:, :-1]
    want = np.zeros_like(R)
    want[:, :, 1:] = 0.5 * (pm[:, 1:] + pm[:, :-1]) * (
        r0g * 0.25 * (fs * fs) * (Z[:, :, 1:] - Z[:, :, :-1]) - 0.5 * rx[:, :, 1:]
        - 0.25 * (rx[:, :, :-1] + np.roll(rx, -1, axis=2)[:, :, 1:]))
    np.testing.assert_allclose(o.field("dRdx")[:, J, I], want[:, J, I], rtol=1e-12, atol=1e-300)
    I, J = slice(2, Lm + 2), slice(4, Mm + 1)
    fs = f[1:] + f[:-1]
    want = np.zeros_like(R)
    want[:, 1:] = 0.5 * (pn[1:] + pn[:-1]) * (
        r0g * 0.25 * (fs * fs) * (Z[:, 1:] - Z[:, :-1]) - 0.5 * ry[:, 1:]
        - 0.25 * (ry[:, :-1] + np.roll(ry, -1, axis=1)[:, 1:]))
    np.testing.assert_allclose(o.field("dRde")[:, J, I], want[:, J, I], rtol=1e-12, atol=1e-300)
    assert np.abs(o.field("dRdx")).max() > 0 and np.abs(o.field("dRde")).max() > 0

    # step3d_uv2's diff3u/v and idRz (inputs: u,v(nnew) after the call, rho1/qp1 of
    # rho_eos(nrhs), hbls/hbbl, the slopes above)
    o.L.or_step3d_uv2(o.h)
    _, _, _, _, _, nnew = o.tindex()
    u = o.field("u")[(nnew - 1) * N:nnew * N]
    v = o.field("v")[(nnew - 1) * N:nnew * N]
    dm_u, dn_v = f2("dm_u"), f2("dn_v")
    I, J = slice(2, Lm + 2), slice(2, Mm + 2)
    gam = 0.0833333333333
    np.testing.assert_allclose(o.field("diff3u")[:, J, I], (np.sqrt(gam * np.abs(u) * dm_u) * dm_u)[:, J, I],
                               rtol=1e-13)
    np.testing.assert_allclose(o.field("diff3v")[:, J, I], (np.sqrt(gam * np.abs(v) * dn_v) * dn_v)[:, J, I],
                               rtol=1e-13)
    X, E, zw = o.field("dRdx"), o.field("dRde"), o.field("z_w")
    hbls, hbbl = f2("hbls"), f2("hbbl")
    dpth = -0.5 * (Z[1:] + Z[:-1])
    dRz = R[:-1] - R[1:] + (Q[:-1] - Q[1:]) * dpth * (1. - 2. * QP2 * dpth)
    dRz = np.maximum(dRz, 0.) + r0g * (f * f) * (Z[1:] - Z[:-1])
    aX, aE = np.abs(X), np.abs(E)
    mx = np.maximum(aX[:-1], aX[1:])
    me = np.maximum(aE[:-1], aE[1:])
    dRx_max = np.maximum(np.maximum(dm_u * mx, np.roll(dm_u * mx, -1, axis=2)),
                         np.maximum(dn_v * me, np.roll(dn_v * me, -1, axis=1)))
    cfs = np.minimum(1., (zw[N] - zw[1:N]) / np.maximum(50., hbls))
    cfb = np.minimum(1., (zw[1:N] - zw[0]) / np.maximum(50., hbbl))
    cff = 2. * cfs * (2. - cfs) * cfb * (2. - cfb)
    want = cff / np.maximum(np.maximum(cff * dRz, dRx_max), 1e-33)
    got = o.field("idRz")[1:N]
    np.testing.assert_allclose(got[:, J, I], want[:, J, I], rtol=1e-12)
    assert np.abs(got[:, J, I]).max() > 0


def test_oracle_iso_changes_the_run():
    """The switch changes T and S (centred fluxes + the rotated operator + Akz)
    and keeps the run finite; Akz > 0 somewhere (STABILIZE)."""
    t = {}
    for iso in (0, 1):
        o = oracle.Oracle(iso_cfg(iso=iso))
        o.init()
        o.step(5)
        t[iso] = o.field("t").copy()
        assert np.isfinite(t[iso]).all()
        if iso:
            assert o.field("Akz").max() > 0
    assert not np.array_equal(t[0], t[1])


# ---------------------------------------------------------------- GPU parity

def _model(cfg, **kw):
    import romsgpu
    per = cfg.case_id == oracle.CASE_FILAMENT
    return romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                   nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                   sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd,
                                   surf_flux=False if per else bool(cfg.surf_flux), obc=cfg.obc,
                                   island=bool(cfg.island), adv_isoneutral=bool(cfg.adv_isoneutral), **kw)


def _gpu_case(kind):
    if kind == "filament":   # periodic both ways, linear EOS, no KPP
        c = oracle.filament_cfg(LLm=40, MMm=24, N=12, np_xi=1, np_eta=1)
        c.adv_isoneutral = 1
        return c
    if kind == "basin_obc":   # open edges (LapT copies at the edges) and an island (masks)
        return iso_cfg(LLm=40, MMm=32, N=16, obc=15, island=1)
    return iso_cfg(LLm=40, MMm=32, N=16)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["basin", "basin_obc", "filament"])
def test_gpu_iso_steps_match_oracle(kind):
    """One whole step within 1e-12 (relative to each field's max, interior; the
    per-routine bound), then 20 steps within the north_star RMS bound,
    ADV_ISONEUTRAL on in both."""
    from test_gpu_parity import PROGNOSTIC, RMS_RUN, check_fields
    cfg = _gpu_case(kind)
    o = oracle.Oracle(cfg)
    o.init()
    m = _model(cfg)
    o.step(1)
    m.step(1)
    m.sync()
    e1 = check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, 1e-12)
    print("ISO %s one step, max relative error per field:" % kind, {k: "%.1e" % v for k, v in e1.items()})
    o.step(19)
    m.step(19)
    check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    m.close()


@pytest.mark.gpu
def test_gpu_iso_switch_changes_tracers():
    """The device run with the switch differs from the one without: the ISO
    path is live (the off path is the rest of the suite's)."""
    out = {}
    for iso in (0, 1):
        m = _model(iso_cfg(LLm=40, MMm=32, N=16, iso=iso))
        m.step(3)
        out[iso] = m.get("t")
        m.close()
    assert np.isfinite(out[1]).all()
    assert not np.array_equal(out[0], out[1])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,npx,npe", [("basin", 2, 2), ("filament", 2, 1)])
def test_gpu_iso_decomposition_bitwise(kind, npx, npe):
    """Subdomains equal the single domain bitwise: the slopes, idRz and
    diff3u/v reach the operator's i-2..i+2 stencil through the exchanges."""
    from test_gpu_multirank import check_decomposition
    if kind == "filament":
        case = dict(case_id=0, LLm=40, MMm=30, N=12, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
                    sizex=8.0e3, sizey=1.5e3, adv_isoneutral=True)
    else:
        case = dict(case_id=1, LLm=36, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                    sizex=108e3, sizey=84e3, lmd=oracle.LMD_ICELAND, surf_flux=True, adv_isoneutral=True)
    check_decomposition(case, npx, npe, nsteps=4)
