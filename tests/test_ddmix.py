"""LMD_DDMIX: double-diffusive additions to the tracer diffusivities
(lmd_vmix.F:95-101 constants, :279-360 salt fingering / diffusive
convection), restated in oracle/oracle_lmd.c (ddmix) and k_lmd.hip
(k_kpp_int<true>).

No reference case enables LMD_DDMIX, so there is no golden vector: the
oracle's restatement is checked here against the formula itself (a numpy
evaluation of Rrho and of the two branches on the same state) and the HIP
kernel against the oracle (parity unpinned to reference output, like every
switch no reference case sets).  The synthetic basin has no vertical salinity
gradient, so the state is re-stratified first: salt fingering (warm salty
over cool fresh, 1 < Rrho < 1.9) in the western half and diffusive
convection (cold fresh over warm salty, 0 < Rrho < 1) in the eastern half.
"""
import numpy as np
import pytest

import oracle

A = dict(A0=+0.665157E-01, A1=+0.170907E-01, A2=-0.203814E-03, A3=+0.298357E-05, A4=-0.255019E-07,
         B0=+0.378110E-02, B1=-0.846960E-04, C0=-0.678662E-05, D0=+0.380374E-04, D1=-0.933746E-06,
         D2=+0.791325E-08, E0=-0.164759E-06, F0=-0.251520E-11, G0=+0.512857E-12, H0=-0.302285E-13)


def ddmix_cfg(LLm=24, MMm=16, N=12, lmd=oracle.LMD_ICELAND | oracle.LMD_DDMIX):
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
    c.sizex, c.sizey = 2.0e3 * LLm, 2.0e3 * MMm
    return c


def restratify(o, cfg):
    """Both time levels of T and S: west half S = 35 + 0.15 (T - 4) (salt
    fingering), east half T' = 18 - T with S = 35 - 0.3 (T - 4) (diffusive
    convection), T the basin's own profile."""
    t = o.field("t")   # (NT*3*N, ny2, nx2): tracer, time level, k
    N = cfg.N
    nx2 = t.shape[2]
    west = np.arange(nx2) < nx2 // 2
    for lev in range(3):
        T = t[lev * N:(lev + 1) * N]
        S = t[3 * N + lev * N:3 * N + (lev + 1) * N]
        T0 = T.copy()
        S[...] = np.where(west, 35.0 + 0.15 * (T0 - 4.0), 35.0 - 0.3 * (T0 - 4.0))
        T[...] = np.where(west, T0, 18.0 - T0)


def rrho(o, cfg, tind):
    """Rrho and ddDS of lmd_vmix.F:288-307 at w-levels 1..N-1 (interior)."""
    N = cfg.N
    t = o.field("t")
    T, S = t[(tind - 1) * N:tind * N], t[3 * N + (tind - 1) * N:3 * N + tind * N]
    zw = o.field("z_w")
    Tt = 0.5 * (T[:-1] + T[1:])
    Ts = 0.5 * (S[:-1] + S[1:]) - 35.0
    Tp = -zw[1:N]
    a = A
    ab = (a["A0"] + Tt * (a["A1"] + Tt * (a["A2"] + Tt * (a["A3"] + Tt * a["A4"]))) + Ts * (a["B0"] + Tt * a["B1"] + Ts * a["C0"])
          + Tp * (a["D0"] + Tt * (a["D1"] + Tt * a["D2"]) + Ts * a["E0"] + Tp * (Ts * a["F0"] + Tt * Tt * a["G0"] + Tp * a["H0"])))
    dT = T[1:] - T[:-1]
    dS = S[1:] - S[:-1]
    dS = np.copysign(1.0, dS) * np.maximum(np.abs(dS), 1e-14)
    return ab * dT / dS, dS


def _mid_run(o, cfg):
    """Two steps, the re-stratification, then the predictor's indices
    (nrhs = nstp, nnew = 3) and rho_eos(nstp) as lmd_vmix(nstp) sees them."""
    o.step(2)
    restratify(o, cfg)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    o.set_tindex([iic, kstp, knew, nstp, nstp, 3])
    o.L.or_rho_eos(o.h, nstp)
    return iic, kstp, knew, nstp


def test_oracle_ddmix_branches_and_sensitivity():
    """CPU: on the re-stratified basin both LMD_DDMIX branches occur (numpy
    evaluation of Rrho), and lmd_vmix with LMD_DDMIX changes Akt(T) and
    raises Akt(S) where the branches add diffusivity, Akv unchanged."""
    out = {}
    for dd in (0, oracle.LMD_DDMIX):
        cfg = ddmix_cfg(lmd=oracle.LMD_ICELAND | dd)
        o = oracle.Oracle(cfg)
        o.init()
        _, _, _, nstp = _mid_run(o, cfg)
        if dd:
            R, dS = rrho(o, cfg, nstp)
            ny, nx = R.shape[1:]
            inner = (slice(None), slice(2, ny - 2), slice(2, nx - 2))
            fing = (R > 1.0) & (R < 1.9) & (dS > 0)
            conv = (R > 0.0) & (R < 1.0) & (dS < 0)
            assert fing[inner].sum() > 20 and conv[inner].sum() > 20, (fing[inner].sum(), conv[inner].sum())
        o.L.or_lmd_vmix(o.h, nstp)
        out[dd] = {n: o.field(n).copy() for n in ("Akv", "Akt")}
    N = ddmix_cfg().N
    assert np.array_equal(out[0]["Akv"], out[oracle.LMD_DDMIX]["Akv"])
    aks0, aks1 = out[0]["Akt"][N + 1:], out[oracle.LMD_DDMIX]["Akt"][N + 1:]
    assert (aks1 > aks0).sum() > 50
    assert not np.array_equal(out[0]["Akt"][:N + 1], out[oracle.LMD_DDMIX]["Akt"][:N + 1])


@pytest.mark.gpu
def test_gpu_ddmix_lmd_vmix_and_run():
    """GPU vs oracle on the re-stratified basin with LMD_DDMIX: one lmd_vmix
    within RTOL_ROUTINE (device exp may differ from glibc's by an ulp), then
    20 whole steps within the north_star RMS bound."""
    import romsgpu
    from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, check_fields, copy_state
    cfg = ddmix_cfg(LLm=40, MMm=32, N=16)

    def model():
        return romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True,
                                       nonlin_eos=True, dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex,
                                       sizey=cfg.sizey, lmd=cfg.lmd, surf_flux=True)
    o = oracle.Oracle(cfg)
    o.init()
    iic, kstp, knew, nstp = _mid_run(o, cfg)
    m = model()
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nstp, 3, nfast=o.nfast())
    o.L.or_lmd_vmix(o.h, nstp)
    m.lmd_vmix(nstp)
    m.sync()
    check_fields(o, m, ["Akv", "Akt", "ghat", "hbls", "hbbl"], cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    m.close()
    o = oracle.Oracle(cfg)
    o.init()
    restratify(o, cfg)
    m = model()
    copy_state(o, m)
    o.step(20)
    m.step(20)
    check_fields(o, m, PROGNOSTIC + ["Akt"], cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    m.close()
