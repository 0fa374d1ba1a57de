"""GPU parity of the open lateral boundaries:
zetabc / u2dbc / v2dbc with OBC_M2FLATHER (tangential components through the
OBC_M2ORLANSKI branch, u2dbc_im.F:270-273), u3dbc / v3dbc with OBC_M3ORLANSKI,
t3dbc with OBC_TORLANSKI, all with *_FRC_BRY boundary data and the ubind
binding velocity; plus the SPONGE bands (set_nudgcof.F) and a land mask.

The case is the synthetic basin with all four edges open, an island and
analytic time-independent boundary data (Iceland switch set,
Examples/Iceland/Iceland_parent/cppdefs.opt; the real Iceland inputs are not
available offline).  The oracle's open-boundary restatement
(oracle/oracle_obc.c) has no golden log of its own -- the reference's OBC
tests need netCDF inputs fetched from GitHub -- so this parity is GPU vs
oracle only ("parity unpinned" for the OBC branches; the closed-wall branches
of the same routines stay pinned by the Filament / Pipes_ana goldens).
Tolerances as in test_gpu_parity: 1e-12 relative per routine (sqrt in
Flather's phase speed may differ by an ulp), field RMS < 1e-10 per run.
"""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, basin_cfg, check_fields, copy_state

pytestmark = pytest.mark.gpu

BRY = ["%s_%s" % (v, e) for v in ("zeta", "ubar", "vbar", "u", "v", "t") for e in ("west", "east", "south", "north")]


def obc_cfg(obc=15, sponge=1.0, island=1, lmd=0, curv=0, **kw):
    c = basin_cfg(nonlin=True, **kw)
    c.obc, c.ubind, c.v_sponge, c.island, c.lmd, c.curvgrid = obc, 0.1, sponge, island, lmd, curv
    return c


def make_pair(cfg):
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex,
                                sizey=cfg.sizey, lmd=cfg.lmd, obc=cfg.obc, v_sponge=cfg.v_sponge,
                                island=bool(cfg.island), curvgrid=bool(cfg.curvgrid))
    return o, m


def full(a, b):
    """Whole arrays incl. ghost rows (the boundary values are the point here)."""
    d = float(np.max(np.abs(a - b)))
    return d / max(float(np.max(np.abs(b))), 1e-300)


def test_init_boundary_data_sponge_and_masks_match_oracle():
    cfg = obc_cfg()
    o, m = make_pair(cfg)
    bad = [(n, full(m.get(n), o.field(n))) for n in BRY + ["visc2_r", "visc2_p", "diff2", "rmask", "umask", "vmask",
                                                          "pmask"]]
    bad = [x for x in bad if not x[1] == 0.0]
    assert not bad, bad
    assert float(np.max(o.field("visc2_r"))) > 0.9 and float(np.min(o.field("rmask"))) == 0.0
    m.close()


@pytest.mark.parametrize("routine", ["step2d", "pre_step3d", "step3d_uv2", "step3d_t"])
@pytest.mark.parametrize("obc", [15, 5, 10])
def test_open_boundary_routine_parity(routine, obc):
    """One routine on identical mid-run states, ghost rows included.  obc=5:
    west+south open (east/north closed, so closed-open corners), 10: east+north."""
    cfg = obc_cfg(obc=obc)
    o, m = make_pair(cfg)
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    if routine == "step2d":
        kstp, knew = knew, knew % 4 + 1
        nrhs, nnew = 3, 3 - nstp
        o.L.or_set_iif(o.h, 2)
    elif routine == "pre_step3d":
        nrhs, nnew = nstp, 3
    else:
        nrhs, nnew = 3, 3 - nstp
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=2, nfast=o.nfast())
    o.call(routine)
    getattr(m, routine)()
    m.sync()
    outs = {"step2d": ["zeta", "ubar", "vbar", "DU_avg1", "DV_avg1", "Zt_avg1"],
            "pre_step3d": ["u", "v", "t"], "step3d_uv2": ["u", "v", "ubar", "vbar", "FlxU", "FlxV"],
            "step3d_t": ["t"]}[routine]
    bad = [(n, full(m.get(n), o.field(n))) for n in outs]
    bad = [x for x in bad if not x[1] <= RTOL_ROUTINE]
    assert not bad, (routine, obc, bad)
    m.close()


@pytest.mark.parametrize("routine", ["pre_step3d", "step3d_uv1"])
def test_curvgrid_momentum_rhs_parity(routine):
    """CURVGRID curvature terms in the momentum r.h.s. (compute_horiz_rhs_uv_terms.h:4-12)
    on non-uniform metrics; ru/rv carry them into u,v(nnew)."""
    cfg = obc_cfg(curv=1)
    o, m = make_pair(cfg)
    assert float(np.max(np.abs(o.field("dndx")))) > 0.0 and float(np.max(np.abs(o.field("dmde")))) > 0.0
    bad = [(n, full(m.get(n), o.field(n))) for n in ("dndx", "dmde", "pm", "pn")]
    assert all(e == 0.0 for _, e in bad), bad
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    if routine == "pre_step3d":
        nrhs, nnew = nstp, 3
        o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, nfast=o.nfast())
        o.call("prsgrd"); m.prsgrd()
    else:
        nrhs, nnew = 3, 3 - nstp
        o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, nfast=o.nfast())
        o.call("prsgrd"); m.prsgrd()
    o.call(routine)
    getattr(m, routine)()
    m.sync()
    check_fields(o, m, ["u", "v", "rufrc", "rvfrc"] if routine == "step3d_uv1" else ["u", "v", "t"], cfg.LLm,
                 cfg.MMm, RTOL_ROUTINE)
    m.close()


@pytest.mark.parametrize("lmd,curv", [(0, 0), (oracle.LMD_ALL, 0), (oracle.LMD_ICELAND, 1)])
def test_open_basin_30_steps_rms(lmd, curv):
    """(1, 1) is the Iceland switch set: OBC + SPONGE + MASKING + CURVGRID + LMD/KPP + NONLIN/SPLIT EOS."""
    cfg = obc_cfg(lmd=lmd, curv=curv)
    o, m = make_pair(cfg)
    o.step(30)
    m.step(30)
    check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    # the open edges carried flow: the western ghost column moved off its initial state
    ub = o.field("ubar")
    assert float(np.max(np.abs(ub[:, 2:-2, 2]))) > 1e-4
    for n in ("zeta", "ubar", "vbar", "u", "v", "t"):   # ghost rows too
        a, b = m.get(n), o.field(n)
        assert float(np.sqrt(np.mean((a - b) ** 2))) / max(1.0, float(np.sqrt(np.mean(b ** 2)))) < RMS_RUN, n
    m.close()


@pytest.mark.parametrize("npx,npe", [(2, 1), (1, 2), (2, 2), (3, 2)])
def test_open_basin_decomposition_bitwise(npx, npe):
    """Open edges + island on a processor grid equal the single domain bitwise
    (no sponge: the reference sets its bands on each rank's own points only)."""
    from test_gpu_multirank import test_decomposition_bitwise_equals_single_domain as run
    run("basin_obc", npx, npe)


def _ub_arrays(cfg, scale):
    """Per-edge binding coefficients spanning below 0, (0,1) and above the cap 1."""
    nj, ni = cfg.MMm + 2, cfg.LLm + 2
    x = lambda n, ph: scale * (0.5 + 1.5 * np.sin(np.arange(n) * 0.37 + ph))
    return [x(nj, 0.0), x(nj, 1.0), x(ni, 2.0), x(ni, 3.0)]


@pytest.mark.parametrize("obc", [15, 5])
def test_sponge_tune_t3dbc_parity(obc):
    """SPONGE_TUNE with ub_tune (t3dbc_im.F:73-74): the radiation blend's rate
    is floored by min(ub(j), 1); step3d_t on identical states, then 20 steps."""
    cfg = obc_cfg(obc=obc, lmd=oracle.LMD_ICELAND)
    o, m = make_pair(cfg)
    ub = _ub_arrays(cfg, 1.0)
    o.set_ub(ub)
    m.set_ub_tune(ub)
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    nrhs, nnew = 3, 3 - nstp
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=2, nfast=o.nfast())
    o.call("step3d_t")
    m.step3d_t()
    m.sync()
    assert full(m.get("t"), o.field("t")) <= RTOL_ROUTINE
    m.close()
    o2, m2 = make_pair(cfg)
    o2.set_ub(ub)
    m2.set_ub_tune(ub)
    o2.step(20)
    m2.step(20)
    a, b = m2.get("t"), o2.field("t")
    assert float(np.sqrt(np.mean((a - b) ** 2))) / max(1.0, float(np.sqrt(np.mean(b ** 2)))) < RMS_RUN
    m2.close()


def test_sponge_tune_limits():
    """ub <= 0 leaves the Orlanski rate unchanged (bitwise equal to ub_tune
    off); ub >= 1 pins the boundary tracers to the boundary data."""
    cfg = obc_cfg(obc=15)
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, obc=15,
                                v_sponge=cfg.v_sponge, island=True)
    m.step(8)
    off = m.get("t")
    m.close()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, obc=15,
                                v_sponge=cfg.v_sponge, island=True)
    m.set_ub_tune([-np.ones(cfg.MMm + 2), np.zeros(cfg.MMm + 2), -np.ones(cfg.LLm + 2), np.zeros(cfg.LLm + 2)])
    m.step(8)
    assert np.array_equal(m.get("t"), off)
    m.set_ub_tune([5 * np.ones(cfg.MMm + 2)] * 2 + [5 * np.ones(cfg.LLm + 2)] * 2)
    m.step(1)
    t = m.get("t").reshape(cfg.NT, 3, cfg.N, cfg.MMm + 4, cfg.LLm + 4)[:, m.t.nnew - 1]
    tw = m.get("t_west").reshape(cfg.NT, cfg.N, cfg.MMm + 2)
    rm = m.get("rmask")[0]
    j = np.arange(1, cfg.MMm + 1)
    assert np.array_equal(t[:, :, j + 1, 1], tw[:, :, j] * rm[j + 1, 1])   # western ghost column i = 0
    m.close()


@pytest.mark.parametrize("routine", ["pre_step3d", "step3d_uv2"])
def test_sponge_tune_uv3dbc_parity_and_sensitivity(routine):
    """SPONGE_TUNE on the 3-D momentum edges (u3dbc_im.F:101-103,190-192,
    262-264,341-343; v3dbc_im.F:97-99,189-191,264-266,344-346): the Orlanski
    blend's rate is floored by min(ub, 1) on all four sides, normal and
    tangential.  Both routines that call u3dbc/v3dbc on identical states,
    ghost rows included, against the oracle; and the edge values move when
    ub is switched on (this failed before the floor was restated)."""
    cfg = obc_cfg(obc=15, lmd=oracle.LMD_ICELAND)
    ub = _ub_arrays(cfg, 1.0)
    res = {}
    for tuned in (False, True):
        o, m = make_pair(cfg)
        if tuned:
            o.set_ub(ub)
            m.set_ub_tune(ub)
        o.step(3)
        iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
        nrhs, nnew = (nstp, 3) if routine == "pre_step3d" else (3, 3 - nstp)
        o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, iif=2, nfast=o.nfast())
        o.call(routine)
        getattr(m, routine)()
        m.sync()
        bad = [(n, full(m.get(n), o.field(n))) for n in ("u", "v")]
        bad = [x for x in bad if not x[1] <= RTOL_ROUTINE]
        assert not bad, (routine, tuned, bad)
        res[tuned] = (m.get("u").copy(), m.get("v").copy())
        m.close()
    L, M = cfg.LLm, cfg.MMm
    u0, u1 = res[False][0], res[True][0]
    v0, v1 = res[False][1], res[True][1]
    # western u column (i = 1 -> index 2) and southern v row (j = 1 -> index 2)
    assert not np.array_equal(u0[..., 3:M + 1, 2], u1[..., 3:M + 1, 2])
    assert not np.array_equal(v0[..., 2, 3:L + 1], v1[..., 2, 3:L + 1])
    # tangential: southern u ghost row (j = 0) and western v ghost column (i = 0)
    assert not np.array_equal(u0[..., 1, 3:L + 1], u1[..., 1, 3:L + 1])
    assert not np.array_equal(v0[..., 3:M + 1, 1], v1[..., 3:M + 1, 1])


def test_sponge_tune_uv_20_steps_rms():
    """ub_tune on, 20 steps of the Iceland switch set: u, v, t against the oracle."""
    cfg = obc_cfg(obc=15, lmd=oracle.LMD_ICELAND)
    ub = _ub_arrays(cfg, 1.0)
    o, m = make_pair(cfg)
    o.set_ub(ub)
    m.set_ub_tune(ub)
    o.step(20)
    m.step(20)
    for n in ("zeta", "ubar", "vbar", "u", "v", "t"):
        a, b = m.get(n), o.field(n)
        assert float(np.sqrt(np.mean((a - b) ** 2))) / max(1.0, float(np.sqrt(np.mean(b ** 2)))) < RMS_RUN, n
    m.close()
