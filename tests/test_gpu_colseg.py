"""GPU parity of the segment-partitioned column solvers (k_colseg.h), which
replace the sequential Thomas sweeps for deep grids (N > 63: the C3 workload;
forced on at N = 50 here): the predictor's tracer and momentum columns
(pre_step3d), the corrector's momentum columns (step3d_uv1) and the tracer
corrector (step3d_t).  Their elimination order differs from the reference's, so the
bound is the north_star floating-point tolerance rather than bit equality:
1e-12 relative per routine call, field RMS < 1e-10 over a run.

Cases: the closed basin with nonlinear EOS at N = 50 (C2 depth) and with
LMD/KPP + surface fluxes at N = 100 (C3 depth), on small horizontal grids so
the oracle finishes in seconds.  Each routine is also compared with the
library's own sequential path (ROMS_GPU_COLSEG=0) on the same state.
"""
import os

import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_parity import PROGNOSTIC, RMS_RUN, RTOL_ROUTINE, basin_cfg, check_fields, copy_state, interior, relerr

pytestmark = pytest.mark.gpu


def seg_cfg(case):
    if case == "n50":
        return basin_cfg(nonlin=True, LLm=40, MMm=24, N=50)
    c = basin_cfg(nonlin=True, LLm=24, MMm=20, N=100)
    c.lmd, c.surf_flux = oracle.LMD_ALL, 1
    return c


def make_model(cfg, colseg):
    old = os.environ.get("ROMS_GPU_COLSEG")
    os.environ["ROMS_GPU_COLSEG"] = str(colseg)
    try:
        return romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                       nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                       sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd,
                                       surf_flux=bool(cfg.surf_flux))
    finally:
        if old is None:
            del os.environ["ROMS_GPU_COLSEG"]
        else:
            os.environ["ROMS_GPU_COLSEG"] = old


# ru/rv after pre_step3d and step3d_uv1 are dead in the reference (the next
# read is preceded by prsgrd's assignment, prsgrd.F:293), so the segment
# solvers do not store them; their effect is checked through u, v, rufrc, rvfrc
ROUTINES = [("pre_step3d", "pred", ["t", "u", "v"]),
            ("step3d_uv1", "corr", ["u", "v", "rufrc", "rvfrc"]),
            ("step3d_t", "corr", ["t"])]


@pytest.mark.parametrize("case", ["n50", "n100"])
@pytest.mark.parametrize("routine,mode,outs", ROUTINES, ids=[r[0] for r in ROUTINES])
def test_seg_routine_parity(case, routine, mode, outs):
    cfg = seg_cfg(case)
    o = oracle.Oracle(cfg)
    o.init()
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    if mode == "corr":
        nrhs, nnew = 3, 3 - nstp
    else:
        nrhs, nnew = nstp, 3
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    # level-varying mixing and implicit vertical fluxes, so every per-level
    # input of the column solves is distinct (without LMD, Akv/Akt are the
    # constant background and Wi stays zero in these cases)
    rng = np.random.default_rng(11)
    for name in ("Akv", "Akt"):
        a = o.field(name)
        a[...] = a * (1.0 + 0.5 * rng.random(a.shape))
    we, wi = o.field("We"), o.field("Wi")
    wi[...] = wi + 0.01 * float(np.abs(we).max()) * rng.standard_normal(wi.shape)
    res = {}
    for colseg in (1, 0):
        m = make_model(cfg, colseg)
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, nfast=o.nfast())
        getattr(m, routine)()
        m.sync()
        res[colseg] = {n: interior(m.get(n), cfg.LLm, cfg.MMm) for n in outs}
        m.close()
    o.call(routine)
    for n in outs:
        ref = interior(o.field(n), cfg.LLm, cfg.MMm)
        assert relerr(res[0][n], ref) <= RTOL_ROUTINE, (n, "sequential")
        e = relerr(res[1][n], ref)
        assert e <= RTOL_ROUTINE, (n, e)
        assert e > 0.0 or np.array_equal(res[1][n], ref)


@pytest.mark.parametrize("case", ["n50", "n100"])
def test_seg_run_rms(case):
    cfg = seg_cfg(case)
    o = oracle.Oracle(cfg)
    o.init()
    m = make_model(cfg, 1)
    o.step(30)
    m.step(30)
    check_fields(o, m, PROGNOSTIC, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    m.close()


def _run_colreg(cfg, mask, nsteps):
    old = os.environ.get("ROMS_GPU_COLREG")
    os.environ["ROMS_GPU_COLREG"] = str(mask)
    try:
        m = make_model(cfg, 0)
    finally:
        if old is None:
            del os.environ["ROMS_GPU_COLREG"]
        else:
            os.environ["ROMS_GPU_COLREG"] = old
    m.step(nsteps)
    out = {n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "ru", "rv", "rufrc", "rvfrc", "FlxU", "We")}
    m.close()
    return out


@pytest.mark.parametrize("lmd", [0, oracle.LMD_ALL])
def test_register_column_kernels_bitwise(lmd):
    """N = 50 register-resident column solvers (k_uv1_reg, k_pre_tracer_v_reg:
    ROMS_GPU_COLREG bits 1, 2) keep the sequential LDS solvers' expressions
    and order: 12 steps equal the LDS forms bitwise."""
    cfg = seg_cfg("n50")
    cfg.lmd, cfg.surf_flux = lmd, int(lmd != 0)
    a = _run_colreg(cfg, 0, 12)
    b = _run_colreg(cfg, 3, 12)
    for n in a:
        assert np.array_equal(a[n], b[n]), n


@pytest.mark.parametrize("case", ["n50", "n100"])
@pytest.mark.parametrize("switch", ["ROMS_GPU_PREUV_LDS", "ROMS_GPU_OMEGA_SEG", "ROMS_GPU_UV1_LDS", "ROMS_GPU_OMEGA_HB"])
def test_seg_variants_bitwise(case, switch, monkeypatch):
    """Variants that keep the reference's operations and order, so 6 steps
    equal the plain forms bitwise:
    - k_pre_uv_seg<true> (ROMS_GPU_PREUV_LDS, default) forms the predictor's
      cf_stp*u(nstp) + cf_bak*u(indx) and u(indx) = Hz*u(nstp) in its spline
      phase and keeps them in LDS instead of reloading u and Hz later;
    - k_omega_seg (ROMS_GPU_OMEGA_SEG, default) reads each input once and runs
      the partial sums of the divergence as one chain through the waves;
    - k_uv1_seg<true> (ROMS_GPU_UV1_LDS, default) keeps the spline phase's Hz
      pairs in LDS for the viscosity rows and chains the rufrc sum through
      the waves in k order;
    - k_omega_seg<true> (ROMS_GPU_OMEGA_HB, default) forms pre_step3d's
      Hz_bak/Hz_fwd in the predictor's omega with k_pre_tracer_h1's
      expression, the tracer kernel loading them instead."""
    cfg = seg_cfg(case)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv(switch, env)
        m = make_model(cfg, 1)
        m.step(6)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


@pytest.mark.parametrize("lmd", [0, oracle.LMD_ALL])
def test_seg_buffer_forms_bitwise(lmd, monkeypatch):
    """Segment solvers with buffer loads (ROMS_GPU_SEG_BUF bits: 1
    k_pre_tracer_segb, 2 k_step3d_t_segb, 32 k_uv1_segb, 128 k_pre_uv_segb
    -- wave-uniform level offsets in SGPRs, the lane's column in one VGPR --,
    4 / 16 / 64 / 256 their diffusion rows' inputs prefetched with the spline inputs, 8
    step3d_t reloading Hz for its diffusion rows, 512 / 1024 the momentum /
    tracer forms with the level offsets in the VGPR offset) keep the
    expressions and
    their order: 6 steps at
    N = 100, with and without KPP, equal the pointer forms bitwise."""
    cfg = seg_cfg("n100")
    cfg.lmd, cfg.surf_flux = lmd, int(lmd != 0)
    out = []
    for env in ("0", "3", "23", "11", "32", "96", "128", "487", "551", "679", "743", "1031"):
        monkeypatch.setenv("ROMS_GPU_SEG_BUF", env)
        m = make_model(cfg, 1)
        m.step(6)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")})
        m.close()
    for o in out[1:]:
        for n in out[0]:
            assert np.array_equal(out[0][n], o[n]), n


@pytest.mark.parametrize("chunk", ["5", "16"])
def test_tracer_strip_chunks_bitwise(chunk, monkeypatch):
    """ROMS_GPU_TCHUNK: the tracer horizontal kernels and segment solvers of
    pre_step3d and step3d_t alternate over strips of rows (the first strip
    of the predictor also forms the ring j = jstr-1); 6 steps at N = 100 with
    KPP equal the whole-range launches bitwise."""
    cfg = seg_cfg("n100")
    cfg.lmd, cfg.surf_flux = oracle.LMD_ALL, 1
    out = []
    for env in ("0", chunk):
        monkeypatch.setenv("ROMS_GPU_TCHUNK", env)
        m = make_model(cfg, 1)
        m.step(6)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


def _omega_cfg(case):
    if case == "n50":
        return seg_cfg("n50")
    c = basin_cfg(nonlin=True, LLm=40, MMm=16, N=100)   # >= 32 columns wide: the segment form runs
    c.lmd, c.surf_flux = oracle.LMD_ALL, 1
    return c


@pytest.mark.parametrize("case", ["n50", "n100"])
def test_omega_blocks(case, monkeypatch):
    """k_omega_seg on 64-, 32- and 16-column blocks (ROMS_GPU_OMEGA_CW), with
    the k-order chain of partial sums (ROMS_GPU_OMEGA_PAR=0) and with each
    segment summing its own levels while the others do (PAR=1):
    - the chain keeps the reference's order: 6 whole steps (predictor omega
      with Hz_bak/Hz_fwd, corrector, closing omega) equal across block widths
      and block orders (ROMS_GPU_OMEGA_ORD) bitwise; so do the PAR forms
      among themselves (same segment partition);
    - PAR reassociates the sums: one omega call within RTOL_ROUTINE of the
      oracle, and 6 whole steps within RMS_RUN of the chain form."""
    cfg = _omega_cfg(case)
    names = ("zeta", "ubar", "vbar", "u", "v", "t", "We", "Wi", "rufrc", "rvfrc")
    runs = {}
    for par in ("0", "1"):
        for cw in ("64", "32", "16"):
            monkeypatch.setenv("ROMS_GPU_OMEGA_PAR", par)
            monkeypatch.setenv("ROMS_GPU_OMEGA_CW", cw)
            m = make_model(cfg, 1)
            m.step(6)
            runs[par, cw] = {n: m.get(n) for n in names}
            m.close()
    # the segment solvers' grouped block order (ROMS_GPU_OMEGA_ORD=3) only
    # changes which block runs which tile
    monkeypatch.setenv("ROMS_GPU_OMEGA_PAR", "0")
    monkeypatch.setenv("ROMS_GPU_OMEGA_CW", "16")
    monkeypatch.setenv("ROMS_GPU_OMEGA_ORD", "3")
    m = make_model(cfg, 1)
    m.step(6)
    runs["0", "16o3"] = {n: m.get(n) for n in names}
    m.close()
    monkeypatch.delenv("ROMS_GPU_OMEGA_ORD")
    for par, cw in (("0", "32"), ("0", "16"), ("0", "16o3"), ("1", "32"), ("1", "16")):
        for n in names:
            assert np.array_equal(runs[par, "64"][n], runs[par, cw][n]), (par, cw, n)
    for n in names:
        a, b = runs["0", "64"][n], runs["1", "64"][n]
        rms = float(np.sqrt(np.mean((a - b) ** 2)))
        # Wi is cancellation noise (~1e-13) where the Courant split leaves it
        # zero: measured against We's scale, as in test_gpu_bulk
        ref = runs["0", "64"]["We" if n == "Wi" else n]
        assert rms <= RMS_RUN * max(float(np.sqrt(np.mean(ref ** 2))), 1e-30), (n, rms)
    o = oracle.Oracle(cfg)
    o.init()
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    o.set_tindex([iic, kstp, knew, nstp, 3, 3 - nstp])
    for cw in ("64", "16"):
        monkeypatch.setenv("ROMS_GPU_OMEGA_PAR", "1")
        monkeypatch.setenv("ROMS_GPU_OMEGA_CW", cw)
        m = make_model(cfg, 1)
        copy_state(o, m)
        m.set_tindex(iic, kstp, knew, nstp, 3, 3 - nstp, nfast=o.nfast())
        m.omega()
        m.sync()
        res = {n: interior(m.get(n), cfg.LLm, cfg.MMm) for n in ("We", "Wi")}
        m.close()
        if cw == "64":
            o.call("omega")
        for n in ("We", "Wi"):
            ref = interior(o.field(n), cfg.LLm, cfg.MMm)
            scale = float(np.abs(interior(o.field("We"), cfg.LLm, cfg.MMm)).max())
            err = float(np.abs(res[n] - ref).max()) / scale
            assert err <= RTOL_ROUTINE, (cw, n, err)
