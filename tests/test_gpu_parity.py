"""GPU parity: the HIP path (libromsgpu.so through the C ABI) against the CPU
oracle (oracle/, pinned bit-exactly to the reference golden log).

Tolerances: FP64 throughout; kernels are built with -ffp-contract=off and
keep the reference's operation order, so most routines agree to the last bit.
The few transcendental calls (log in the bottom drag, sqrt) may differ by an
ulp between ROCm's device libm and glibc, hence a per-routine relative bound
of 1e-12 and the north_star bound for whole runs: field RMS error < 1e-10.
"""
import os

import numpy as np
import pytest

import oracle
import romsgpu

pytestmark = pytest.mark.gpu

RTOL_ROUTINE = 1e-12
RMS_RUN = 1e-10


def basin_cfg(LLm=48, MMm=40, N=12, NT=2, nonlin=False, dt=60.0, ndtfast=30, sizex=96e3, sizey=80e3):
    c = oracle.OrCfg()
    c.LLm, c.MMm, c.N, c.NT = LLm, MMm, N, NT
    c.ew_periodic = c.ns_periodic = 0
    c.salinity, c.nonlin_eos, c.lmd = 1, int(nonlin), 0
    c.case_id = oracle.CASE_BASIN
    c.dt, c.ndtfast = dt, ndtfast
    c.theta_s, c.theta_b, c.hc, c.rho0 = 6.0, 2.0, 250.0, 1027.5
    c.rdrg, c.rdrg2, c.Zob = 0.0, 1.0e-3, 1.0e-2
    c.Akv_bak = 1.0e-4
    c.Akt_bak[0] = c.Akt_bak[1] = 1.0e-5
    c.Tcoef, c.T0, c.Scoef, c.S0 = 0.20, 1.0, 0.822, 1.0
    c.sizex, c.sizey = sizex, sizey
    c.diag_np_xi = c.diag_np_eta = 1
    return c


def make_pair(cfg):
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                sizex=cfg.sizex, sizey=cfg.sizey)
    return o, m


def interior(a, Lm, Mm):
    return a[..., 2:Mm + 2, 2:Lm + 2]


def relerr(a, b):
    d = np.max(np.abs(a - b))
    s = max(np.max(np.abs(b)), 1e-300)
    return d / s


def rms(a, b):
    """Field RMS error, in the field's units for O(1) fields (zeta, u, t ...)
    and relative to the field's own RMS when that exceeds 1 (FlxU, FlxV, We,
    Wi in m^3/s, depths and layer thicknesses in m)."""
    scale = max(1.0, float(np.sqrt(np.mean(b ** 2))))
    return float(np.sqrt(np.mean((a - b) ** 2))) / scale


def rms_abs(a, b):
    """Field RMS error in the field's own units (north_star: u, v, w, T, S, zeta)."""
    return float(np.sqrt(np.mean((a - b) ** 2)))


# north_star's prognostic fields: their whole-run bound is absolute (T in
# deg C and S in PSU are O(10), so a bound relative to their RMS would be
# ~35x looser); w = pm*pn*(We + Wi) in m/s is formed from the fluxes
ABSOLUTE = ("zeta", "ubar", "vbar", "u", "v", "t", "w")


def copy_state(o, m):
    for name in romsgpu.FIELDS:
        m.put(name, o.field(name))


PROGNOSTIC = ["zeta", "ubar", "vbar", "u", "v", "t", "Hz", "z_r", "z_w", "FlxU", "FlxV", "We", "Wi"]


def _w(src, get):
    """pm*pn*(We+Wi) at w points (basic_output.F's history omega)."""
    pmpn = get("pm") * get("pn")
    return (get("We") + get("Wi")) * pmpn


def check_fields(o, m, names, Lm, Mm, tol, kind="rel"):
    """Interior (1..Lm, 1..Mm) error of every named field, relative to the
    field's max for kind 'rel' (per-routine checks), RMS for kind 'rms' (whole
    runs: absolute for ABSOLUTE, scaled for the rest; a run that checks We
    and Wi also checks w absolutely).  Returns {name: error}."""
    names = list(names)
    if kind == "rms" and "We" in names and "Wi" in names and "w" not in names:
        names.append("w")
    bad, errs = [], {}
    for n in names:
        if n == "w":
            a, b = interior(_w(m, m.get), Lm, Mm), interior(_w(o, o.field), Lm, Mm)
        else:
            a, b = interior(m.get(n), Lm, Mm), interior(o.field(n), Lm, Mm)
        if kind == "rel":
            e = relerr(a, b)
        else:
            e = rms_abs(a, b) if n in ABSOLUTE else rms(a, b)
        errs[n] = e
        if not (e <= tol):
            bad.append((n, e))
    assert not bad, bad
    return errs


def test_filament_init_matches_oracle():
    cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    o, m = make_pair(cfg)
    check_fields(o, m, PROGNOSTIC + ["rho", "rhoA", "rhoS", "DU_avg1", "DV_avg1"], 32, 24, RTOL_ROUTINE)
    m.close()


ROUTINE_CASES = [
    # (name, tindex mutation, outputs)
    ("rho_eos", None, ["rho", "rhoA", "rhoS"]),
    ("set_HUV", None, ["FlxU", "FlxV", "Hz_u", "Hz_v"]),
    ("omega", None, ["We", "Wi"]),
    ("prsgrd", None, ["ru", "rv"]),
    ("pre_step3d", None, ["t", "u", "v", "r_D"]),
    ("set_HUV1", None, ["u", "v", "FlxU", "FlxV"]),
    ("step3d_uv1", "corr", ["u", "v", "rufrc", "rvfrc"]),
    ("visc3d", "corr", ["u", "v", "rufrc", "rvfrc"]),
    ("step3d_uv2", "corr", ["u", "v", "ubar", "vbar", "FlxU", "FlxV"]),
    ("step3d_t", "corr", ["t"]),
    ("t3dmix", "corr", ["t"]),
    ("set_depth", None, ["z_w", "z_r", "Hz"]),
]


@pytest.mark.parametrize("case", ["filament", "basin", "basin_nonlin"])
@pytest.mark.parametrize("routine,mode,outs", ROUTINE_CASES, ids=[r[0] for r in ROUTINE_CASES])
def test_routine_parity(case, routine, mode, outs):
    if case == "filament":
        cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    else:
        cfg = basin_cfg(nonlin=(case == "basin_nonlin"))
    o, m = make_pair(cfg)
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    if mode == "corr":
        nrhs, nnew = 3, 3 - nstp
    else:
        nrhs, nnew = nstp, 3
    o.set_tindex([iic, kstp, knew, nstp, nrhs, nnew])
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nrhs, nnew, nfast=o.nfast())
    if routine == "rho_eos":
        o.call("rho_eos", nrhs)
        m.rho_eos(nrhs)
        if cfg.nonlin_eos:
            outs = ["rho1", "qp1", "rhoA", "rhoS"]
    else:
        o.call(routine)
        getattr(m, routine)()
    m.sync()
    check_fields(o, m, outs, cfg.LLm, cfg.MMm, RTOL_ROUTINE)
    m.close()


@pytest.mark.parametrize("case", ["filament", "basin", "basin_nonlin"])
def test_prsgrd_fused_variant_parity(case, monkeypatch):
    """The opt-in one-kernel prsgrd (ROMS_GPU_PRSGRD_FUSED=1) is bit-identical."""
    monkeypatch.setenv("ROMS_GPU_PRSGRD_FUSED", "1")
    test_routine_parity(case, "prsgrd", None, ["ru", "rv"])


def test_step2d_fast_loop_parity():
    cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    o, m = make_pair(cfg)
    o.step(2)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    copy_state(o, m)
    for iif in (1, 2, 3, 4):
        kstp, knew = knew, knew % 4 + 1
        o.set_tindex([iic, kstp, knew, nstp, 3, 3 - nstp])
        o.L.or_set_iif(o.h, iif)
        o.call("step2d")
        m.set_tindex(iic, kstp, knew, nstp, 3, 3 - nstp, iif=iif, nfast=o.nfast())
        m.step2d()
    check_fields(o, m, ["zeta", "ubar", "vbar", "Zt_avg1", "DU_avg1", "DV_avg1", "DU_avg2", "DV_avg2", "rufrc"],
                 32, 24, RTOL_ROUTINE)
    m.close()


def test_filament_20_steps_golden_and_fields():
    """Reference Filament case (64x64x32, 20 steps) on the GPU: diag norms vs
    the golden log within reduction-order noise, fields vs the oracle."""
    import json
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "filament_github_gnu.json")))["rows"]
    cfg = oracle.filament_cfg()
    o, m = make_pair(cfg)
    for s in range(1, 21):
        o.step()
        m.step()
        g = m.diag()
        r = gold[s]
        for key, val in zip(("ke", "ke2b", "cu_adv"), g[:3]):
            ref = float(r[key])
            assert abs(val - ref) <= 1e-11 * abs(ref), (s, key, val, ref)
    check_fields(o, m, PROGNOSTIC, 64, 64, RMS_RUN, kind="rms")
    m.close()


def test_basin_nonlin_100_steps_rms():
    """Closed synthetic basin, nonlinear split EOS, T+S: 100 steps, field RMS
    against the oracle below the north_star bound."""
    cfg = basin_cfg(LLm=40, MMm=32, N=10, nonlin=True)
    o, m = make_pair(cfg)
    o.step(100)
    m.step(100)
    m.sync()
    assert o.tindex() == m.t.as_list()
    check_fields(o, m, PROGNOSTIC, 40, 32, RMS_RUN, kind="rms")
    m.close()


def test_graph_replay_bitwise_equals_eager():
    cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    m1 = romsgpu.Model.from_case(0, 32, 24, 16, sizex=cfg.sizex, sizey=cfg.sizey)
    m1.step(6)
    a = {n: m1.get(n) for n in ("zeta", "u", "v", "t")}
    m1.close()
    os.environ["ROMS_GPU_NO_GRAPH"] = "1"
    try:
        m2 = romsgpu.Model.from_case(0, 32, 24, 16, sizex=cfg.sizex, sizey=cfg.sizey)
        m2.step(6)
        for n, v in a.items():
            assert np.array_equal(m2.get(n), v), n
        m2.close()
    finally:
        os.environ.pop("ROMS_GPU_NO_GRAPH", None)


@pytest.mark.parametrize("graphs", [True, False])
def test_rho_eos_reuse_bitwise_and_invalidated(graphs, monkeypatch):
    """A step opens with rho_eos(nrhs) (main.F:397) on the t, z_r, Hz the
    previous step's closing rho_eos(nnew) (main.F:479) already used; the
    library skips the repeat (roms_shim.cpp g.rho_slot).  With the skip on
    and off the runs are bitwise equal, including after the host changes the
    state between steps through each entry that can: copy_in of
    t, a registered mirror's upload of t, copy_in of z_r, new pipe sources
    (set_pipe_frc) and a host-side forcing interpolation (frc_record +
    frc_interp of stflx) -- each must invalidate the reuse."""
    if not graphs:
        monkeypatch.setenv("ROMS_GPU_NO_GRAPH", "1")
    cfg = oracle.pipes_cfg(LLm=40, MMm=40, np_xi=1, np_eta=1)

    def edit(m, how):
        if how == "copy_in_t":
            t = m.get("t")
            t[:, 15:25, 15:25] += 0.75     # every level and slot of T (and S) in a patch
            m.put("t", t)
        elif how == "upload_t":
            t = np.ascontiguousarray(m.get("t")).ravel().copy()
            m.register("t", t)
            t.reshape(m.get("t").shape)[:, 10:20, 20:30] -= 0.5
            m.upload("t")
        elif how == "copy_in_zr":
            z = m.get("z_r")
            z[:, 12:18, 12:18] *= 1.001
            m.put("z_r", z)
        elif how == "pipe":
            idx = np.zeros(m.shape2, dtype=np.int32)
            flx = np.zeros(m.shape2)
            idx[20, 20] = 1
            flx[20, 20] = 1.0
            m.set_pipe_frc(idx, flx, np.full((1, cfg.N), 1.0 / cfg.N), np.array([[5.0, 1.0]]))
        elif how == "frc_interp":
            st = m.get("stflx")
            m.frc_record("stflx", 0, 0.0, st)
            m.frc_record("stflx", 1, 1.0, st + 1e-5)
            m.frc_interp(0.5, m.FRC_SURFACE)

    def run(reuse, how):
        monkeypatch.setenv("ROMS_GPU_RHO_REUSE", "1" if reuse else "0")
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                    dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd)
        m.step(3)
        m.diag()
        edit(m, how)
        m.step(3)
        out = {n: m.get(n) for n in ("rho1", "qp1", "bvf", "t", "u", "v", "zeta", "Akv", "Akt")}
        m.close()
        return out

    for how in ("copy_in_t", "upload_t", "copy_in_zr", "pipe", "frc_interp"):
        a, b = run(True, how), run(False, how)
        for n in a:
            assert np.array_equal(a[n], b[n]), (how, n)


def test_s2d_edges_folded_bitwise(monkeypatch):
    """The closed-wall edge phases of the fast step run inside k_s2d_fb
    (default) or as the separate k_s2d_edges launches (ROMS_GPU_S2D_EDGES=1,
    u2dbc/v2dbc and the boundary flux averages of step2d_FB.F:444-529): the
    runs are bitwise equal, on a grid whose last tile row / column holds more
    than the edge cell (folded) and on one where the host must fall back."""
    for LLm, MMm in ((40, 26), (63, 27)):
        cfg = basin_cfg(LLm=LLm, MMm=MMm, N=12, nonlin=True)
        out = []
        for env in ("1", "0"):
            monkeypatch.setenv("ROMS_GPU_S2D_EDGES", env)
            m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                        nonlin_eos=True, dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex,
                                        sizey=cfg.sizey)
            m.step(4)
            out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "DU_avg1", "DV_avg1")})
            m.close()
        for n in out[0]:
            assert np.array_equal(out[0][n], out[1][n]), (LLm, MMm, n)


@pytest.mark.parametrize("case", ["basin_fold", "basin_edges", "basin_nofold", "filament", "mask_edit"])
def test_s2d_window_bitwise(case, monkeypatch):
    """k_s2d_fb addresses its 25 2-D fields through one buffer window (one
    descriptor, a 32-bit offset per field; roms_gpu_s2d_window) or through
    their pointers (ROMS_GPU_S2D_WIN=0): the same loads and stores, bitwise
    equal runs -- closed walls folded in, the separate edge launches
    (ROMS_GPU_S2D_EDGES=1, with the zeta_new/Dnew scratch stores), a grid the
    host cannot fold, and the periodic Filament with its halo images
    (step2d_FB.F:77-570); mask_edit writes land cells and non-binary mask
    values between steps, which both forms must apply identically."""
    if case == "filament":
        cfg = oracle.filament_cfg(LLm=48, MMm=32, N=16, np_xi=1, np_eta=1)
    else:
        cfg = basin_cfg(LLm=63 if case == "basin_nofold" else 40, MMm=27 if case == "basin_nofold" else 26, N=12,
                        nonlin=True)
    monkeypatch.setenv("ROMS_GPU_S2D_EDGES", "1" if case == "basin_edges" else "0")
    out = []
    for env in ("1", "0"):
        monkeypatch.setenv("ROMS_GPU_S2D_WIN", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey)
        assert m.s2d_window() == (env == "1")
        m.step(4)
        if case == "mask_edit":
            rm, um, vm = m.get("rmask"), m.get("umask"), m.get("vmask")
            rm[0, 10:14, 12:15] = 0.0
            um[0, 10:14, 12:16] = 0.0
            vm[0, 10:15, 12:15] = 0.0
            rm[0, 20, 30] = 0.5
            um[0, 21, 31] = 0.75
            vm[0, 22, 32] = 0.25
            m.put("rmask", rm)
            m.put("umask", um)
            m.put("vmask", vm)
            m.step(3)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "DU_avg1", "DV_avg1", "Zt_avg1",
                                          "DU_avg2", "rufrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), (case, n)


@pytest.mark.parametrize("case", ["basin", "filament"])
def test_prsgrd_uv_fused_bitwise(case, monkeypatch):
    """Whole steps run the horizontal momentum r.h.s. of pre_step3d /
    step3d_uv1 inside the prsgrd kernel before them (compute_horiz_rhs_uv_terms.h
    on the same u, v, FlxU, FlxV, Hz; ru/rv stored once); ROMS_GPU_PRS_UV=0
    keeps the two kernels.  Bitwise equal."""
    if case == "basin":
        cfg = basin_cfg(LLm=40, MMm=26, N=12, nonlin=True)
    else:
        cfg = oracle.filament_cfg(LLm=48, MMm=32, N=16, np_xi=1, np_eta=1)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("ROMS_GPU_PRS_UV", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey)
        m.step(4)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "ru", "rv", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


def test_diag_blowup_flag_is_fatal():
    """A non-finite norm is diag.F's 'Abnormal termination: BLOWUP'
    (diag.F:621-633): roms_gpu_diag fails instead of printing NaN."""
    cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    m = romsgpu.Model.from_case(0, 32, 24, 16, sizex=cfg.sizex, sizey=cfg.sizey)
    m.step(2)
    assert all(np.isfinite(m.diag()))
    u = m.get("u")
    u[:, 10, 10] = np.nan
    m.put("u", u)
    with pytest.raises(romsgpu.RomsGpuError, match="BLOWUP"):
        m.diag()
    m.close()


def _routine_fields(cfg, routine, outs, env, monkeypatch):
    """One routine from the oracle's state after 3 steps (corrector indices),
    with the library initialised under `env`; returns the GPU outputs."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    o, m = make_pair(cfg)
    o.step(3)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, 3, 3 - nstp, nfast=o.nfast())
    getattr(m, routine)()
    m.sync()
    res = {n: m.get(n).copy() for n in outs}
    m.close()
    return res


@pytest.mark.parametrize("case", ["filament", "basin", "basin_n100"])
def test_uv2_fused_bitwise_equals_two_kernels(case, monkeypatch):
    """k_uv2_fused (one pass, segment-chained sums in the reference's k order)
    gives exactly the bits of k_uv2_couple + u3dbc/v3dbc + k_uv2_flux, on a
    periodic domain, a closed basin (edge columns through the split path)
    and a 100-level basin (25 levels per lane)."""
    if case == "filament":
        cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    elif case == "basin":
        cfg = basin_cfg(nonlin=True)
    else:
        cfg = basin_cfg(LLm=40, MMm=36, N=100, nonlin=True)
    outs = ["u", "v", "ubar", "vbar", "FlxU", "FlxV"]
    a = _routine_fields(cfg, "step3d_uv2", outs, {"ROMS_GPU_UV2_FUSED": "1"}, monkeypatch)
    b = _routine_fields(cfg, "step3d_uv2", outs, {"ROMS_GPU_UV2_FUSED": "0"}, monkeypatch)
    for n in outs:
        assert np.array_equal(a[n], b[n]), n


@pytest.mark.parametrize("case", ["filament", "basin", "basin_n100", "basin_n90"])
@pytest.mark.parametrize("routine,outs", [("set_HUV1", ["u", "v", "FlxU", "FlxV"])])
def test_chain_kernels_bitwise_equal_column_sweeps(case, routine, outs, monkeypatch):
    """The chained 4-lane column kernel (k_chain.h: set_HUV1; buffer-addressed,
    with N = 100 the full-segment form and N = 90 the guarded one of KL = 25)
    gives exactly the bits of the one-lane-per-column sweeps (ROMS_GPU_CHAIN=0)."""
    if case == "filament":
        cfg = oracle.filament_cfg(LLm=32, MMm=24, N=16, np_xi=1, np_eta=1)
    elif case == "basin":
        cfg = basin_cfg(nonlin=True)
    else:
        cfg = basin_cfg(LLm=40, MMm=36, N=int(case[7:]), nonlin=True)
    a = _routine_fields(cfg, routine, outs, {"ROMS_GPU_CHAIN": "1"}, monkeypatch)
    b = _routine_fields(cfg, routine, outs, {"ROMS_GPU_CHAIN": "0"}, monkeypatch)
    for n in outs:
        assert np.array_equal(a[n], b[n]), n


@pytest.mark.parametrize("grp", ["1", "2"])
def test_tile_group_order_bitwise(grp, monkeypatch):
    """ROMS_GPU_TILE_GRP re-orders the tiles of the hoisted per-level kernels
    (h_tile: y fastest inside groups of grp x-tiles, a narrower last group);
    every tile is still computed once: 4 steps equal the plain order bitwise.
    152 x 40 columns give 3 x-tiles (one full group of 2 and a remainder)."""
    cfg = basin_cfg(LLm=150, MMm=40, N=8, nonlin=True, sizex=300e3)
    out = []
    for env in ("0", grp):
        monkeypatch.setenv("ROMS_GPU_TILE_GRP", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey)
        m.step(4)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


def test_hz_uv_stored_on_request(monkeypatch):
    """Hz_u/Hz_v (set_depth.F:220,227) feed only extract_data.F; whole steps
    skip their stores unless asked (ROMS_GPU_HZ_UV=1 or a registered host
    mirror).  Asked: after 3 steps they equal the oracle's set_HUV values.
    Not asked: reading them fails loudly instead of returning stale data, and
    the prognostic state is bitwise the same either way."""
    cfg = basin_cfg(LLm=40, MMm=32, N=10, nonlin=True)
    out = {}
    for env in ("1", "0"):
        monkeypatch.setenv("ROMS_GPU_HZ_UV", env)
        o, m = make_pair(cfg)
        o.step(3)
        m.step(3)
        out[env] = {n: m.get(n) for n in ("zeta", "u", "v", "t", "FlxU", "FlxV")}
        if env == "1":
            check_fields(o, m, ["Hz_u", "Hz_v"], cfg.LLm, cfg.MMm, RTOL_ROUTINE)
        else:
            with pytest.raises(romsgpu.RomsGpuError, match="Hz_u/Hz_v"):
                m.get("Hz_u")
            m.set_HUV()   # the routine itself always stores them
            m.sync()
            assert np.isfinite(m.get("Hz_v")).all()
        m.close()
    for n in out["0"]:
        assert np.array_equal(out["0"][n], out["1"][n]), n


@pytest.mark.parametrize("case", ["filament", "basin"])
@pytest.mark.parametrize("switch", ["ROMS_GPU_OMEGA_HB", "ROMS_GPU_P_IN_RHO", "ROMS_GPU_PRS_BUF"])
def test_step_producer_variants_bitwise(case, switch, monkeypatch):
    """Producers that form a later routine's inputs with its expressions: 4
    whole steps bitwise equal to the consumer forming them (=0), periodic
    (Filament, linear EOS) and closed (basin, split EOS):
    - ROMS_GPU_OMEGA_HB: the predictor's omega forms pre_step3d's
      Hz_bak/Hz_fwd of the interior cells;
    - ROMS_GPU_P_IN_RHO: every rho_eos also forms prsgrd's P in its sweep,
      so whole steps skip k_prsgrd_P;
    - ROMS_GPU_PRS_BUF: k_prsgrd_uv's windows through buffer loads."""
    if case == "basin":
        cfg = basin_cfg(LLm=70, MMm=40, N=12, nonlin=True)
    else:
        cfg = oracle.filament_cfg(LLm=64, MMm=40, N=16, np_xi=1, np_eta=1)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv(switch, env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey)
        m.step(4)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "We", "Wi", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


@pytest.mark.parametrize("case", ["filament", "basin"])
def test_prsgrd_uv_tile_rows_bitwise(case, monkeypatch):
    """k_prsgrd_uv on 64x8 tiles (ROMS_GPU_PRS_TY=8) equals the 64x4 form
    bitwise over 4 whole steps (periodic Filament, closed split-EOS basin)."""
    if case == "basin":
        cfg = basin_cfg(LLm=70, MMm=42, N=12, nonlin=True)
    else:
        cfg = oracle.filament_cfg(LLm=64, MMm=40, N=16, np_xi=1, np_eta=1)
    out = []
    for env in ("4", "8"):
        monkeypatch.setenv("ROMS_GPU_PRS_TY", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey)
        m.step(4)
        out.append({n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


@pytest.mark.parametrize("case", ["filament", "basin_odd", "basin_obc_odd"])
def test_ld16_windows_bitwise(case, monkeypatch):
    """LDS windows read two doubles per lane (ROMS_GPU_LD16=1, opt-in, needs
    the padded pitch: k_prsgrd_uv's raw and u/v windows) equal the 8-B form
    bitwise over 4 whole steps and one prsgrd routine call; odd Lm puts the
    last pair of a row half outside -1..Lm+2 (its upper double must read as 0)."""
    if case == "basin_odd":
        cfg = basin_cfg(LLm=71, MMm=41, N=12, nonlin=True)
    elif case == "basin_obc_odd":
        cfg = basin_cfg(LLm=69, MMm=37, N=10, nonlin=True)
        cfg.obc, cfg.island, cfg.curvgrid = 15, 1, 0
    else:
        cfg = oracle.filament_cfg(LLm=64, MMm=40, N=16, np_xi=1, np_eta=1)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("ROMS_GPU_LD16", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey, obc=cfg.obc, island=bool(cfg.island))
        m.step(4)
        r = {n: m.get(n) for n in ("zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc")}
        m.prsgrd()
        m.sync()
        r["ru"], r["rv"] = m.get("ru"), m.get("rv")
        out.append(r)
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


@pytest.mark.parametrize("lmd", [oracle.LMD_ICELAND, oracle.LMD_ALL | oracle.LMD_DDMIX])
def test_kpp_int_staged_rig_bitwise(lmd, monkeypatch):
    """k_kpp_int with the Rig stencil windows staged in LDS (ROMS_GPU_KPP_TY
    4 = the default, 2, 8, 43) equals the one-row form (=0) bitwise over 4 whole steps of
    the split-EOS basin with KPP (edge clamps at all four closed walls, a
    partial last block row: MMm = 42)."""
    cfg = basin_cfg(LLm=70, MMm=42, N=12, nonlin=True)
    out = []
    for env in ("0", "4", "2", "8", "43"):   # one row; 64x4; 64x2; 64x8; 64x4 at 3 waves/SIMD
        monkeypatch.setenv("ROMS_GPU_KPP_TY", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                    dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, lmd=lmd,
                                    surf_flux=True)
        m.step(4)
        out.append({n: m.get(n) for n in ("u", "v", "t", "Akv", "Akt", "hbls", "hbbl", "ghat")})
        m.close()
    for o in out[1:]:
        for n in out[0]:
            assert np.array_equal(out[0][n], o[n]), n


@pytest.mark.parametrize("obc", [15, 0])
def test_visc3d_staged_windows_bitwise(obc, monkeypatch):
    """visc3d with the level's raw u, v, Hz windows staged in LDS
    (ROMS_GPU_VISC_STG=1) equals the per-point-load form bitwise over 4 whole
    steps: the open basin with an island and sponge bands (nonzero visc2_r /
    visc2_p there), and the closed basin."""
    cfg = basin_cfg(LLm=70, MMm=42, N=12, nonlin=True)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("ROMS_GPU_VISC_STG", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                    dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, obc=obc,
                                    v_sponge=1.0 if obc else 0.0, island=bool(obc))
        if obc:
            assert float(np.abs(m.get("visc2_r")).max()) > 0
        m.step(4)
        out.append({n: m.get(n) for n in ("u", "v", "t", "rufrc", "rvfrc", "ubar", "vbar")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n


@pytest.mark.parametrize("obc", [15, 0])
def test_t3dmix_staged_windows_bitwise(obc, monkeypatch):
    """t3dmix with the level's Hz, T, S windows staged in LDS
    (ROMS_GPU_T3DMIX_STG=1) equals the per-point-load form bitwise over 4
    whole steps (sponge bands give nonzero diff2 in the open basin)."""
    cfg = basin_cfg(LLm=70, MMm=42, N=12, nonlin=True)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("ROMS_GPU_T3DMIX_STG", env)
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=True, nonlin_eos=True,
                                    dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey, obc=obc,
                                    v_sponge=1.0 if obc else 0.0, island=bool(obc))
        if obc:
            assert float(np.abs(m.get("diff2")).max()) > 0
        m.step(4)
        out.append({n: m.get(n) for n in ("u", "v", "t", "zeta")})
        m.close()
    for n in out[0]:
        assert np.array_equal(out[0][n], out[1][n]), n
