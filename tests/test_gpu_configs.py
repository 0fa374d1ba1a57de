"""The BASELINE.json configurations against the oracle, and the cppdefs.opt
switch variants.

  C2  Filament + SALINITY (linear EOS, T and S, NT = 2), doubly periodic,
      dx = 100 m, dy = 25 m: 64x64x50 for 100 steps (field RMS < 1e-10, the
      north_star bound) and the full 512x512x50 bench grid for 2 steps.
  C4  Iceland-size stand-in (the real Iceland inputs are offline-unavailable,
      SURVEY.md 8(c)): 192x192x20 synthetic basin with the Iceland switch set
      of Examples/Iceland/Iceland_parent/cppdefs.opt -- OBC_M2FLATHER /
      M3ORLANSKI / TORLANSKI with *_FRC_BRY data, SPONGE, MASKING (island),
      CURVGRID, NONLIN+SPLIT EOS, LMD_MIXING+KPP+BKPP+RIMIX+NONLOCAL without
      LMD_CONVEC -- dt = 900 s, ndtfast = 30 (nfast 41, .../roms.in).
      Single domain vs the oracle; 4x2 processor grid (8 subdomains, one
      thread each) vs the single domain bitwise.  The 4x2 check runs without
      the sponge: the reference sets the sponge bands on each rank's own
      points only (set_nudgcof.F:89-111, no exchange after it) while
      visc3d_S.F / t3dmix_S.F:55 read them across the halo, so a sponge run is
      decomposition dependent in the reference itself.
  C5  C4 + 8 passive tracers (NT = 10, param.opt nt_passive): passive
      tracers take Akt(min(itrc, iTandS)) (step3d_t_ISO.F:1044), no EOS or
      KPP surface terms; initial Gaussian blobs.
  Switch variants: LMD_RIMIX / LMD_CONVEC / LMD_NONLOCAL individually off,
  UV_ADV and UV_COR off (compute_horiz_rhs_uv_terms.h, compute_vert_rhs_uv_terms.h).

The OBC/SPONGE/CURVGRID branches of the oracle have no runnable golden log
offline (test_gpu_obc.py): "parity unpinned" there; everything else is
pinned through the Filament / Pipes_ana goldens (test_oracle_golden.py).
"""
import os

import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_multirank import check_decomposition
from test_gpu_parity import PROGNOSTIC, RMS_RUN, basin_cfg, check_fields, rms

pytestmark = pytest.mark.gpu


def pair(cfg):
    o = oracle.Oracle(cfg)
    o.init()
    m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex,
                                sizey=cfg.sizey, lmd=cfg.lmd, surf_flux=bool(cfg.surf_flux), obc=cfg.obc,
                                v_sponge=cfg.v_sponge, island=bool(cfg.island), curvgrid=bool(cfg.curvgrid),
                                uv_adv=bool(cfg.uv_adv), uv_cor=bool(cfg.uv_cor), bulk_frc=bool(cfg.bulk_frc))
    return o, m


def c2_cfg(L, M, N=50):
    """C2: Filament physics + SALINITY at dx = 100 m, dy = 25 m."""
    return oracle.filament_cfg(LLm=L, MMm=M, N=N, NT=2, salinity=True, sizex=100.0 * L, sizey=25.0 * M,
                               np_xi=1, np_eta=1)


def test_c2_filament_salinity_100_steps():
    cfg = c2_cfg(64, 64)
    o, m = pair(cfg)
    o.step(100)
    m.step(100)
    m.sync()
    dump = os.environ.get("ROMS_TEST_DUMP")
    if dump:   # debugging aid: both sides' fields of this run
        np.savez(dump, **{"gpu_" + n: m.get(n) for n in ("zeta", "u", "v", "t")},
                 **{"orc_" + n: o.field(n) for n in ("zeta", "u", "v", "t")})
    assert o.tindex() == m.t.as_list()
    check_fields(o, m, PROGNOSTIC, 64, 64, RMS_RUN, kind="rms")
    # both tracers moved and stayed distinct (S is really advected)
    t = m.get("t")
    assert t.shape[0] == 3 * 2 * 50
    m.close()


def test_models_in_sequence_are_independent():
    """A new model's first kernels see its zero-filled arrays, not what an
    earlier model of the same process left in recycled device memory: the
    fill is a null-stream hipMemset, which the library's non-blocking stream
    does not wait for, so dev_alloc waits for it (before that fix the C2
    100-step test failed in some test-process histories).  This sequence is
    the end-to-end symptom; test_zero_fill_lands_before_the_stream below
    drives the allocation path itself."""
    def run(cfg, n):
        m = romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                    nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast,
                                    sizex=cfg.sizex, sizey=cfg.sizey, lmd=cfg.lmd, surf_flux=bool(cfg.surf_flux))
        m.step(n)
        out = {k: m.get(k) for k in ("zeta", "ubar", "u", "v", "t", "We")}
        m.close()
        return out
    c2 = c2_cfg(64, 64)
    a = run(c2, 20)
    other = basin_cfg(LLm=40, MMm=24, N=50, nonlin=True)   # leaves nonzero data in freed memory
    other.lmd, other.surf_flux = oracle.LMD_ALL, 1
    run(other, 5)
    b = run(c2, 20)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_zero_fill_lands_before_the_stream():
    """Regression test of the round-2 race, through the library's own
    allocator (roms_gpu_selftest_zero_fill): many small arrays filled with
    ones and freed, allocated again (recycled memory) with the zero fill,
    read and overwritten on the library stream at once.  With the
    null-stream fill not joined (the round-2 dev_alloc, rebuilt as an A/B
    library) these two shapes report 14-65 thousand bad elements in 20 of 20
    tries; the library reports 0 (profiles/r3_k_zero_fill_probe.txt)."""
    m = romsgpu.Model.from_case(0, 32, 24, 16, sizex=12.8e3, sizey=3.2e3)
    for n, chunks in ((1 << 16, 512), (1 << 14, 1024)):
        for _ in range(3):
            assert m.selftest_zero_fill(n, chunks) == 0, (n, chunks)
    m.close()


def test_c2_full_grid_2_steps():
    """The bench workload itself (512x512x50, NT = 2) for 2 steps."""
    cfg = c2_cfg(512, 512)
    o, m = pair(cfg)
    o.step(2)
    m.step(2)
    m.sync()
    check_fields(o, m, ["zeta", "ubar", "vbar", "u", "v", "t", "We", "Hz"], 512, 512, RMS_RUN, kind="rms")
    m.close()


def c4_cfg(NT=2, L=192, sponge=1.0e3, island=1):
    """C4 stand-in: Iceland switches on a 192x192x20 synthetic open basin."""
    c = basin_cfg(LLm=L, MMm=L, N=20, NT=NT, nonlin=True, dt=900.0, ndtfast=30, sizex=15.0e3 * L,
                  sizey=15.0e3 * L)
    c.obc, c.ubind, c.v_sponge, c.island, c.curvgrid = 15, 0.1, sponge, island, 1
    # BULK_FRC (cppdefs.opt:15) over the synthetic analytic atmosphere: the
    # surface fluxes, u* under KPP and the rain heat of step3d_t come from it
    c.lmd, c.surf_flux, c.bulk_frc = oracle.LMD_ICELAND, 0, 1
    return c


def _case(cfg):
    return dict(case_id=cfg.case_id, LLm=cfg.LLm, MMm=cfg.MMm, N=cfg.N, NT=cfg.NT, salinity=bool(cfg.salinity),
                nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex, sizey=cfg.sizey,
                lmd=cfg.lmd, surf_flux=bool(cfg.surf_flux), obc=cfg.obc, v_sponge=cfg.v_sponge,
                island=bool(cfg.island), curvgrid=bool(cfg.curvgrid), bulk_frc=bool(cfg.bulk_frc))


@pytest.mark.parametrize("NT", [2, 10], ids=["C4", "C5"])
def test_c4_c5_single_domain_vs_oracle(NT):
    cfg = c4_cfg(NT=NT)
    o, m = pair(cfg)
    assert m.t.nfast == 41
    o.step(40)
    m.step(40)
    m.sync()
    check_fields(o, m, PROGNOSTIC + ["Akv", "Akt", "hbls", "hbbl", "stflx", "swflx", "sustr"], cfg.LLm, cfg.MMm,
                 RMS_RUN, kind="rms")
    assert float(np.max(np.abs(o.field("swflx")))) > 0.0   # rain: the BULK_FRC heat-of-rain term is live
    if NT == 10:   # every passive tracer separately (each carries its own blob)
        a, b = m.get("t"), o.field("t")
        n3 = cfg.N
        for it in range(NT):
            sl = slice(it * 3 * n3, (it + 1) * 3 * n3)
            e = rms(a[sl][..., 2:-2, 2:-2], b[sl][..., 2:-2, 2:-2])
            assert e < RMS_RUN, (it + 1, e)
        assert float(np.max(np.abs(b[9 * 3 * n3:]))) > 0.1   # tracer 10 is not empty
    m.close()


@pytest.mark.parametrize("NT", [2, 10], ids=["C4", "C5"])
def test_c4_c5_4x2_bitwise_equals_single_domain(NT):
    check_decomposition(_case(c4_cfg(NT=NT, sponge=0.0)), 4, 2, nsteps=4)


SWITCHES = [
    ("no_rimix", dict(lmd=oracle.LMD_ICELAND & ~oracle.LMD_RIMIX)),
    ("no_nonlocal", dict(lmd=oracle.LMD_ALL & ~oracle.LMD_NONLOCAL)),
    ("convec", dict(lmd=oracle.LMD_ALL)),
    ("no_uv_adv", dict(uv_adv=0)),
    ("no_uv_cor", dict(uv_cor=0)),
    ("no_uv_adv_cor", dict(uv_adv=0, uv_cor=0)),
    ("curv_no_uv_cor", dict(uv_cor=0, curvgrid=1)),
]


@pytest.mark.parametrize("name,sw", SWITCHES, ids=[s[0] for s in SWITCHES])
def test_switch_variants_30_steps(name, sw):
    c = basin_cfg(LLm=40, MMm=32, N=16, nonlin=True)
    c.surf_flux = 1
    c.lmd = oracle.LMD_ICELAND
    for k, v in sw.items():
        setattr(c, k, v)
    o, m = pair(c)
    o.step(30)
    m.step(30)
    m.sync()
    names = PROGNOSTIC + (["Akv", "Akt", "ghat"] if c.lmd else [])
    check_fields(o, m, names, c.LLm, c.MMm, RMS_RUN, kind="rms")
    m.close()


def test_invalid_lmd_sets_are_rejected():
    """Sets the reference cannot build or run correctly fail loudly."""
    for bad in (1, 1 | 2, 1 | 2 | 4 | 16, 128):
        with pytest.raises(romsgpu.RomsGpuError):
            romsgpu.Model.from_case(1, 16, 16, 8, 2, salinity=True, nonlin_eos=True, lmd=bad, dt=60.0, ndtfast=30,
                                    sizex=32e3, sizey=32e3)
    # LMD_DDMIX reads t(..,isalt) (lmd_vmix.F:289-296): not without SALINITY
    with pytest.raises(romsgpu.RomsGpuError):
        romsgpu.Model.from_case(1, 16, 16, 8, 1, salinity=False, nonlin_eos=True,
                                lmd=romsgpu.LMD_ICELAND | romsgpu.LMD_DDMIX, dt=60.0, ndtfast=30, sizex=32e3,
                                sizey=32e3)


def c3_cfg(L=64, M=48, N=100):
    """C3's switch set and time step exactly as bench.py --workload c3 runs
    it: the closed synthetic basin, NONLIN+SPLIT EOS, T+S,
    LMD_MIXING+KPP+BKPP+RIMIX+NONLOCAL without LMD_CONVEC, wind stress,
    dt = 300 s, ndtfast = 60 (nfast 82), N = 100 (the segment solvers), on
    a smaller horizontal grid with the bench's 2 km spacing."""
    c = basin_cfg(LLm=L, MMm=M, N=N, nonlin=True, dt=300.0, ndtfast=60, sizex=2.0e3 * L, sizey=2.0e3 * M)
    c.lmd = oracle.LMD_ICELAND
    return c


def test_c3_exact_switches_100_steps_vs_oracle():
    """north_star's bound as stated: field RMS < 1e-10 after 100 steps (u, v,
    w, T, S, zeta absolute), at C3's switch set, time step and depth."""
    cfg = c3_cfg()
    o, m = pair(cfg)
    assert m.t.nfast == 82
    o.step(100)
    m.step(100)
    m.sync()
    errs = check_fields(o, m, PROGNOSTIC + ["Akv", "Akt", "hbls", "hbbl", "ghat"], cfg.LLm, cfg.MMm, RMS_RUN,
                        kind="rms")
    print("C3 switch set, 100 steps, RMS error per field:", {k: "%.1e" % v for k, v in errs.items()})
    m.close()


def test_c3_2x2_n100_bitwise_equals_single_domain():
    """C3's 2x2 split at N = 100: 101-level halo messages and the segment
    solvers next to the rank edges, bitwise equal to the single domain."""
    check_decomposition(_case(c3_cfg(L=72, M=56)), 2, 2, nsteps=3)


def test_c3_full_grid_1_step_vs_oracle():
    """C3 at its real size (1024x1024x100, the bench workload itself) against
    the oracle for one step: every routine's multi-block segment tiling and
    the 1040-double row pitch at full size.  One oracle
    step here is 1.05e8 cell updates on one core (about 45 s on the GPU box's
    host, 130 s in the build container); the later steps' time-stepping
    branches are covered at 64x48x100 for 100 steps above."""
    cfg = c3_cfg(L=1024, M=1024)
    o, m = pair(cfg)
    assert m.t.nfast == 82
    o.step(1)
    m.step(1)
    m.sync()
    assert o.tindex() == m.t.as_list()
    names = [n for n in PROGNOSTIC if n not in ("We", "Wi")] + ["w", "Akv", "Akt", "hbls", "hbbl"]
    errs = check_fields(o, m, names, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
    errs.update(check_fields(o, m, ["We", "Wi"], cfg.LLm, cfg.MMm, RMS_WE_WI, kind="rms"))
    print("C3 1024x1024x100, 1 step, RMS error per field:", {k: "%.1e" % v for k, v in errs.items()})
    m.close()
    del o


# The vertical velocity is held absolutely at the north_star bound (w =
# pm*pn*(We+Wi), m/s).  We and Wi in m^3/s are column integrals of a nearly
# cancelling flux divergence a few steps from rest, so the segment solvers'
# 1e-15 reordering of u, v shows up amplified in their relative RMS: measured
# 1.25e-10 after one C3 step (gpurun_out/tests_g3.log of round 5); bounded at
# 4x that.
RMS_WE_WI = 5e-10


def test_c3_512_3_steps_vs_oracle():
    """C3's switch set at 512x512x100 for 3 steps against the oracle: the
    later-step branches at full multi-block segment tiling -- the predictor's
    AB3 coefficients after the forward start (pre_step3d4S.F:83-134),
    set_HUV1's NOW/MID/BAK extrapolation (set_depth.F:283-412) and the fast
    loop's AB3-AM4 weights past its start (step2d_FB.F:87-99) -- which the
    full-grid test above reaches for one step only.  One
    oracle step is 2.6e7 cell updates on one host core (about 12 s on the GPU
    box)."""
    cfg = c3_cfg(L=512, M=512)
    o, m = pair(cfg)
    assert m.t.nfast == 82
    names = [n for n in PROGNOSTIC if n not in ("We", "Wi")] + ["w", "Akv", "Akt", "hbls", "hbbl", "ghat"]
    for step in range(1, 4):
        o.step(1)
        m.step(1)
        m.sync()
        assert o.tindex() == m.t.as_list()
        errs = check_fields(o, m, names, cfg.LLm, cfg.MMm, RMS_RUN, kind="rms")
        errs.update(check_fields(o, m, ["We", "Wi"], cfg.LLm, cfg.MMm, RMS_WE_WI, kind="rms"))
        print("C3 512x512x100, step %d, RMS error per field:" % step, {k: "%.1e" % v for k, v in errs.items()})
    m.close()
    del o


def test_c3_full_grid_2x2_bitwise_equals_single_domain():
    """The full C3 basin split 2x2 (four 512x512x100 subdomains on threads of
    one GPU, the bench's N = 4 layout) equals the single domain bitwise."""
    check_decomposition(_case(c3_cfg(L=1024, M=1024)), 2, 2, nsteps=2)
