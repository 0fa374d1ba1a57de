"""Device layout and block shapes that must not change a single bit.

* Device row pitch (roms_dev.h): rows of Lm+4 doubles rounded up to 128 B
  and every array's base shifted so that i = 1 starts a line.  Host data
  cross the ABI in the reference's layout (rows of Lm+4) both ways; runs with
  the padded pitch (default) and the host pitch on the device
  (ROMS_GPU_PITCH=0) are bitwise equal, on grids whose Lm+4 is and is not a
  multiple of 16, closed and periodic, with open edges, forcing records and
  a decomposition (the halo messages index the device rows).  The restart
  and history files (test_gpu_io.py) and the pipe/river/tide inputs
  (test_gpu_pipes.py, test_gpu_rivers.py, test_gpu_forcing.py) run on the
  padded layout by default.
* v columns of the momentum segment solvers on 16 x 4 tiles per wavefront
  (ROMS_GPU_SEG_VTILE, k_colseg.h): the same column arithmetic as rows of 64,
  so bitwise equal.
* j-marching per-level horizontal kernels (ROMS_GPU_HJC): windows in an LDS
  ring, same expressions as the 64 x 4 tiles.
* routines without a data dependence on two streams inside the step
  (ROMS_GPU_PAR=1, opt-in): the same kernels on the same inputs.
"""
import numpy as np
import pytest

import oracle
import romsgpu
from test_gpu_configs import c3_cfg
from test_gpu_multirank import run_decomposed
from test_gpu_parity import basin_cfg

pytestmark = pytest.mark.gpu

FIELDS = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "z_r", "z_w", "rho", "rufrc",
          "rvfrc", "DU_avg1", "DV_avg1", "Zt_avg1")


def _model(cfg, **kw):
    return romsgpu.Model.from_case(cfg.case_id, cfg.LLm, cfg.MMm, cfg.N, cfg.NT, salinity=bool(cfg.salinity),
                                   nonlin_eos=bool(cfg.nonlin_eos), dt=cfg.dt, ndtfast=cfg.ndtfast, sizex=cfg.sizex,
                                   sizey=cfg.sizey, lmd=cfg.lmd, obc=cfg.obc, island=bool(cfg.island),
                                   v_sponge=cfg.v_sponge, curvgrid=bool(cfg.curvgrid), **kw)


def _cfg(kind):
    if kind == "filament_61":       # Lm+4 = 65: padded to 80
        return oracle.filament_cfg(LLm=61, MMm=37, N=16, np_xi=1, np_eta=1)
    if kind == "basin_60":          # Lm+4 = 64: already a multiple of 16 (pitch unchanged, base shifted)
        c = basin_cfg(LLm=60, MMm=44, N=12, nonlin=True)
        c.lmd = oracle.LMD_ICELAND
        return c
    if kind == "obc_island":        # open edges, boundary arrays (not planar), sponge, curvilinear grid
        c = basin_cfg(LLm=45, MMm=38, N=12, nonlin=True)
        c.obc, c.ubind, c.v_sponge, c.island, c.curvgrid, c.lmd = 15, 0.1, 1.0, 1, 1, oracle.LMD_ICELAND
        return c
    return c3_cfg(L=70, M=52)       # N = 100: the segment solvers


def _run(kind, env, monkeypatch, nsteps=4):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = _cfg(kind)
    m = _model(cfg)
    if kind == "obc_island":        # forcing records of a planar field and a boundary array through the ABI
        rng = np.random.default_rng(7)
        for name in ("sustr", "zeta_west"):
            a = m.get(name)
            m.frc_record(name, 0, 0.0, a)
            m.frc_record(name, 1, 1.0, a + 1e-3 * rng.standard_normal(a.shape))
        m.frc_interp(0.25)
    m.step(nsteps)
    out = {n: m.get(n) for n in FIELDS}
    m.close()
    for k in env:
        monkeypatch.delenv(k)
    return out


@pytest.mark.parametrize("kind", ["filament_61", "basin_60", "obc_island", "c3_n100"])
def test_device_row_pitch_bitwise(kind, monkeypatch):
    a = _run(kind, {"ROMS_GPU_PITCH": "0"}, monkeypatch)
    b = _run(kind, {}, monkeypatch)
    for n in FIELDS:
        assert np.array_equal(a[n], b[n]), n


def test_device_row_pitch_decomposed_bitwise(monkeypatch):
    """2x2 subdomains (in-process transport: the halo pack/unpack index the
    device rows) with and without the padded pitch."""
    case = dict(case_id=1, LLm=50, MMm=36, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                sizex=100e3, sizey=72e3, lmd=True)
    monkeypatch.setenv("ROMS_GPU_PITCH", "0")
    a, _ = run_decomposed(case, 2, 2, 3)
    monkeypatch.delenv("ROMS_GPU_PITCH")
    b, _ = run_decomposed(case, 2, 2, 3)
    for r in range(4):
        for f in a[r][4]:
            assert np.array_equal(a[r][4][f], b[r][4][f]), (r, f)


def test_seg_vtile_bitwise(monkeypatch):
    """v columns on 16 x 4 tiles (default) vs rows of 64: pre_step3d and
    step3d_uv1 segment solvers, C3 switch set at N = 100, bitwise."""
    a = _run("c3_n100", {"ROMS_GPU_SEG_VTILE": "0"}, monkeypatch, nsteps=3)
    b = _run("c3_n100", {}, monkeypatch, nsteps=3)
    for n in FIELDS:
        assert np.array_equal(a[n], b[n]), n


@pytest.mark.parametrize("kind", ["filament_61", "basin_60", "obc_island", "c3_n100"])
def test_j_marching_horizontal_kernels_bitwise(kind, monkeypatch):
    """The per-level horizontal kernels that walk 64-wide strips through
    ROMS_GPU_HJC rows with their windows in an LDS ring (default 32) equal the
    64 x 4 tile forms (ROMS_GPU_HJC=0) bitwise; 8 rows (two ring turns per
    block) and the default on grids whose row count is not a multiple of the
    chunk."""
    a = _run(kind, {"ROMS_GPU_HJC": "0"}, monkeypatch)
    for jc in ("8", "32"):
        b = _run(kind, {"ROMS_GPU_HJC": jc}, monkeypatch)
        for n in FIELDS:
            assert np.array_equal(a[n], b[n]), (jc, n)


@pytest.mark.parametrize("kind", ["filament_61", "basin_60", "obc_island", "c3_n100"])
def test_two_stream_step_bitwise(kind, monkeypatch):
    """Whole steps with the independent routines on two streams (lmd_vmix
    beside prsgrd, the corrector's omega beside rho_eos, ...; opt-in,
    ROMS_GPU_PAR=1, measured slower) equal the one-stream order (the default)
    bitwise, eager first step and graph replays alike."""
    a = _run(kind, {}, monkeypatch, nsteps=5)
    b = _run(kind, {"ROMS_GPU_PAR": "1"}, monkeypatch, nsteps=5)
    for n in FIELDS:
        assert np.array_equal(a[n], b[n]), n
