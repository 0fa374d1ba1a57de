"""The j-marching strip kernels (the defaults in whole steps) against the
tiles they replace, whole runs bitwise equal:
  * prsgrd's ru/rv with the momentum r.h.s. (k_prsgrd_strip.hip) against the
    k_prsgrd_uv tiles (ROMS_GPU_PRS_STRIP=0);
  * the horizontal tracer advection of pre_step3d and step3d_t
    (k_tracer_strip.hip) against the k_pre_tracer_h1 / k_step3d_t_h1 tiles
    (ROMS_GPU_T_STRIP=0).

The strips evaluate each elementary difference, harmonic mean and advective
flux once per face and take the i-neighbours' values through DPP lane shifts;
the tiles stage everything through LDS and evaluate each flux twice.  Same
expressions in the same order, so every field matches bit for bit.  The cases
cover both EOS forms (SPLIT_EOS and linear), one and two tracers, closed
edges (the strips at the west/east edge shuffle the clamped column, the
south/north bands stay on tiles), periodic edges, a land mask, open
boundaries, grids with a partial last strip and a partial last row chunk,
pre_step3d's Hz_bak/Hz_fwd formed in the strips (ROMS_GPU_OMEGA_HB=0) or read
from the predictor's omega, and the C3 depth and time step (prsgrd.F:229-421,
compute_horiz_rhs_uv_terms.h, compute_horiz_tracer_fluxes.h,
pre_step3d4S.F:136-180, step3d_t_ISO.F:188-213).
"""
import os

import numpy as np
import pytest

import romsgpu

pytestmark = pytest.mark.gpu

FIELDS = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "rufrc", "rvfrc", "Hz", "Akt")

CASES = {
    # closed basin, SPLIT_EOS + KPP, 3 strips (the last one partial), rows 3..Mm-1 in strips
    "basin_split": dict(case_id=1, LLm=150, MMm=45, N=12, NT=2, salinity=True, nonlin_eos=True, dt=300.0,
                        ndtfast=60, sizex=300e3, sizey=90e3, lmd=romsgpu.LMD_ICELAND),
    # C3's depth on a grid with one full strip and a 4-column remainder
    "c3_depth": dict(case_id=1, LLm=64, MMm=40, N=100, NT=2, salinity=True, nonlin_eos=True, dt=300.0,
                     ndtfast=60, sizex=128e3, sizey=80e3, lmd=romsgpu.LMD_ICELAND),
    # doubly periodic Filament, linear EOS (no strip at an edge)
    "filament": dict(case_id=0, LLm=130, MMm=33, N=10, NT=2, salinity=True, nonlin_eos=False, dt=5.0, ndtfast=60,
                     sizex=13e3, sizey=0.8e3),
    # one tracer
    "filament_nt1": dict(case_id=0, LLm=70, MMm=30, N=8, NT=1, salinity=False, nonlin_eos=False, dt=5.0,
                         ndtfast=60, sizex=7e3, sizey=0.75e3),
    # Pipes_ana: land mask, KPP, pipe sources
    "pipes": dict(case_id=2, LLm=100, MMm=60, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                  sizex=30e3, sizey=18e3, lmd=True),
    # open boundaries (Flather / Orlanski) and an island
    "basin_obc": dict(case_id=1, LLm=125, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                      sizex=250e3, sizey=56e3, lmd=romsgpu.LMD_ICELAND, obc=15, island=True),
}


def _run(case, env, nsteps):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = romsgpu.Model.from_case(**case)
        m.step(nsteps)
        m.sync()
        out = {f: m.get(f) for f in FIELDS}
        m.close()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return out


def _same(a, b):
    bad = [(f, float(np.nanmax(np.abs(a[f] - b[f])))) for f in FIELDS if not np.array_equal(a[f], b[f])]
    assert not bad, bad
    assert all(np.isfinite(b[f]).all() for f in FIELDS)


@pytest.mark.parametrize("name", list(CASES))
def test_strips_bitwise_equal_tiles(name):
    case = CASES[name]
    tiles = _run(case, {"ROMS_GPU_PRS_STRIP": "0", "ROMS_GPU_T_STRIP": "0"}, 4)
    _same(tiles, _run(case, {"ROMS_GPU_PRS_STRIP": "1", "ROMS_GPU_T_STRIP": "1"}, 4))


@pytest.mark.parametrize("name", ["basin_split", "pipes"])
def test_tracer_strips_form_hz_bak_fwd_bitwise(name):
    """pre_step3d's Hz_bak / Hz_fwd formed in the tracer strips themselves
    (ROMS_GPU_OMEGA_HB=0: not by the predictor's omega) against the tiles."""
    case = CASES[name]
    tiles = _run(case, {"ROMS_GPU_T_STRIP": "0", "ROMS_GPU_OMEGA_HB": "0"}, 3)
    _same(tiles, _run(case, {"ROMS_GPU_T_STRIP": "1", "ROMS_GPU_OMEGA_HB": "0"}, 3))
