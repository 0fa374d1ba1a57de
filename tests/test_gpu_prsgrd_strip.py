"""prsgrd's ru/rv with the momentum r.h.s. in j-marching strips
(k_prsgrd_strip.hip, the default in whole steps) against the k_prsgrd_uv
tiles (ROMS_GPU_PRS_STRIP=0): whole runs bitwise equal.

The strips evaluate each elementary difference, harmonic mean and advective
flux once per face and take the i-neighbours' values through DPP lane shifts;
the tiles stage everything through LDS and evaluate each flux twice.  Same
expressions in the same order, so every field matches bit for bit.  The cases
cover both EOS forms (SPLIT_EOS and linear), closed edges (the strips at the
west/east edge shuffle the clamped column, the south/north bands stay on
tiles), periodic edges, a land mask, open boundaries, grids with a partial
last strip and a partial last row chunk, and the C3 depth and time step
(prsgrd.F:229-421, compute_horiz_rhs_uv_terms.h).
"""
import os

import numpy as np
import pytest

import romsgpu

pytestmark = pytest.mark.gpu

FIELDS = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "rufrc", "rvfrc")

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
    # Pipes_ana: land mask, KPP, pipe sources
    "pipes": dict(case_id=2, LLm=100, MMm=60, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                  sizex=30e3, sizey=18e3, lmd=True),
    # open boundaries (Flather / Orlanski) and an island
    "basin_obc": dict(case_id=1, LLm=125, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                      sizex=250e3, sizey=56e3, lmd=romsgpu.LMD_ICELAND, obc=15, island=True),
}


def _run(case, strip, nsteps):
    os.environ["ROMS_GPU_PRS_STRIP"] = strip
    try:
        m = romsgpu.Model.from_case(**case)
        m.step(nsteps)
        m.sync()
        out = {f: m.get(f) for f in FIELDS}
        m.close()
    finally:
        del os.environ["ROMS_GPU_PRS_STRIP"]
    return out


@pytest.mark.parametrize("name", list(CASES))
def test_strips_bitwise_equal_tiles(name):
    case = CASES[name]
    a = _run(case, "0", 4)
    b = _run(case, "1", 4)
    bad = [(f, float(np.nanmax(np.abs(a[f] - b[f])))) for f in FIELDS if not np.array_equal(a[f], b[f])]
    assert not bad, bad
    assert all(np.isfinite(b[f]).all() for f in FIELDS)
