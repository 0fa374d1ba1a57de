"""Pin the CPU oracle against the reference's own golden logs.

tests/Filament/benchmark.result_github_gnu (reference) holds the per-step
diag norms of the Filament case at 3x2 MPI ranks, 20 steps; the oracle
emulates the same per-rank pairwise + tree reductions (diag.F:409-535) and
must reproduce every printed ES23.16 digit.

tests/Pipes_ana/benchmark.result_github_{gnu,ifx} pin the KPP/BKPP mixing
(lmd_vmix.F, lmd_kpp.F), the nonlinear split EOS, land masking and the pipe
sources: the reference's two compilers already disagree by up to 1.3e-14
(relative) over those 20 steps, and the oracle must stay inside that spread.
"""
import json
import os

import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _rows(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)["rows"]


def _fmt(x):
    return "%23.16E" % x


def test_filament_golden_bit_exact():
    rows = _rows("filament_github_gnu")
    o = oracle.Oracle(oracle.filament_cfg())
    o.init()
    assert o.nfast() == 82          # benchmark.result_github_gnu: "nfast =  82"
    got = [o.norms()]
    for _ in range(20):
        o.step()
        got.append(o.norms())
    for r, g in zip(rows, got):
        assert [r["ke"], r["ke2b"], r["cu_adv"], r["cu_w"]] == [_fmt(v).strip() for v in g], r["step"]


def test_filament_gnu_vs_ifx_spread():
    """The two reference compilers differ ~1e-13; the oracle sits on gnu."""
    gnu, ifx = _rows("filament_github_gnu"), _rows("filament_github_ifx")
    for a, b in zip(gnu, ifx):
        ka, kb = float(a["ke"]), float(b["ke"])
        assert abs(ka - kb) <= 1e-12 * abs(ka)


def test_weights_normalised():
    o = oracle.Oracle(oracle.filament_cfg(LLm=8, MMm=8, N=4))
    o.init()
    w = o.weights()
    nf = o.nfast()
    assert abs(w[0, :nf].sum() - 1.0) < 1e-14
    assert abs(w[1, :nf].sum() - 1.0) < 1e-14


_KEYS = ("ke", "ke2b", "cu_adv", "cu_w")


def _rel(a, b):
    return abs(a - b) / abs(b) if b != 0 else abs(a)


def test_pipes_ana_golden_within_compiler_spread():
    gnu, ifx = _rows("pipes_ana_github_gnu"), _rows("pipes_ana_github_ifx")
    o = oracle.Oracle(oracle.pipes_cfg())
    o.init()
    assert o.nfast() == 41          # benchmark.result_github_gnu: "nfast =  41"
    got = [o.norms()]
    for _ in range(20):
        o.step()
        got.append(o.norms())
    spread = max(_rel(float(x[k]), float(g[k])) for g, x in zip(gnu, ifx) for k in _KEYS)
    assert spread < 2e-14
    worst = 0.0
    for g, v in zip(gnu, got):
        for k, val in zip(_KEYS, v):
            worst = max(worst, _rel(val, float(g[k])))
    assert worst <= spread, (worst, spread)
    # step 0 (init: omega with the pipe inflow) is bit-exact
    assert [gnu[0][k] for k in _KEYS] == [_fmt(v).strip() for v in got[0]]


def test_rivers_ana_golden_single_domain_drift():
    """tests/Rivers_ana (river_frc.F analytic river, KPP, land mask).  The
    reference's golden log comes from a 3x2 MPI run whose ana_grid.h fills
    only 0..nx+1, 0..ny+1 of each rank, and ANA_GRID exchanges nothing
    (grid.F:444-446): the outer halo ring keeps h = pm = pn = 0 at the ranks'
    shared edges, so the reference's result depends on its decomposition.
    The single-domain oracle therefore matches the log within the gnu/ifx
    spread for the first step and drifts slowly after (measured: 2.4e-11 at
    step 2, 2e-9 at step 9, then 1e-3 by step 20 once KPP thresholds flip);
    the GPU run decomposed like the reference reproduces the log within the
    spread (tests/test_gpu_multirank.py::test_rivers_ana_3x2_within_compiler_spread)."""
    gnu, ifx = _rows("rivers_ana_github_gnu"), _rows("rivers_ana_github_ifx")
    o = oracle.Oracle(oracle.rivers_cfg())
    o.init()
    assert o.nfast() == 41          # benchmark.result_github_gnu: "nfast =  41"
    got = [o.norms()]
    for _ in range(9):
        o.step()
        got.append(o.norms())
    spread = max(_rel(float(x[k]), float(g[k])) for g, x in zip(gnu, ifx) for k in _KEYS)
    for s, (g, v) in enumerate(zip(gnu, got)):
        worst = max(_rel(val, float(g[k])) for k, val in zip(_KEYS, v))
        assert worst <= (spread if s <= 1 else 5e-9), (s, worst, spread)
