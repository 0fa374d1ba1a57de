"""Pin the CPU oracle against the reference's own golden logs.

tests/Filament/benchmark.result_github_gnu (reference) holds the per-step
diag norms of the Filament case at 3x2 MPI ranks, 20 steps; the oracle
emulates the same per-rank pairwise + tree reductions (diag.F:409-535) and
must reproduce every printed ES23.16 digit.
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
