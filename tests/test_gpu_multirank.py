"""Domain decomposition on the GPU (mpi_setup.F + mpi_exchanges.F semantics).

Subdomains of one processor grid are driven by threads of this process
(roms_gpu_comm_create_local: the library's pack/unpack kernels with device
copies as transport), so one GPU checks the decomposition end to end:
  * every subdomain's fields equal the single-domain run's window bitwise,
    for the periodic Filament and the closed basin, on 2x1, 1x2, 2x2, 3x2;
  * Filament on the reference's own 3x2 grid reproduces the golden diag log
    digit for digit (per-rank pairwise sums + the tree over ranks);
  * the RCCL transport (self-addressed send/recv on one GPU, captured in the
    step graph) gives the same fields as the single-rank wrap.
"""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import romsgpu

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "z_r", "z_w", "rho", "rufrc",
          "rvfrc", "DU_avg1", "DV_avg1", "DU_avg2", "DV_avg2", "Zt_avg1")
_group = [100]


def _case(kind):
    if kind == "filament":
        return dict(case_id=0, LLm=40, MMm=30, N=12, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
                    sizex=8.0e3, sizey=1.5e3)
    if kind == "pipes":   # tests/Pipes_ana: KPP/BKPP, land mask, pipe sources
        return dict(case_id=2, LLm=50, MMm=50, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                    sizex=30e3, sizey=30e3, lmd=True)
    if kind == "basin_flux":   # LMD with surface cooling/short-wave (convective KPP branches)
        return dict(case_id=1, LLm=36, MMm=28, N=20, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                    sizex=72e3, sizey=56e3, lmd=True, surf_flux=True)
    if kind == "basin_obc":   # open edges (Flather/Orlanski + boundary data) and an island; no sponge, whose
        # bands the reference sets on each rank's own points only (set_nudgcof.F, no exchange), so a
        # sponge run is decomposition dependent in the reference itself
        return dict(case_id=1, LLm=36, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                    sizex=72e3, sizey=56e3, lmd=True, obc=15, island=True)
    return dict(case_id=1, LLm=36, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                sizex=72e3, sizey=56e3, lmd=(kind == "basin_lmd"))


def run_decomposed(case, npx, npe, nsteps, fields=FIELDS, diag=False, probe=None):
    """Run every subdomain in its own thread; returns per-rank field dicts
    (and per-step diag norms of rank 0 when diag=True); probe(model) after
    the steps lands as the 6th item of each rank's tuple."""
    n = npx * npe
    _group[0] += 1
    grp = _group[0]
    out, errs, norms = [None] * n, [], []

    def work(rank):
        try:
            h = romsgpu.comm_create_local(grp, n, rank)
            m = romsgpu.Model.from_case(np_xi=npx, np_eta=npe, comm=h, rank=rank, **case)
            if diag:   # diag is collective: every rank calls it
                d = m.diag()
                if rank == 0:
                    norms.append(d)
            for _ in range(nsteps):
                m.step()
                d = m.diag() if diag else None
                if diag and rank == 0:
                    norms.append(d)
            m.sync()
            out[rank] = (m.iSW, m.jSW, m.Lm, m.Mm, {f: m.get(f) for f in fields}, probe(m) if probe else None)
            m.close()
            romsgpu.comm_destroy(h)
        except Exception as e:  # surfaced in the main thread
            errs.append((rank, repr(e)))

    th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not errs, errs
    return out, norms


def window(a, iSW, jSW, Lm, Mm):
    return a[..., jSW:jSW + Mm + 4, iSW:iSW + Lm + 4]


EXCHANGED = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "z_r", "z_w",
             "Akv", "Akt", "hbls", "hbbl")
LMD_FIELDS = ("Akv", "Akt", "hbls", "hbbl", "ghat", "swr_frac")


def check_decomposition(case, npx, npe, nsteps=5, fields=None):
    """Every subdomain of an npx x npe run equals the single-domain run's
    window bitwise (owned cells, and halos of the exchanged fields)."""
    per = case["case_id"] == 0
    if fields is None:
        fields = FIELDS + (LMD_FIELDS if case.get("lmd") else ())
    m = romsgpu.Model.from_case(**case)
    m.step(nsteps)
    ref = {f: m.get(f) for f in fields}
    m.close()
    parts, _ = run_decomposed(case, npx, npe, nsteps, fields=fields)
    bad = []
    for rank, (iSW, jSW, Lm, Mm, got, _) in enumerate(parts):
        jn, inn = divmod(rank, npx)
        # owned cells: interior + the closed-edge ghost row/column the BC code sets
        i_lo = 0 if (not per and inn == 0) else 1
        i_hi = Lm + 1 if (not per and inn == npx - 1) else Lm
        j_lo = 0 if (not per and jn == 0) else 1
        j_hi = Mm + 1 if (not per and jn == npe - 1) else Mm
        own = (Ellipsis, slice(j_lo + 1, j_hi + 2), slice(i_lo + 1, i_hi + 2))
        for f in fields:
            w = window(ref[f], iSW, jSW, Lm, Mm)
            g = got[f]
            if not np.array_equal(g[own], w[own]):
                bad.append((rank, f, "owned", float(np.max(np.abs(g[own] - w[own])))))
            elif f in EXCHANGED and not np.array_equal(g, w):
                bad.append((rank, f, "halo", float(np.max(np.abs(g - w)))))
    assert not bad, (npx, npe, bad[:6])


@pytest.mark.parametrize("kind", ["filament", "basin", "basin_lmd", "basin_flux", "pipes"])
@pytest.mark.parametrize("npx,npe", [(2, 1), (1, 2), (2, 2), (3, 2)])
def test_decomposition_bitwise_equals_single_domain(kind, npx, npe):
    check_decomposition(_case(kind), npx, npe)


@pytest.mark.parametrize("kind", ["filament", "basin"])
def test_fast_loop_overlap_bitwise(kind, monkeypatch):
    """Opt-in fast-loop overlap (ROMS_GPU_S2D_OVERLAP=1): each fast step's
    zeta/ubar/vbar exchange runs on a second stream while the next fast step's
    interior tiles compute; the rim tiles join it.  The subdomains must still
    equal the single-domain run bitwise."""
    monkeypatch.setenv("ROMS_GPU_S2D_OVERLAP", "1")
    test_decomposition_bitwise_equals_single_domain(kind, 2, 2)


@pytest.mark.parametrize("k", ["1", "2", "3"])
@pytest.mark.parametrize("kind,npx,npe", [("filament", 2, 2), ("basin", 3, 2), ("basin_lmd", 2, 2),
                                          ("basin_flux", 1, 2), ("filament", 3, 2)])
def test_fast_loop_exchange_interval_bitwise(kind, npx, npe, k, monkeypatch):
    """Barotropic exchange reduction (launch_step2d): the fast loop swaps
    zeta/ubar/vbar 2K deep after every K-th fast step and recomputes the
    overlap in between, instead of the reference's 2-deep swap after every
    fast step (step2d_FB.F:572-574).  K = 1 (every step), 2 and 3 give
    subdomains bitwise equal to the single-domain run, as the default K = 4
    does in test_decomposition_bitwise_equals_single_domain."""
    monkeypatch.setenv("ROMS_GPU_S2D_K", k)
    check_decomposition(_case(kind), npx, npe)


@pytest.mark.parametrize("k", ["6", "8"])
@pytest.mark.parametrize("kind,npx,npe", [("filament", 2, 1), ("basin", 2, 1)])
def test_fast_loop_wide_interval_bitwise(kind, npx, npe, k, monkeypatch):
    """The longest exchange intervals (halos 12 and 16 deep, 10 and 14 extra
    ghost cells) on subdomains just wide enough (LLm/np >= 2K+2): bitwise
    equal to the single domain, and the interval actually taken (one
    zeta/ubar/vbar swap per K fast steps)."""
    monkeypatch.setenv("ROMS_GPU_S2D_K", k)
    case = _case(kind)
    assert case["LLm"] // npx >= 2 * int(k) + 2 and case["MMm"] // npe >= 2 * int(k) + 2
    check_decomposition(case, npx, npe)
    parts, _ = run_decomposed(case, npx, npe, 1, fields=("zeta",), probe=lambda m: m.halo_exchanges())
    assert {p[5][1] for p in parts} == {int(k)}


@pytest.mark.parametrize("kind", ["filament", "basin"])
@pytest.mark.parametrize("LL,npx,k,k_taken", [(81, 8, "4", 2), (100, 12, "3", 1)])
def test_fast_loop_interval_fits_uneven_split(kind, LL, npx, k, k_taken, monkeypatch):
    """Uneven mpi_setup splits (mpi_setup.F:115-125): the edge ranks lose the
    remainder, so LLm/np is not the smallest subdomain (81 over 8: the east
    rank is 7 wide; 100 over 12: the edge ranks are 5 wide).  The library
    lowers K until 2K+2 fits the narrowest rank -- every rank
    takes the same K -- and the run stays bitwise equal to the single domain."""
    monkeypatch.setenv("ROMS_GPU_S2D_K", k)
    base = _case(kind)
    case = dict(base, LLm=LL, MMm=16, sizex=base["sizex"] * LL / base["LLm"], sizey=base["sizey"] * 16 / base["MMm"])
    widths = [romsgpu.rank_extent(LL, npx, r)[0] for r in range(npx)]
    assert min(widths) < LL // npx
    check_decomposition(case, npx, 1, nsteps=3)
    parts, _ = run_decomposed(case, npx, 1, 1, fields=("zeta",), probe=lambda m: m.halo_exchanges())
    assert {p[5][1] for p in parts} == {k_taken}, (widths, [p[5] for p in parts])


def test_fast_loop_exchange_count(monkeypatch):
    """Exchanges per whole step on a 2x2 grid: one per fast step at K = 1;
    with K > 1 one per K fast steps plus the start-of-loop swap of the fast
    step's other inputs, and nothing else changes."""
    case = _case("basin")
    got = {}
    for k in ("1", "2", "3", "4"):
        monkeypatch.setenv("ROMS_GPU_S2D_K", k)
        parts, _ = run_decomposed(case, 2, 2, 2, fields=("zeta",), probe=lambda m: m.halo_exchanges() + (m.t.nfast,))
        counts = {p[5] for p in parts}
        assert len(counts) == 1, counts   # every rank enqueues the same exchanges
        got[int(k)] = counts.pop()
    n1, k1, nfast = got[1]
    assert k1 == 1 and nfast > 8
    for k in (2, 3, 4):
        nk, kk, _ = got[k]
        assert kk == k
        assert nk == n1 - nfast + (nfast + k - 1) // k + 1, (k, nk, n1, nfast)
    print("exchanges per step (K: count):", {k: v[0] for k, v in got.items()}, "nfast", nfast)


def test_filament_3x2_matches_golden_digits():
    """The reference's Filament benchmark runs on a 3x2 MPI grid; with the
    same per-rank pairwise sums and tree over ranks the GPU run prints the
    golden log's ES23.16 digits."""
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "filament_github_gnu.json")))["rows"]
    case = dict(case_id=0, LLm=64, MMm=64, N=32, NT=1, salinity=False, nonlin_eos=False, dt=5.0, ndtfast=60,
                sizex=12.8e3, sizey=3.2e3)
    _, norms = run_decomposed(case, 3, 2, 20, fields=("zeta",), diag=True)
    assert len(norms) == 21
    bad = []
    for s, (r, g) in enumerate(zip(gold, norms)):
        want = [r["ke"], r["ke2b"], r["cu_adv"], r["cu_w"]]
        have = [("%23.16E" % v).strip() for v in g]
        if want != have:
            bad.append((s, want, have))
    assert not bad, bad[:3]


def test_pipes_ana_3x2_within_compiler_spread():
    """Pipes_ana (KPP, land mask, pipe) on the reference's 3x2 grid: every
    printed norm within the gfortran/ifx spread of the golden logs."""
    keys = ("ke", "ke2b", "cu_adv", "cu_w")
    gnu = json.load(open(os.path.join(ROOT, "tests", "golden", "pipes_ana_github_gnu.json")))["rows"]
    ifx = json.load(open(os.path.join(ROOT, "tests", "golden", "pipes_ana_github_ifx.json")))["rows"]
    spread = max(abs(float(x[k]) - float(g[k])) / abs(float(g[k])) for g, x in zip(gnu, ifx) for k in keys
                 if float(g[k]) != 0.0)
    case = dict(case_id=2, LLm=100, MMm=100, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                sizex=30e3, sizey=30e3, lmd=True)
    _, norms = run_decomposed(case, 3, 2, 20, fields=("zeta",), diag=True)
    assert len(norms) == 21
    assert [("%23.16E" % v).strip() for v in norms[0]] == [gnu[0][k] for k in keys]
    worst = max(abs(v - float(g[k])) / abs(float(g[k])) for g, n in zip(gnu, norms) for k, v in zip(keys, n)
                if float(g[k]) != 0.0)
    assert worst <= spread, (worst, spread)


def test_rivers_ana_3x2_within_compiler_spread():
    """Rivers_ana (river_frc.F analytic river, KPP, land mask) on the
    reference's 3x2 grid.  Its ana_grid.h fills 0..nx+1, 0..ny+1 of each rank
    and ANA_GRID exchanges nothing (grid.F:444-446), so the outer halo ring
    keeps its allocation values at the ranks' shared edges and the reference's
    result depends on its decomposition: the single-domain oracle drifts from
    the golden log after a few steps (tests/test_oracle_golden.py), while this
    run, decomposed like the reference, stays within the gnu/ifx spread."""
    keys = ("ke", "ke2b", "cu_adv", "cu_w")
    gnu = json.load(open(os.path.join(ROOT, "tests", "golden", "rivers_ana_github_gnu.json")))["rows"]
    ifx = json.load(open(os.path.join(ROOT, "tests", "golden", "rivers_ana_github_ifx.json")))["rows"]
    spread = max(abs(float(x[k]) - float(g[k])) / abs(float(g[k])) for g, x in zip(gnu, ifx) for k in keys
                 if float(g[k]) != 0.0)
    case = dict(case_id=3, LLm=100, MMm=100, N=10, NT=2, salinity=True, nonlin_eos=True, dt=20.0, ndtfast=30,
                sizex=10e3, sizey=10e3, lmd=True)
    _, norms = run_decomposed(case, 3, 2, 20, fields=("zeta",), diag=True)
    assert len(norms) == 21
    worst = max(abs(v - float(g[k])) / abs(float(g[k])) for g, n in zip(gnu, norms) for k, v in zip(keys, n)
                if float(g[k]) != 0.0)
    # measured: 4.3e-13 (step 1 MAX_VERT_CFL, equal to the ifx value) against a spread of 4.3e-13
    assert worst <= spread, (worst, spread)


RCCL_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
import numpy as np, romsgpu
case = dict(case_id=0, LLm=32, MMm=24, N=8, NT=1, dt=5.0, ndtfast=60, sizex=6.4e3, sizey=1.2e3)
m = romsgpu.Model.from_case(**case)
m.step(4)
ref = {f: m.get(f) for f in ("zeta", "u", "v", "t", "FlxU", "We")}
m.close()
uid = romsgpu.comm_unique_id()
h = romsgpu.comm_create(uid, 1, 0, 0)
m = romsgpu.Model.from_case(np_xi=1, np_eta=1, comm=h, rank=0, **case)
want = os.environ.get("ROMS_EXPECT_TRANSPORT")
if want:
    assert m.halo_transport() == want, m.halo_transport()
m.step(4)
if want:
    assert m.halo_transport() == want, m.halo_transport()   # no timed-out wait during the run
for f, v in ref.items():
    g = m.get(f)
    assert np.array_equal(g[..., 1:-1, 1:-1], v[..., 1:-1, 1:-1]), f
m.close()
romsgpu.comm_destroy(h)
print("RCCL_OK")
"""


@pytest.mark.parametrize("overlap,transport", [("0", "ipc"), ("1", "ipc"), ("0", "rccl")])
def test_rccl_transport_self_routed_equals_wrap(overlap, transport):
    """Single rank with a communicator: every exchange goes through the
    multi-rank transport (IPC peer writes to itself after the init self-test,
    or RCCL self-sends with ROMS_GPU_HALO_IPC=0), graph-captured; fields equal
    the on-device periodic wrap bitwise."""
    env = dict(os.environ, ROMS_GPU_RCCL_SELF="1", ROMS_GPU_S2D_OVERLAP=overlap, ROMS_EXPECT_TRANSPORT=transport,
               ROMS_GPU_HALO_IPC="1" if transport == "ipc" else "0")
    r = subprocess.run([sys.executable, "-c", RCCL_SCRIPT, ROOT], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_rim_first_overlap_bitwise_equals_serial_exchanges():
    """launch_rim_first (rim strips, exchange forked on the halo stream, interior
    concurrently; omega, set_HUV, step3d_t, t3dmix) gives the same fields as
    the serial exchange order (the default; ROMS_GPU_OVERLAP3D=1 turns the
    overlap on) on a 2x2 grid."""
    case = _case("basin_lmd")
    serial, _ = run_decomposed(case, 2, 2, 6)
    os.environ["ROMS_GPU_OVERLAP3D"] = "1"
    try:
        over, _ = run_decomposed(case, 2, 2, 6)
    finally:
        del os.environ["ROMS_GPU_OVERLAP3D"]
    for r in range(4):
        for f in FIELDS:
            assert np.array_equal(serial[r][4][f], over[r][4][f]), (r, f)


# The deferred-exchange checks run in a child process with 16 hardware
# queues (GPU_MAX_HW_QUEUES; HIP's default of 4 is shared by every rank's
# library and halo streams here, and streams that share a hardware queue run
# in submission order, which would join every exchange by accident).
DEFER_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import test_gpu_multirank as mr
try:
    mr.check_decomposition(mr._case(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
except AssertionError as e:
    print("MISMATCH", str(e)[:400])
    raise SystemExit(3)
print("BITWISE")
"""


def _deferred(kind, npx, npe, env):
    e = dict(os.environ, GPU_MAX_HW_QUEUES="16", ROMS_GPU_XOVERLAP="1", **env)
    r = subprocess.run([sys.executable, "-c", DEFER_SCRIPT, ROOT, kind, str(npx), str(npe)], env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode in (0, 3), (r.returncode, r.stdout[-1500:], r.stderr[-3000:])
    return r.returncode == 0, r.stdout


@pytest.mark.parametrize("kind", ["basin_lmd", "filament", "basin_flux", "pipes"])
@pytest.mark.parametrize("npx,npe", [(2, 1), (2, 2)])
def test_deferred_exchanges_late_unpack_bitwise(kind, npx, npe):
    """Deferred 3-D exchanges (ROMS_GPU_XOVERLAP=1, opt-in):
    set_HUV's beside lmd_vmix(nstp), omega's and lmd_vmix's beside prsgrd,
    pre_step3d's tracer swap beside set_HUV1, set_HUV1's beside rho_eos(nrhs),
    the corrector's omega and lmd_vmix beside prsgrd, the closing omega's
    beside step3d_t.  With every forked exchange's unpack held back 300 us
    (ROMS_GPU_XDELAY_US) a routine that reads a halo before its join would
    read the previous step's values: the subdomains still equal the single
    domain bitwise."""
    ok, out = _deferred(kind, npx, npe, {"ROMS_GPU_XDELAY_US": "300"})
    assert ok, out[-1500:]


def test_deferred_exchanges_off_equals_on():
    """The default (every exchange in place, the reference's order) and the
    deferred order (ROMS_GPU_XOVERLAP=1) give the same fields bitwise."""
    case = _case("basin_lmd")
    off, _ = run_decomposed(case, 2, 2, 5)
    os.environ["ROMS_GPU_XOVERLAP"] = "1"
    try:
        on, _ = run_decomposed(case, 2, 2, 5)
    finally:
        del os.environ["ROMS_GPU_XOVERLAP"]
    for r in range(4):
        for f in FIELDS:
            assert np.array_equal(on[r][4][f], off[r][4][f]), (r, f)


@pytest.mark.parametrize("bit,kind,reader", [(1, "basin", "omega (predictor)"), (8, "basin_flux", "omega (corrector)"),
                                             (16, "basin_flux", "step3d_uv1")])
def test_deferred_exchange_missing_join_is_detected(bit, kind, reader):
    """The delay hook is a real check: with one join left out (test hook
    ROMS_GPU_XTEST_SKIPJOIN=bit) the routine after it reads a halo before the
    late unpack -- whose destination the hook first sets to NaN, so even a
    stale value equal to the fresh one shows -- and the decomposition no
    longer matches.  In process, the joins of the last exchange forked before
    their reader show this way; the in-process transport's host wait inside
    each exchange completes the earlier ones (bits 2 and 4, and bit 1 when
    lmd_vmix's exchange is forked between set_HUV's and omega), so
    tests/test_gpu_ipc.py::test_processes_missing_join_is_detected shows all
    five joins across processes, where no host wait intervenes."""
    ok, out = _deferred(kind, 2, 1, {"ROMS_GPU_XDELAY_US": "2000", "ROMS_GPU_XTEST_SKIPJOIN": str(bit)})
    assert not ok, out[-1500:]
    ok, out = _deferred(kind, 2, 1, {"ROMS_GPU_XDELAY_US": "2000"})
    assert ok, out[-1500:]
