"""Multi-process halo transport on one GPU (mpi_exchanges.F semantics over
one process per subdomain, the layout of the 8-GPU runs).

  * 2 and 4 processes, one host-channel communicator each
    (roms_gpu_comm_create_host: the processes' own allgather -- here through
    files, MPI_Allgather in a Fortran host -- carries the IPC handles at init
    and the diag gathers; RCCL is not involved): every halo exchange is an
    IPC peer write into the other process's receive buffer
    (hipIpcOpenMemHandle, cross-process arrival counters with system-scope
    release/acquire), the code path the 8-GPU node uses across xGMI.  Filament
    and the open basin, 2x1 and 2x2, reproduce the single-domain run bitwise,
    with the step graphs replaying the IPC kernels.
  * RCCL itself refuses two ranks on one GPU (its duplicate-device check), so
    the RCCL transport is covered self-routed on one process
    (test_gpu_multirank.py::test_rccl_transport_self_routed_equals_wrap).
  * a halo wait that never completes is fatal: with the test hook
    ROMS_GPU_IPC_TEST_DROP one exchange does not signal, the wait gives up
    after ROMS_GPU_IPC_TIMEOUT seconds and every later entry fails with
    "timed out" instead of computing on stale halos (halo.hip).
"""
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = r"""
import os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
import numpy as np, romsgpu
rank, chan, kind, npx, npe = int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
if kind == "filament":
    case = dict(case_id=0, LLm=40, MMm=24, N=8, NT=1, dt=5.0, ndtfast=60, sizex=4.0e3, sizey=0.6e3)
else:
    case = dict(case_id=1, LLm=36, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                sizex=72e3, sizey=56e3, lmd=romsgpu.LMD_ICELAND, obc=15, island=True, curvgrid=True)
fields = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "We", "Hz")
m = romsgpu.Model.from_case(**case)
m.step(5)
ref = {f: m.get(f) for f in fields}
norms_ref = m.diag()
m.close()
ag = romsgpu.FileAllgather(chan, npx * npe, rank)
h = romsgpu.comm_create_host(npx * npe, rank, ag)
m = romsgpu.Model.from_case(np_xi=npx, np_eta=npe, comm=h, rank=rank, **case)
tr = m.halo_transport()
m.step(5)
norms = m.diag()   # collective through the host channel
m.sync()
iSW, jSW, Lm, Mm = m.iSW, m.jSW, m.Lm, m.Mm
bad = []
for f in fields:
    g = m.get(f)
    w = ref[f][..., jSW:jSW + Mm + 4, iSW:iSW + Lm + 4]
    if not np.array_equal(g[..., 1:-1, 1:-1], w[..., 1:-1, 1:-1]):
        bad.append((f, float(np.max(np.abs(g[..., 1:-1, 1:-1] - w[..., 1:-1, 1:-1])))))
tr_end = m.halo_transport()
m.close()
romsgpu.comm_destroy(h)
print("TRANSPORT", tr, tr_end)
print("NORMS", max(abs(a - b) / max(abs(b), 1e-300) for a, b in zip(norms, norms_ref)))
print("BAD", bad)
raise SystemExit(1 if bad else 0)
"""


def _ranks(kind, npx, npe, env=None):
    with tempfile.TemporaryDirectory() as td:
        ps = [subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, ROOT, str(r), td, kind, str(npx), str(npe)],
                               env=dict(os.environ, **(env or {})), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True)
              for r in range(npx * npe)]
        outs = []
        for p in ps:
            try:
                o, e = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in ps:
                    q.kill()
                raise
            outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, (rc, o[-2000:], e[-3000:])
        assert "TRANSPORT ipc ipc" in o, o
        # diag's tree over ranks sums in another order than one domain: reduction noise only
        nerr = float(o.split("NORMS")[1].split()[0])
        assert nerr < 1e-12, o
    return outs


@pytest.mark.parametrize("kind", ["filament", "basin_obc"])
@pytest.mark.parametrize("npx,npe", [(2, 1), (2, 2)])
def test_processes_one_gpu_ipc_host_channel_bitwise(kind, npx, npe):
    _ranks(kind, npx, npe)


@pytest.mark.parametrize("kind", ["filament", "basin_obc"])
def test_processes_deferred_exchanges_ipc_bitwise(kind):
    """The deferred 3-D exchanges (ROMS_GPU_XOVERLAP=1) between processes:
    the IPC pack / wait / unpack kernels on each rank's halo stream beside
    the next routine, graph-captured, with every unpack held back 300 us; the
    2x2 subdomains still equal the single domain."""
    _ranks(kind, 2, 2, {"ROMS_GPU_XOVERLAP": "1", "ROMS_GPU_XDELAY_US": "300"})


SKIP_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
import numpy as np, romsgpu
rank, chan, npx, npe = int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
case = dict(case_id=1, LLm=36, MMm=28, N=20, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
            sizex=72e3, sizey=56e3, lmd=True, surf_flux=True)
fields = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "FlxV", "We", "Wi", "Hz", "Akv", "Akt")
m = romsgpu.Model.from_case(**case)
m.step(4)
ref = {f: m.get(f) for f in fields}
m.close()
ag = romsgpu.FileAllgather(chan, npx * npe, rank)
h = romsgpu.comm_create_host(npx * npe, rank, ag)
m = romsgpu.Model.from_case(np_xi=npx, np_eta=npe, comm=h, rank=rank, **case)
assert m.halo_overlap(), "deferred exchanges expected on"
m.step(4)
m.sync()
iSW, jSW, Lm, Mm = m.iSW, m.jSW, m.Lm, m.Mm
bad = []
for f in fields:
    g = m.get(f)
    w = ref[f][..., jSW:jSW + Mm + 4, iSW:iSW + Lm + 4]
    if not np.array_equal(g[..., 2:-2, 2:-2], w[..., 2:-2, 2:-2]):
        bad.append(f)
m.close()
romsgpu.comm_destroy(h)
print("BAD", bad)
"""


def _skip_ranks(npx, npe, env):
    """Every rank's BAD list (owned cells that differ from the single domain)."""
    with tempfile.TemporaryDirectory() as td:
        ps = [subprocess.Popen([sys.executable, "-c", SKIP_SCRIPT, ROOT, str(r), td, str(npx), str(npe)],
                               env=dict(os.environ, **env), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for r in range(npx * npe)]
        outs = []
        for p in ps:
            try:
                o, e = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in ps:
                    q.kill()
                raise
            outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0 and "BAD" in o, (rc, o[-2000:], e[-3000:])
    return [o.split("BAD", 1)[1].strip() for _, o, _ in outs]


@pytest.mark.parametrize("bit,reader", [(1, "omega (predictor)"), (2, "pre_step3d"), (4, "rho_eos (corrector)"),
                                        (8, "omega (corrector)"), (16, "step3d_uv1")])
def test_processes_missing_join_is_detected(bit, reader):
    """Each join of the deferred order guards a real read (ADVICE/VERDICT r5):
    with one join left out (ROMS_GPU_XTEST_SKIPJOIN=bit) and every deferred
    exchange's destination halo set to NaN before its held-back unpack
    (ROMS_GPU_XDELAY_US), the routine after the missing join reads NaN and the
    owned cells no longer equal the single domain -- for every one of the
    five joins.  Across processes no host wait completes an earlier exchange
    early (the in-process transport's do), and the NaN shows a stale read even
    where stale and fresh halos agree.  The same run with every join kept is
    bitwise."""
    base = {"ROMS_GPU_XOVERLAP": "1", "ROMS_GPU_XDELAY_US": "2000", "GPU_MAX_HW_QUEUES": "16"}
    bad = _skip_ranks(2, 1, dict(base, ROMS_GPU_XTEST_SKIPJOIN=str(bit)))
    assert any(b != "[]" for b in bad), (reader, bad)
    good = _skip_ranks(2, 1, base)
    assert all(b == "[]" for b in good), good


FATAL_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
import romsgpu
case = dict(case_id=0, LLm=32, MMm=24, N=8, NT=1, dt=5.0, ndtfast=60, sizex=6.4e3, sizey=1.2e3)
h = romsgpu.comm_create(romsgpu.comm_unique_id(), 1, 0, 0)
m = romsgpu.Model.from_case(np_xi=1, np_eta=1, comm=h, rank=0, **case)
assert m.halo_transport() == "ipc", m.halo_transport()
try:
    for _ in range(6):
        m.step()
    m.sync()
except romsgpu.RomsGpuError as e:
    print("FATAL_OK", e)
    assert m.halo_transport() == "ipc-timeout"
    raise SystemExit(0)
raise SystemExit("a dropped halo message went unnoticed")
"""


def test_ipc_wait_timeout_is_fatal():
    env = dict(os.environ, ROMS_GPU_RCCL_SELF="1", ROMS_GPU_HALO_IPC="1", ROMS_GPU_NO_GRAPH="1",
               ROMS_GPU_IPC_TIMEOUT="0.5", ROMS_GPU_IPC_TEST_DROP="40")
    r = subprocess.run([sys.executable, "-c", FATAL_SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "FATAL_OK" in r.stdout and "timed out" in r.stdout, (r.returncode, r.stdout[-2000:],
                                                                                     r.stderr[-3000:])
