"""Multi-process halo transports on one GPU (mpi_exchanges.F semantics over
one process per subdomain, the layout of the 8-GPU runs).

  * two processes, one communicator (RCCL bootstrap through a file), 2x1
    Filament and open-basin grids: the IPC transport (hipIpcOpenMemHandle of
    the other process's receive buffers, the code path the 8-GPU node uses
    across xGMI) and the RCCL transport both reproduce the single-domain run
    bitwise;
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
rank, uidf, kind = int(sys.argv[2]), sys.argv[3], sys.argv[4]
if kind == "filament":
    case = dict(case_id=0, LLm=40, MMm=24, N=8, NT=1, dt=5.0, ndtfast=60, sizex=4.0e3, sizey=0.6e3)
else:
    case = dict(case_id=1, LLm=36, MMm=28, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
                sizex=72e3, sizey=56e3, lmd=romsgpu.LMD_ICELAND, obc=15, island=True, curvgrid=True)
fields = ("zeta", "ubar", "vbar", "u", "v", "t", "FlxU", "We", "Hz")
m = romsgpu.Model.from_case(**case)
m.step(5)
ref = {f: m.get(f) for f in fields}
m.close()
if rank == 0:
    with open(uidf + ".tmp", "wb") as fh:
        fh.write(romsgpu.comm_unique_id())
    os.rename(uidf + ".tmp", uidf)
t0 = time.time()
while not os.path.exists(uidf):
    if time.time() - t0 > 60:
        raise SystemExit("no unique id")
    time.sleep(0.05)
uid = open(uidf, "rb").read()
try:
    h = romsgpu.comm_create(uid, 2, rank, 0)
except romsgpu.RomsGpuError as e:
    print("COMM_FAIL", e)
    raise SystemExit(3)
m = romsgpu.Model.from_case(np_xi=2, np_eta=1, comm=h, rank=rank, **case)
tr = m.halo_transport()
m.step(5)
m.sync()
iSW, Lm, Mm = m.iSW, m.Lm, m.Mm
bad = []
for f in fields:
    g = m.get(f)
    w = ref[f][..., 0:Mm + 4, iSW:iSW + Lm + 4]
    if not np.array_equal(g[..., 1:-1, 1:-1], w[..., 1:-1, 1:-1]):
        bad.append((f, float(np.max(np.abs(g[..., 1:-1, 1:-1] - w[..., 1:-1, 1:-1])))))
m.close()
romsgpu.comm_destroy(h)
print("TRANSPORT", tr)
print("BAD", bad)
raise SystemExit(1 if bad else 0)
"""


def _two_ranks(kind, ipc):
    env = dict(os.environ, ROMS_GPU_HALO_IPC="1" if ipc else "0")
    with tempfile.TemporaryDirectory() as td:
        uidf = os.path.join(td, "uid")
        ps = [subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, ROOT, str(r), uidf, kind], env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = []
        for p in ps:
            try:
                o, e = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in ps:
                    q.kill()
                raise
            outs.append((p.returncode, o, e))
    if any(rc == 3 for rc, _, _ in outs):
        pytest.skip("RCCL refused two ranks on one GPU: %s" % outs[0][1][-300:])
    for rc, o, e in outs:
        assert rc == 0, (rc, o[-2000:], e[-3000:])
        assert ("TRANSPORT %s" % ("ipc" if ipc else "rccl")) in o, o
    return outs


@pytest.mark.parametrize("kind", ["filament", "basin_obc"])
@pytest.mark.parametrize("ipc", [True, False], ids=["ipc", "rccl"])
def test_two_processes_one_gpu_bitwise(kind, ipc):
    _two_ranks(kind, ipc)


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
