"""Cross-process IPC halo transport on one GPU: 2 ranks (2x1) of a C2-like
periodic domain (per rank LxLx50, NT=2), host-channel communicator (file
allgather), ms/step with the current environment (ROMS_GPU_OVERLAP3D,
ROMS_GPU_S2D_OVERLAP).  Both ranks share the one GPU, so this measures the
IPC path and the overlap mechanics, not xGMI.
usage: python tools/ipc_overlap_ab.py [L]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK = r"""
import os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "ucla-roms_amd"))
import romsgpu
rank, chan, L = int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
ag = romsgpu.FileAllgather(chan, 2, rank)
h = romsgpu.comm_create_host(2, rank, ag)
m = romsgpu.Model.from_case(0, 2 * L, L, 50, 2, salinity=True, dt=5.0, ndtfast=60, sizex=100.0 * 2 * L,
                            sizey=25.0 * L, np_xi=2, np_eta=1, comm=h, rank=rank)
m.step(3)
m.sync()
ms = m.time_steps(10)
print("RANK", rank, m.halo_transport(), "%.3f" % (ms / 10), flush=True)
m.close()
romsgpu.comm_destroy(h)
"""


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    with tempfile.TemporaryDirectory() as td:
        ps = [subprocess.Popen([sys.executable, "-c", RANK, ROOT, str(r), td, str(L)], stdout=subprocess.PIPE,
                               text=True) for r in range(2)]
        outs = [p.communicate(timeout=300)[0] for p in ps]
    ms = [float(o.split()[-1]) for o in outs]
    print("env OVERLAP3D=%s S2D_OVERLAP=%s: %s -> max %.3f ms/step" % (
        os.environ.get("ROMS_GPU_OVERLAP3D", "0"), os.environ.get("ROMS_GPU_S2D_OVERLAP", "0"),
        " | ".join(o.strip() for o in outs), max(ms)))


if __name__ == "__main__":
    main()
