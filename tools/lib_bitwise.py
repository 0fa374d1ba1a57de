"""Bitwise regression between two builds of libromsgpu.so (GPU box).

Each case runs a few whole steps in a child process per library (the library
is chosen by ROMS_GPU_LIB when romsgpu is imported) and the prognostic and
diagnostic fields of both runs are compared bit for bit.  For changes that
keep every expression and its order (buffer addressing, register forwarding)
while replacing a kernel in place, where no environment switch can select the
old form any more.

usage: python tools/lib_bitwise.py LIB_A LIB_B [steps]
       (tools/build_rev.sh REV TAG builds LIB_A from an earlier revision)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/oracle", sys.argv[1] + "/ucla-roms_amd", sys.argv[1] + "/tests"]
import oracle, romsgpu
case, steps, out = sys.argv[2], int(sys.argv[3]), sys.argv[4]
c = oracle.OrCfg()
if case.startswith("filament"):
    c = oracle.filament_cfg(LLm=64, MMm=48, N=16, np_xi=1, np_eta=1)
    lmd, sf = 0, False
else:
    N = int(case.split("_n")[1])
    c.LLm, c.MMm, c.N, c.NT = 64, 48, N, 2
    c.ew_periodic = c.ns_periodic = 0
    c.salinity, c.nonlin_eos = 1, int("linear" not in case)
    c.case_id = oracle.CASE_BASIN
    c.dt, c.ndtfast = 60.0, 30
    c.sizex, c.sizey = 96e3, 80e3
    lmd, sf = oracle.LMD_ALL, True
m = romsgpu.Model.from_case(c.case_id, c.LLm, c.MMm, c.N, c.NT, salinity=bool(c.salinity),
                            nonlin_eos=bool(c.nonlin_eos), dt=c.dt, ndtfast=c.ndtfast, sizex=c.sizex,
                            sizey=c.sizey, lmd=lmd, surf_flux=sf)
m.step(steps)
names = ["zeta", "ubar", "vbar", "u", "v", "t", "rufrc", "rvfrc", "FlxU", "FlxV", "We", "Wi", "Akv", "Akt",
         "hbls", "hbbl", "rho1", "qp1", "bvf"]
got = {}
for n in names:
    try:
        got[n] = m.get(n)
    except Exception:
        pass
m.close()
np.savez(out, **got)
"""
CASES = ["basin_lmd_n100", "basin_lmd_n50", "basin_linear_lmd_n20", "filament"]


def run(lib, case, steps, out):
    env = dict(os.environ, ROMS_GPU_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CHILD, R, case, str(steps), out], env=env, capture_output=True,
                       text=True, timeout=300)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:])
        raise SystemExit("child failed: %s %s" % (lib, case))


def main():
    a, b = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for case in CASES:
            fa, fb = os.path.join(td, "a_%s.npz" % case), os.path.join(td, "b_%s.npz" % case)
            run(a, case, steps, fa)
            run(b, case, steps, fb)
            za, zb = np.load(fa), np.load(fb)
            diff = [n for n in za.files if n in zb.files and not np.array_equal(za[n], zb[n])]
            print("%-22s %d fields compared, %s" % (case, len(za.files), "bitwise equal" if not diff else
                                                    "DIFFER: " + " ".join(diff)))
            bad += len(diff)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
