"""ISA census of the HIP kernels (gfx950): per kernel, the patterns that make
a wave pay a full memory round trip where the source meant to overlap loads.

  loads / waits    vector-memory loads and `s_waitcnt vmcnt` instructions
  load->wait0      a load followed within a few instructions by vmcnt(0):
                   the load's latency is not hidden (a scan with one load per
                   iteration, or a load the compiler sank into a branch)
  wait0->store     vmcnt(0) right before a store: the wave waits for every
                   earlier store (vmcnt counts stores too on gfx950)
  waterfall        readfirstlane loops: an SGPR operand (a buffer soffset)
                   that differs between lanes

Counts are static (instructions in the ISA), so a site inside a branch that
a configuration never takes (pipes, rivers, open edges) counts as well; read
the site before acting on it.  Round 5 used this to find the KPP depth scans
and the tracer corrector's KPP-term loads and row stores.

usage: python tools/isa_census.py [KERNEL_REGEX] > profiles/rN_isa_census.txt
"""
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "ucla-roms_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-function", "-Wno-unused-variable"]
LOAD = ("buffer_load", "global_load")
STORE = ("buffer_store", "global_store")


def kernels(asm):
    lines = asm.split("\n")
    starts = [(i, m.group(1)) for i, l in enumerate(lines) for m in [re.match(r"^(_Z\S+):", l)] if m]
    for n, (st, name) in enumerate(starts):
        en = starts[n + 1][0] if n + 1 < len(starts) else len(lines)
        yield name, [l.strip() for l in lines[st:en]]


def census(body):
    loads = sum(1 for l in body if l.startswith(LOAD))
    waits = sum(1 for l in body if l.startswith("s_waitcnt") and "vmcnt" in l)
    lw0 = sum(1 for i, l in enumerate(body)
              if l.startswith(LOAD) and any("vmcnt(0)" in x for x in body[i + 1:i + 6]))
    w0s = sum(1 for i, l in enumerate(body)
              if l.startswith(STORE) and i > 0 and "vmcnt(0)" in body[i - 1])
    wf = sum(1 for i, l in enumerate(body)
             if l.startswith("v_readfirstlane_b32") and any(x.startswith("v_cmp_eq_u32") for x in body[i + 1:i + 3]))
    return loads, waits, lw0, w0s, wf


def main():
    pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
    print("%-72s %6s %6s %11s %12s %9s" % ("kernel (gfx950)", "loads", "waits", "load->wait0", "wait0->store",
                                           "waterfall"))
    with tempfile.TemporaryDirectory() as td:
        for f in sorted(os.listdir(SRC)):
            if not f.endswith(".hip"):
                continue
            out = os.path.join(td, f + ".s")
            r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + FLAGS +
                               ["--cuda-device-only", "-S", os.path.join(SRC, f), "-o", out],
                               capture_output=True, text=True, cwd=SRC)
            if r.returncode != 0:
                print("# %s: compile failed" % f)
                continue
            for name, body in kernels(open(out).read()):
                dem = subprocess.run(["c++filt", name], capture_output=True,
                                     text=True).stdout.strip()
                short = re.sub(r"\(.*", "", dem.replace("roms::", "").replace("(anonymous namespace)::", ""))
                if pat and not pat.search(short):
                    continue
                print("%-72s %6d %6d %11d %12d %9d" % ((short[:72],) + census(body)))


if __name__ == "__main__":
    main()
