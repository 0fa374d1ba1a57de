"""Register / LDS / spill table of every kernel of libromsgpu (gfx950), from
hipcc -Rpass-analysis=kernel-resource-usage over each HIP source, with the
Makefile's flags.  usage: python tools/resource_usage.py [PATTERN] > profiles/rN_resource_usage.txt"""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "ucla-roms_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only", "-c"]
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
print("%-64s %5s %5s %6s %6s %7s %4s %7s" % ("kernel (gfx950)", "VGPR", "SGPR", "sSpill", "vSpill", "scratch", "occ",
                                               "LDS"))
for f in sorted(os.listdir(SRC)):
    if not f.endswith(".hip"):
        continue
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + [os.path.join(SRC, f), "-o", "/tmp/_ru.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd=SRC)
    cur, d = None, {}
    for ln in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = m.group(1)
            d[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\d+)", ln)
        if m and cur:
            d[cur][m.group(1).strip()] = int(m.group(2))
    for k, v in d.items():
        if pat and not pat.search(k):
            continue
        name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        name = name.replace("(anonymous namespace)::", "").replace("roms::", "").split("(")[0].replace("void ", "")
        print("%-64s %5d %5d %6d %6d %7d %4d %7d" % (name[:64], v.get("VGPRs", 0), v.get("TotalSGPRs", v.get("SGPRs", 0)),
                                                   v.get("SGPRs Spill", 0), v.get("VGPRs Spill", 0),
                                                   v.get("ScratchSize [bytes/lane]", 0),
                                                   v.get("Occupancy [waves/SIMD]", 0), v.get("LDS Size [bytes/block]", 0)))
