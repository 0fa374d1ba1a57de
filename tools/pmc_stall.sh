#!/bin/bash
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/pmc_s2d -o run -- python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 --steps 3 --warmup 1 > $O/pmc_s2d.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --output-format csv -d $O/pmc_s2d2 -o run -- python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 --steps 3 --warmup 1 > $O/pmc_s2d2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ("pmc_s2d", "pmc_s2d2"):
    f = glob.glob("/root/repo/gpurun_out/%s/**/*counter_collection.csv" % d, recursive=True)
    tot = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k in ("k_s2d_fb", "k_prsgrd_uv", "k_uv1", "k_pre_uv", "k_omega_seg", "k_pre_tracer_h1"):
        if k in tot:
            n = max(cnt[(k, c)] for c in tot[k])
            print(d, k, "dispatches", n, " ".join("%s=%.3g" % (c, v / n) for c, v in sorted(tot[k].items())))
PY
