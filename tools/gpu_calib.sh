#!/bin/bash
# PMC calibration passes for tools/pmc_calib (run on the box).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/pmc_calib > $O/calib_plain.txt 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_f -o run -- $R/tools/pmc_calib > $O/calib_f.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_w -o run -- $R/tools/pmc_calib > $O/calib_w.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/calib_h -o run -- $R/tools/pmc_calib > $O/calib_h.log 2>&1 || exit $?
cat $O/calib_plain.txt
for f in $O/calib_f $O/calib_w $O/calib_h; do
  python3 - "$f" <<'PY'
import csv, glob, sys, collections
p = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(p)):
    agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print("%-12s %-14s %s" % (k, c, " ".join("%.4g" % x for x in v)))
PY
done
