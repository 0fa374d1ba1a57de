"""Print the routine table of bench JSON lines (usage: python tools/bench_table.py a.json [b.json ...])."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("%s: value %.3e ms/step %.2f model-s/s %.1f step-roofline %.1f%%" % (
        f, d["value"], d["ms_per_step"], d["model_seconds_per_wallclock_sec"], 100 * d["roofline_step"]["frac"]))
    for r, v in sorted(d["routines"].items(), key=lambda x: -x[1]["ms_per_step"]):
        print("  %-11s %7.3f ms/step %5.1f calls %6.0f GB/s %4.1f%%" % (
            r, v["ms_per_step"], v["calls_per_step"], v["achieved_GBs"], 100 * v["frac"]))
