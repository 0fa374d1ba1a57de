"""Per-kernel table from any number of rocprofv3 --pmc passes (counter_collection
CSVs) plus an optional kernel trace: mean counter value per dispatch, HBM
traffic = 2*FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md gfx950 note), and the
SQ cycle split (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as % of
WAVE_CYCLES) when those counters are present.
usage: python tools/pmc_table.py CSV [CSV ...] [--trace kernel_trace.csv] [--top 30]
"""
import argparse
import collections
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("roms::", "")[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for p in a.csvs:
        for r in csv.DictReader(open(p)):
            k, c = short(r["Kernel_Name"]), r["Counter_Name"]
            val[k][c] += float(r["Counter_Value"])
            cnt[k][c] += 1
    dur = collections.defaultdict(list)
    if a.trace:
        for r in csv.DictReader(open(a.trace)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k in val:
        m = {c: val[k][c] / cnt[k][c] for c in val[k]}
        d = dur.get(k)
        us = sorted(d)[len(d) // 2] if d else float("nan")
        calls = len(d) if d else max(cnt[k].values())
        tr = None
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            tr = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024.0 / 1e6
        rows.append((k, calls, us, tr, m))
    # by time per step (trace) or, without one, by wave cycles over all dispatches
    rows.sort(key=lambda r: -(r[2] * r[1] if r[2] == r[2] else r[4].get("SQ_WAVE_CYCLES", 0.0) * r[1]))
    print("%-40s %6s %9s %9s %7s %6s %6s %6s %7s %7s %7s %6s %7s %6s" % (
        "kernel", "calls", "us/call", "trafMB", "GB/s", "wait%", "stall%", "actv%", "valu/w", "salu/w", "vmem/w",
        "lds%", "waves", "L2hit"))
    for k, calls, us, tr, m in rows[:a.top]:
        wc = m.get("SQ_WAVE_CYCLES")
        pct = lambda c: (100.0 * m[c] / wc) if (wc and c in m) else float("nan")
        waves = m.get("SQ_WAVES", float("nan"))
        vpw = m["SQ_INSTS_VALU"] / waves if ("SQ_INSTS_VALU" in m and waves == waves and waves) else float("nan")
        gbs = tr / us * 1e3 if (tr is not None and us == us) else float("nan")
        hit = m.get("TCC_HIT_sum"); miss = m.get("TCC_MISS_sum")
        l2 = 100.0 * hit / (hit + miss) if (hit is not None and miss is not None and hit + miss) else float("nan")
        per = lambda c: m[c] / waves if (c in m and waves == waves and waves) else float("nan")
        vmem = per("SQ_INSTS_VMEM_RD") + (per("SQ_INSTS_VMEM_WR") if "SQ_INSTS_VMEM_WR" in m else 0.0)
        print("%-40s %6d %9.1f %9s %7.0f %6.1f %6.1f %6.1f %7.0f %7.0f %7.0f %6.1f %7.0f %6.1f" % (
            k, calls, us, "%.1f" % tr if tr is not None else "-", gbs, pct("SQ_WAIT_ANY"), pct("SQ_WAIT_INST_ANY"),
            pct("SQ_ACTIVE_INST_ANY"), vpw, per("SQ_INSTS_SALU"), vmem, pct("SQ_WAIT_INST_LDS"), waves, l2))


if __name__ == "__main__":
    main()
