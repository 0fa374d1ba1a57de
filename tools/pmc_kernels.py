"""Per-kernel HBM traffic (2*FETCH_SIZE + WRITE_SIZE, calibrated for our 8-B
and 16-B per-lane accesses by tools/pmc_calib.hip) and, when a kernel trace is
given, mean duration and achieved traffic bandwidth.
usage: python tools/pmc_kernels.py FETCH.csv WRITE.csv [--trace kernel_trace.csv]
"""
import argparse
import collections
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("roms::", "")


def read(path, counter):
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") == counter:
            k = short(r["Kernel_Name"])
            tot[k] += float(r["Counter_Value"]) * 1024.0
            cnt[k] += 1
    return tot, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--trace")
    a = ap.parse_args()
    f, fc = read(a.fetch, "FETCH_SIZE")
    w, wc = read(a.write, "WRITE_SIZE")
    dur = collections.defaultdict(list)
    if a.trace:
        for r in csv.DictReader(open(a.trace)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("%-32s %6s %10s %10s %10s %9s %8s" % ("kernel", "calls", "fetchMB", "writeMB", "trafficMB", "us/call", "GB/s"))
    rows = []
    for k in f:
        fm = 2 * f[k] / fc[k] / 1e6
        wm = w.get(k, 0.0) / max(wc.get(k, 1), 1) / 1e6
        d = dur.get(k)
        us = sorted(d)[len(d) // 2] if d else float("nan")
        rows.append((k, fc[k], fm, wm, fm + wm, us, (fm + wm) / us * 1e-3 * 1e3 if d else float("nan")))
    for r in sorted(rows, key=lambda r: -r[4] * r[1]):
        print("%-32s %6d %10.1f %10.1f %10.1f %9.1f %8.0f" % r)


if __name__ == "__main__":
    main()
