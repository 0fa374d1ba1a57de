"""Per-kernel mean of every counter in one or more rocprofv3 counter_collection.csv
files (one PMC pass each), printed as a table; optional ratio columns.
usage: python tools/pmc_generic.py pass1.csv pass2.csv ... [--kernels k1,k2]
"""
import argparse
import collections
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("roms::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernels", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.Counter())
    names = []
    for p in a.csv:
        for r in csv.DictReader(open(p)):
            k, c = short(r["Kernel_Name"]), r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            cnt[k][c] += 1
            if c not in names:
                names.append(c)
    want = [x for x in a.kernels.split(",") if x]
    ks = [k for k in tot if not want or any(w in k for w in want)]
    ks.sort(key=lambda k: -sum(tot[k].values()))
    print("%-28s " % "kernel" + " ".join("%16s" % n[:16] for n in names) + "  L2hit%")
    for k in ks:
        vals = [tot[k][n] / max(cnt[k][n], 1) for n in names]
        h, m = tot[k].get("TCC_HIT_sum"), tot[k].get("TCC_MISS_sum")
        hr = 100.0 * h / (h + m) if h is not None and m is not None and h + m > 0 else float("nan")
        print("%-28s " % k[:28] + " ".join("%16.4g" % v for v in vals) + "  %5.1f" % hr)


if __name__ == "__main__":
    main()
