"""Per-step kernel-time breakdown from a rocprofv3 kernel_trace.csv or rocpd results.db.

Steps are delimited by the step's single k_step3d_t dispatch; only the last
`--steps` steps are summarised (warm-up and first-touch dispatches dropped).
Usage: python tools/prof_summary.py run_kernel_trace.csv --steps 10
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="k_step3d_t(")
    a = ap.parse_args()
    if a.trace.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(a.trace)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s0, "End_Timestamp": e0}
                for n, s0, e0 in con.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [n for n, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < a.steps + 1:
        raise SystemExit("not enough steps in trace")
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    win = rows[lo:hi]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in win:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[name] += 1
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
    busy = sum(tot.values())
    print("%-36s %8s %10s %10s %6s" % ("kernel", "calls/st", "us/step", "us/call", "%busy"))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("%-36s %8.1f %10.1f %10.2f %6.1f" % (k[:36], cnt[k] / a.steps, v / a.steps, v / cnt[k], 100 * v / busy))
    print("busy %.1f us/step, span %.1f us/step, gaps %.1f%%" % (busy / a.steps, span / a.steps, 100 * (1 - busy / span)))


if __name__ == "__main__":
    main()
