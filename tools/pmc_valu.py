"""VALU instruction mix per kernel from one rocprofv3 --pmc pass:
SQ_WAVES, SQ_INSTS_VALU and the FP64 classes (ADD/MUL/FMA/TRANS_F64),
INT32, INT64 -- mean per dispatch -> profiles/pmc_valu_c3.json.  bench.py
turns it into the dominant kernel's VALU issue fraction (roofline.valu_frac):
a wave64 FP64 instruction holds a SIMD 4 cycles (78.6 TF FP64 = 16 lanes per
cycle per SIMD on 1024 SIMDs at 2.4 GHz), every other VALU instruction 2.
usage: python tools/pmc_valu.py counter_collection.csv --out profiles/pmc_valu_c3.json"""
import argparse
import collections
import csv
import json

F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    return n.split("<")[0].split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for p in a.csvs:
        for r in csv.DictReader(open(p)):
            k, c = short(r["Kernel_Name"]), r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[k][c]))
    out = {"source": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 "
                     "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 (one pass), mean per dispatch",
           "kernels": {}}
    for k, m in tot.items():
        n = max(len(v) for v in disp[k].values())
        per = {c: v / n for c, v in m.items()}
        waves = per.get("SQ_WAVES", 0.0)
        valu = per.get("SQ_INSTS_VALU", 0.0)
        f64 = sum(per.get(c, 0.0) for c in F64)
        out["kernels"][k] = {"dispatches": n, "waves": waves, "valu": valu, "valu_f64": f64,
                             "valu_int32": per.get("SQ_INSTS_VALU_INT32", 0.0),
                             "valu_int64": per.get("SQ_INSTS_VALU_INT64", 0.0),
                             "valu_per_wave": valu / waves if waves else None,
                             "f64_per_wave": f64 / waves if waves else None}
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["valu"])[:20]:
        print("%-24s waves %10.0f  VALU/wave %7.1f  F64/wave %7.1f" % (k, v["waves"], v["valu_per_wave"] or 0,
                                                                      v["f64_per_wave"] or 0))


if __name__ == "__main__":
    main()
