"""Per-routine HBM traffic from rocprofv3 PMC passes.

MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are collected
in separate passes (FETCH_SIZE costs 3 TCC counters, WRITE_SIZE 2); on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so
traffic = 2*FETCH_SIZE + WRITE_SIZE (KB units -> bytes).  Kernels map to the
reference routine that launches them; k_uv_horiz runs once in pre_step3d and
once in step3d_uv1 and is split evenly (in whole steps it rides inside
k_prsgrd_uv, whose bytes then count as prsgrd); halo wraps are reported
separately.  rho_eos runs twice per step (the step-opening one is reused).

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv
          --steps-marker k_step3d_t_v --out profiles/pmc_traffic.json
"""
import argparse
import collections
import csv
import json

ROUTINE_OF = {
    "k_rho_eos_linear": "rho_eos", "k_rho_eos_split": "rho_eos", "k_set_huv": "set_HUV", "k_omega": "omega",
    "k_omega_edges": "omega", "k_omega_seg": "omega", "k_prsgrd_P": "prsgrd", "k_prsgrd_uv": "prsgrd", "k_pre_tracer_h": "pre_step3d",
    "k_pre_tracer_v": "pre_step3d", "k_rd": "pre_step3d", "k_pre_uv": "pre_step3d", "k_set_huv1": "set_HUV1",
    "k_uv1": "step3d_uv1", "k_visc3d": "visc3d", "k_s2d_zeta": "step2d", "k_s2d_mom": "step2d",
    "k_s2d_zetabc": "step2d", "k_s2d_fb": "step2d", "k_visc3d_frc": "visc3d", "k_s2d_edges": "step2d", "k_s2d_last": "step2d", "k_set_depth": "step2d",
    "k_uv2_couple": "step3d_uv2", "k_uv2_flux": "step3d_uv2", "k_step3d_t_h": "step3d_t", "k_step3d_t_v": "step3d_t",
    "k_t3dmix": "t3dmix", "k_step3d_t_seg": "step3d_t", "k_periodic_wrap": "halo", "k_halo_pack": "halo", "k_halo_unpack": "halo",
    # round-2 kernels: register / segment / chained forms
    "k_uv1_reg": "step3d_uv1", "k_uv1_seg": "step3d_uv1", "k_pre_tracer_v_reg": "pre_step3d",
    "k_pre_tracer_seg": "pre_step3d", "k_pre_uv_seg": "pre_step3d", "k_uv2_fused": "step3d_uv2",
    "k_set_huv1_chain": "set_HUV1", "k_kpp_ext": "lmd_vmix", "k_kpp_int": "lmd_vmix", "k_prsgrd_fused": "prsgrd",
    "k_bulk_flux": "bulk_flux", "k_t3dbc_edges": "step3d_t", "k_t3dbc_corners": "step3d_t", "k_u3dbc": "step3d_uv2",
    "k_v3dbc": "step3d_uv2", "k_pre_tracer_h1": "pre_step3d", "k_step3d_t_h1": "step3d_t",
    # round-3 late: staged-window forms
    "k_visc3d_stg": "visc3d", "k_t3dmix_stg": "t3dmix",
    # round 5: buffer-addressed segment solvers
    "k_pre_tracer_segb": "pre_step3d", "k_pre_uv_segb": "pre_step3d", "k_uv1_segb": "step3d_uv1",
    "k_step3d_t_segb": "step3d_t",
    # round 6: prsgrd + momentum r.h.s. in j-marching strips
    "k_prsgrd_strip": "prsgrd",
}
CALLS_PER_STEP = {"rho_eos": 2, "set_HUV": 1, "omega": 3, "prsgrd": 2, "pre_step3d": 1, "set_HUV1": 1,
                  "step3d_uv1": 1, "visc3d": 1, "step2d": None, "step3d_uv2": 1, "step3d_t": 1, "t3dmix": 1,
                  "lmd_vmix": 2, "bulk_flux": 2}


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    return n.split("<")[0].split("::")[-1]


def read(path, counter):
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = short(r["Kernel_Name"])
        tot[k] += float(r["Counter_Value"]) * 1024.0  # KB
        cnt[k] += 1
    return tot, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--steps-marker", default="k_step3d_t_v")
    ap.add_argument("--nfast", type=int, default=82)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    f, fc = read(a.fetch, "FETCH_SIZE")
    w, _ = read(a.write, "WRITE_SIZE")
    steps = fc.get(a.steps_marker, 0)
    if steps == 0:
        raise SystemExit("marker kernel %s not found" % a.steps_marker)
    kern = {}
    per_routine = collections.defaultdict(float)
    for k in sorted(set(f) | set(w)):
        b = 2.0 * f.get(k, 0.0) + w.get(k, 0.0)
        kern[k] = {"dispatches": fc.get(k, 0), "fetch_size_bytes": f.get(k, 0.0), "write_size_bytes": w.get(k, 0.0),
                   "traffic_bytes": b}
        r = ROUTINE_OF.get(k)
        if k in ("k_uv_horiz", "k_uv_horiz1"):
            per_routine["pre_step3d"] += 0.5 * b
            per_routine["step3d_uv1"] += 0.5 * b
        elif r:
            per_routine[r] += b
    routines = {}
    for r, b in per_routine.items():
        calls = steps * (a.nfast if r == "step2d" else CALLS_PER_STEP.get(r, 1) or 1)
        routines[r] = {"bytes_total": b, "calls": calls, "bytes_per_launch": b / calls}
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), traffic = 2*FETCH + WRITE",
           "steps": steps, "routines": routines, "kernels": kern}
    json.dump(out, open(a.out, "w"), indent=1)
    for r, v in sorted(routines.items(), key=lambda kv: -kv[1]["bytes_total"]):
        print("%-12s %10.1f MB/launch  (%d launches)" % (r, v["bytes_per_launch"] / 1e6, v["calls"]))


if __name__ == "__main__":
    main()
