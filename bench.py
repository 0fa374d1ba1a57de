"""Benchmark of the MI355X split-explicit ROMS step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): Filament physics +
salinity (linear EOS, T and S), 512x512x50, dt=5 s, ndtfast=60 -> nfast=82,
domain 51.2 km x 12.8 km (dx=100 m, dy=25 m), doubly periodic, synthetic
analytic initial state.  One "step" = one full roms_step (main.F:333-520):
2 rho_eos, 3 omega, 2 prsgrd, pre_step3d, set_HUV/HUV1, step3d_uv1, visc3d,
82 barotropic step2d_FB, step3d_uv2, step3d_t, t3dmix.  State is resident
in HBM before the timed region; steady steps replay captured HIP graphs.

value = grid-cell updates per second summed over ranks (weak scaling: each
rank advances its own 512x512x50 subdomain); model seconds per wall second
reported beside it, with the HBM roofline of the step and of its dominant
kernel (algorithmic bytes, SURVEY.md 8(d) pass counts, / measured time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ucla-roms_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# C2 workload
LLM, MMM, NZ, NT = 512, 512, 50, 2
DT, NDTFAST = 5.0, 60
SIZEX, SIZEY = 51.2e3, 12.8e3


def step_bytes(I, J, N, NT_, NT_TS, nfast):
    """B_step = 8*(P3D*I*J*N + 35*nfast*I*J), linear EOS, no LMD:
    P3D = 105 + 5*NT_TS + 10*NT."""
    P3D = 105 + 5 * NT_TS + 10 * NT_
    return 8.0 * (P3D * I * J * N + 35.0 * nfast * I * J)


def cpu_baseline(nsteps=3):
    """Oracle (plain-C restatement, 1 thread) on the same 512x512x50 workload,
    a bounded sample of `nsteps` steps after init."""
    import oracle
    cfg = oracle.filament_cfg(LLm=LLM, MMm=MMM, N=NZ, NT=NT, salinity=True, sizex=SIZEX, sizey=SIZEY,
                              np_xi=1, np_eta=1)
    o = oracle.Oracle(cfg)
    o.init()
    t0 = time.perf_counter()
    o.step(nsteps)
    dt_wall = time.perf_counter() - t0
    return {"value": nsteps * LLM * MMM * NZ / dt_wall, "unit": "cell-updates/s", "cores": 1, "kind": "port",
            "sample": "%d roms_step of the 512x512x50 C2 workload on the oracle (oracle/, gcc -O2, 1 thread), %.1f s"
                      % (nsteps, dt_wall),
            "model_seconds_per_wallclock_sec": nsteps * DT / dt_wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")

    import romsgpu
    m = romsgpu.Model.from_case(romsgpu.CASE_FILAMENT, LLM, MMM, NZ, NT, salinity=True, dt=DT, ndtfast=NDTFAST,
                                sizex=SIZEX, sizey=SIZEY, device=local_rank)
    nfast = m.t.nfast
    m.step(args.warmup)
    m.sync()

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    m.sync()
    t0 = time.perf_counter()
    ev_ms = m.time_steps(args.steps)  # HIP events on the library stream around K steps
    m.sync()
    wall = time.perf_counter() - t0
    barrier()
    elapsed = max(wall, ev_ms / 1e3)
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # sanity: the run must stay finite (blow-up check as diag.F does)
    norms = m.diag()
    if not all(map(lambda x: x == x and abs(x) < 1e30, norms)):
        raise SystemExit("bench: non-finite diag norms %r" % norms)

    ms_step = 1e3 * elapsed / args.steps
    cells = LLM * MMM * NZ
    B = step_bytes(LLM, MMM, NZ, NT, 2, nfast)
    step_gbs = B / (ms_step * 1e-3) / 1e9

    # dominant kernel: time it in isolation with HIP events on the library stream
    dom = m.kernel_roofline() if hasattr(m, "kernel_roofline") else None

    out = {
        "metric": "grid-cell-updates/sec",
        "value": world * cells * args.steps / elapsed,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (analytic Filament+S initial state, ana_grid/ana_init of tests/Filament)",
        "config": {"workload": "C2: Filament+S 512x512x50 per GPU, NT=2, dt=5s, ndtfast=60 (nfast=%d)" % nfast,
                   "grid": [LLM, MMM, NZ], "NT": NT, "dt": DT, "nfast": nfast, "parallelism": "%d GPU" % world},
        "model_seconds_per_wallclock_sec": args.steps * DT / elapsed,
        "roofline_step": {"bound": "hbm", "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": step_gbs / HBM_PEAK_GBS, "bytes_per_step": B},
    }
    if dom is not None:
        out["roofline"] = dom
    else:
        out["roofline"] = dict(out["roofline_step"], kernel="whole roms_step (graph)", traffic=None)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    m.close()
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
