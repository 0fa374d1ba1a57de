"""Benchmark of the MI355X split-explicit ROMS step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): Filament physics +
salinity (linear EOS, T and S), 512x512x50 per GPU, dt=5 s, ndtfast=60 ->
nfast=82, dx=100 m, dy=25 m, doubly periodic, synthetic analytic initial
state.  One "step" = one full roms_step (main.F:333-520): 3 rho_eos, 3 omega,
2 prsgrd, pre_step3d, set_HUV/HUV1, step3d_uv1, visc3d, 82 barotropic
step2d_FB, step3d_uv2, step3d_t, t3dmix.  State is resident in HBM before
the timed region; steady steps replay captured HIP graphs.

N GPUs (one process each, torchrun): weak scaling on an npx x npe processor
grid (1x1, 2x1, 2x2, 4x2, ...) of 512x512 subdomains of one periodic domain;
halo exchanges go over RCCL (xGMI) inside the step graphs.

value = grid-cell updates per second summed over ranks; model seconds per
wall second beside it.  roofline: algorithmic bytes (SURVEY.md 8(d) pass
counts) / mean launch duration measured with HIP events on the library
stream, for the dominant kernel (C2: k_s2d_fb, one fast step, 35 2-D passes;
C3: its routine pre_step3d); "roofline_routine" is the dominant routine and
"routines" the full per-routine table.

--workload c3 (not the default): SURVEY.md 8(d) C3, the 1024x1024x100 closed
basin with NONLIN+SPLIT EOS, T+S and LMD/KPP/BKPP mixing (dt=300 s, nfast=82),
strong-scaled over the processor grid (the north_star's roofline target).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3]
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

# C2 workload, per GPU
LLM, MMM, NZ, NT = 512, 512, 50, 2
DT, NDTFAST = 5.0, 60
SIZEX, SIZEY = 51.2e3, 12.8e3
NT_TS = 2
# C3 workload, whole domain (strong scaling)
C3_L, C3_N, C3_DT, C3_DX = 1024, 100, 300.0, 2.0e3


def routine_passes(NT_, NT_TS_, lmd=False):
    """unique 3-D array passes per call; step2d counts 35 2-D
    passes per fast step (flagged with None).  lmd: the C3 switch set
    (NONLIN+SPLIT EOS, SALINITY, LMD/KPP), P3D = 150 + 10*NT."""
    if lmd:
        return {"rho_eos": 7, "set_HUV": 7, "omega": 6, "prsgrd": 6, "pre_step3d": 18 + 4 * NT_, "set_HUV1": 7,
                "step3d_uv1": 14, "visc3d": 7, "step2d": None, "step3d_uv2": 11, "step3d_t": 9 + 3 * NT_,
                "t3dmix": 1 + 3 * NT_, "lmd_vmix": 11}
    return {"rho_eos": 2 + NT_TS_, "set_HUV": 7, "omega": 6, "prsgrd": 5, "pre_step3d": 16 + NT_TS_ + 4 * NT_,
            "set_HUV1": 7, "step3d_uv1": 14, "visc3d": 7, "step2d": None, "step3d_uv2": 11,
            "step3d_t": 5 + NT_TS_ + 3 * NT_, "t3dmix": 1 + 3 * NT_, "lmd_vmix": 0}


def step_bytes(I, J, N, NT_, NT_TS_, nfast, lmd=False):
    """B_step = 8*(P3D*I*J*N + 35*nfast*I*J),
    P3D = 105+5*NT_TS+10*NT (Filament) or 150+10*NT (C3 switches)."""
    P3D = (150 + 10 * NT_) if lmd else (105 + 5 * NT_TS_ + 10 * NT_)
    return 8.0 * (P3D * I * J * N + 35.0 * nfast * I * J)


def proc_grid(n):
    npx = 1
    while npx * npx < n:
        npx *= 2
    npx = min(npx, n)
    while n % npx:
        npx -= 1
    return npx, n // npx


def cpu_baseline_c3(nsteps=2, L=128):
    """Oracle on a bounded LxLx100 cut of the C3 basin (same switches, dx)."""
    import oracle
    c = oracle.OrCfg()
    c.LLm, c.MMm, c.N, c.NT = L, L, C3_N, 2
    c.ew_periodic = c.ns_periodic = 0
    c.salinity, c.nonlin_eos, c.lmd = 1, 1, oracle.LMD_ICELAND
    c.case_id = oracle.CASE_BASIN
    c.dt, c.ndtfast = C3_DT, NDTFAST
    c.theta_s, c.theta_b, c.hc, c.rho0 = 6.0, 2.0, 250.0, 1027.5
    c.rdrg, c.rdrg2, c.Zob = 0.0, 1.0e-3, 1.0e-2
    c.Akv_bak = 1.0e-4
    c.Akt_bak[0] = c.Akt_bak[1] = 1.0e-5
    c.Tcoef, c.T0, c.Scoef, c.S0 = 0.20, 1.0, 0.822, 1.0
    c.sizex = c.sizey = C3_DX * L
    c.diag_np_xi = c.diag_np_eta = 1
    o = oracle.Oracle(c)
    o.init()
    t0 = time.perf_counter()
    o.step(nsteps)
    dt_wall = time.perf_counter() - t0
    cells = L * L * C3_N
    return {"value": nsteps * cells / dt_wall, "unit": "cell-updates/s", "cores": 1, "kind": "port",
            "sample": "%d roms_step of a %dx%dx%d cut of the C3 basin (LMD/KPP, nonlinear EOS) on the oracle "
                      "(oracle/, gcc -O2, 1 thread), %.1f s" % (nsteps, L, L, C3_N, dt_wall),
            "model_seconds_per_wallclock_sec": nsteps * C3_DT / dt_wall * cells / (C3_L * C3_L * C3_N)}


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


def pmc_kernel_traffic(kernel):
    """HBM bytes per dispatch of one kernel from profiles/pmc_traffic.json
    (2*FETCH_SIZE + WRITE_SIZE), or None when absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        k = json.load(open(p)).get("kernels", {}).get(kernel)
        return None if k is None else float(k["traffic_bytes"]) / float(k["dispatches"])
    except (ValueError, KeyError, TypeError, ZeroDivisionError):
        return None


def pmc_traffic(routine):
    """HBM bytes per launch of `routine` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, FETCH_SIZE*2 + WRITE_SIZE per
    MI355X_MICROARCH.md), or None when absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        r = d.get("routines", {}).get(routine)
        return None if r is None else float(r["bytes_per_launch"])
    except (ValueError, KeyError, TypeError):
        return None


def main():
    # the JSON line is the only thing on stdout: libraries (RCCL prints a
    # version banner at init) write to fd 1, so point it at stderr for the run
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--timing-steps", type=int, default=3, help="eager steps per routine for the event timings")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("c2", "c3"), default="c2")
    args = ap.parse_args()
    c3 = args.workload == "c3"

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import romsgpu

    dist = None
    comm = None
    npx, npe = proc_grid(world)
    # ROMS_BENCH_FORCE_COMM=1: take the multi-rank path even at world size 1
    # (RCCL comm + self-addressed exchanges; rehearses the N>1 plumbing)
    force = os.environ.get("ROMS_BENCH_FORCE_COMM") == "1"
    if world > 1 or force:
        if force:
            os.environ.setdefault("ROMS_GPU_RCCL_SELF", "1")
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")
        # bootstrap the library's own RCCL communicator through torch.distributed
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(romsgpu.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        comm = romsgpu.comm_create(bytes(uid.cpu().numpy().tobytes()), world, rank, local_rank)

    if c3:
        m = romsgpu.Model.from_case(romsgpu.CASE_BASIN, C3_L, C3_L, C3_N, NT, salinity=True, nonlin_eos=True,
                                    lmd=romsgpu.LMD_ICELAND, dt=C3_DT, ndtfast=NDTFAST, sizex=C3_DX * C3_L, sizey=C3_DX * C3_L,
                                    device=local_rank, np_xi=npx, np_eta=npe, comm=comm, rank=rank)
        Lr, Mr, Nz, dt_step = m.Lm, m.Mm, C3_N, C3_DT
    else:
        m = romsgpu.Model.from_case(romsgpu.CASE_FILAMENT, LLM * npx, MMM * npe, NZ, NT, salinity=True, dt=DT,
                                    ndtfast=NDTFAST, sizex=SIZEX * npx, sizey=SIZEY * npe, device=local_rank,
                                    np_xi=npx, np_eta=npe, comm=comm, rank=rank)
        assert (m.Lm, m.Mm) == (LLM, MMM)
        Lr, Mr, Nz, dt_step = LLM, MMM, NZ, DT
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

    # per-routine rooflines: HIP events around each routine's launches
    cells3 = Lr * Mr * Nz
    passes = routine_passes(NT, NT_TS, lmd=c3)
    routines = {}
    for r in romsgpu.ROUTINES:
        if passes.get(r, 0) == 0:   # kernel-level ids and routines off in this workload
            continue
        avg, n = m.time_routine(r, args.timing_steps)
        per_step = n / args.timing_steps
        nbytes = 35.0 * 8 * Lr * Mr if passes[r] is None else 8.0 * passes[r] * cells3
        gbs = nbytes / (avg * 1e-3) / 1e9 if avg > 0 else 0.0
        routines[r] = {"ms_per_call": avg, "calls_per_step": per_step, "ms_per_step": avg * per_step,
                       "bytes_per_call": nbytes, "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}
    dom = max(routines, key=lambda k: routines[k]["ms_per_step"])
    D = routines[dom]
    # the fused barotropic kernel alone (HIP events around its launches only):
    # 35 2-D passes per fast step over its launch time
    # (one event interval per fast loop on a single rank: 82 back-to-back launches)
    fb_ms, fb_n = m.time_routine("k_s2d_fb", args.timing_steps)
    fb_bytes = 35.0 * 8 * Lr * Mr
    fb_gbs = fb_bytes / (fb_ms * 1e-3) / 1e9 if fb_ms > 0 else 0.0
    kernel_fb = {"kernel": "k_s2d_fb", "ms_per_launch": fb_ms, "launches_per_step": fb_n / args.timing_steps,
                 "ms_per_step": fb_ms * fb_n / args.timing_steps, "bytes_per_launch": fb_bytes,
                 "achieved_GBs": fb_gbs, "frac": fb_gbs / HBM_PEAK_GBS}

    transport = m.halo_transport() if comm is not None else "none (single rank)"
    # sanity: the run must stay finite (blow-up check as diag.F does)
    norms = m.diag()
    if not all(map(lambda x: x == x and abs(x) < 1e30, norms)):
        raise SystemExit("bench: non-finite diag norms %r" % norms)

    ms_step = 1e3 * elapsed / args.steps
    B = step_bytes(Lr, Mr, Nz, NT, NT_TS, nfast, lmd=c3)
    step_gbs = B / (ms_step * 1e-3) / 1e9
    traffic = None if c3 else pmc_traffic(dom)   # profiles/pmc_traffic.json is measured on C2

    if not c3:
        # C2: the dominant kernel (largest time per step in the kernel-trace
        # table, profiles/r1_p5_c2_per_step.txt) is the fused barotropic kernel
        roofline = {"bound": "hbm", "achieved": fb_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": fb_gbs / HBM_PEAK_GBS, "traffic": pmc_kernel_traffic("k_s2d_fb"),
                    "kernel": "k_s2d_fb", "bytes_per_launch": fb_bytes, "ms_per_launch": fb_ms}
    else:
        # C3: the dominant kernel is k_pre_uv_seg (profiles/r1_p5_c3_per_step.txt),
        # timed with the rest of its routine (pre_step3d)
        roofline = {"bound": "hbm", "achieved": D["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": D["frac"], "traffic": None, "kernel": dom + " (routine)",
                    "bytes_per_launch": D["bytes_per_call"], "ms_per_launch": D["ms_per_call"]}
    out = {
        "metric": "grid-cell-updates/sec",
        "value": (C3_L * C3_L * C3_N if c3 else world * cells3) * args.steps / elapsed,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if c3 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (analytic closed basin, SURVEY.md 8(d) C3)" if c3 else
                 "synthetic (analytic Filament+S initial state, ana_grid/ana_init of tests/Filament)"),
        "config": {"workload": ("C3: basin 1024x1024x100, NONLIN+SPLIT EOS, T+S, LMD/KPP/BKPP, dt=300s, ndtfast=60 "
                                "(nfast=%d)" % nfast) if c3 else
                               "C2: Filament+S 512x512x50 per GPU, NT=2, dt=5s, ndtfast=60 (nfast=%d)" % nfast,
                   "grid_per_gpu": [Lr, Mr, Nz], "proc_grid": [npx, npe], "NT": NT, "dt": dt_step, "nfast": nfast,
                   "parallelism": "domain decomposition %dx%d" % (npx, npe), "halo_transport": transport},
        "model_seconds_per_wallclock_sec": args.steps * dt_step / elapsed,
        "roofline": roofline,
        "roofline_routine": {"bound": "hbm", "achieved": D["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": D["frac"], "traffic": traffic,
                             "routine": dom + (" (one fast step: k_s2d_fb + edges + halo)" if dom == "step2d" else ""),
                             "bytes_per_launch": D["bytes_per_call"], "ms_per_launch": D["ms_per_call"]},
        "roofline_step": {"bound": "hbm", "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": step_gbs / HBM_PEAK_GBS, "bytes_per_step": B},
        "routines": routines,
        "kernel_s2d_fb": kernel_fb,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_c3() if c3 else cpu_baseline()
    m.close()
    if comm is not None:
        romsgpu.comm_destroy(comm)
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
