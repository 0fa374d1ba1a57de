"""Benchmark of the MI355X split-explicit ROMS step (BASELINE.json metric:
model-seconds/wallclock-sec + grid-cell-updates/sec at 1/2/4/8 GPU; % HBM
roofline).

Primary workload (the north_star's target configuration, SURVEY.md 8(d) C3,
BASELINE.json configs[2] on one GPU): the 1024x1024x100 closed basin with
NONLIN+SPLIT EOS, T+S and LMD_MIXING+KPP+BKPP+RIMIX+NONLOCAL (dt=300 s,
ndtfast=60 -> nfast=82), synthetic analytic initial state.  One "step" = one
full roms_step (main.F:333-520): rho_eos, set_HUV, omega, lmd_vmix, prsgrd,
pre_step3d, set_HUV1, omega, rho_eos, lmd_vmix, prsgrd, step3d_uv1, visc3d,
82 barotropic step2d_FB, step3d_uv2, omega, step3d_t, t3dmix, rho_eos.  The
step-opening rho_eos(nrhs) (main.F:397) reads exactly the t, z_r, Hz the
previous step's closing rho_eos(nnew) (main.F:479) read, so the library keeps
those outputs instead of recomputing them (bitwise-equal runs,
ROMS_GPU_RHO_REUSE=0 turns it off); roofline_step's byte count leaves that pass
out, and the two Hz_u/Hz_v stores of set_HUV that whole steps skip
(extract_data inputs only, ROMS_GPU_HZ_UV=1 keeps them).  State is resident in
HBM before the timed region; steady steps replay captured HIP graphs.  N GPUs:
strong scaling of the one basin over an npx x npe processor grid (1x1, 2x1,
2x2, 4x2), halo exchanges inside the step graphs.  "north_star_loop" is the
north_star's own roofline target: step2d_FB + step3d_uv1 + step3d_uv2 +
step3d_t algorithmic bytes over their summed routine time.

Secondary workload, reported in the same JSON line as "c2" (BASELINE.json
configs[1]): Filament physics + salinity (linear EOS, T and
S), 512x512x50 per GPU, dt=5 s, ndtfast=60 -> nfast=82, dx=100 m, dy=25 m,
doubly periodic, weak-scaled (512x512 per GPU).  --workload c2 makes it the
primary line and C3 the secondary ("c3").

value = grid-cell updates per second summed over ranks (interior I*J*N per
baroclinic step); model seconds per wall second beside it.  roofline: the
dominant kernel's algorithmic bytes (SURVEY.md 8(d) pass counts) over its
mean launch duration, measured with HIP events on the library stream;
"routines" has every routine; "roofline_step" the whole step.

cpu_baseline (rank 0, N=1): the plain-C oracle (oracle/, the CPU restatement,
"port") on a bounded sample of the same workloads, one process per available
host core (P processes x 1 thread, each on its own cut of the grid, started
together), run before the GPU is touched.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2] [--no-secondary]
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set
before any GPU call) and relays rank 0's line; under torchrun it is one rank.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ucla-roms_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# C2 workload, per GPU
C2_L, C2_N, NT, C2_DT, NDTFAST = 512, 50, 2, 5.0, 60
C2_DX, C2_DY = 100.0, 25.0
NT_TS = 2
# C3 workload, whole domain (strong scaling)
C3_L, C3_N, C3_DT, C3_DX = 1024, 100, 300.0, 2.0e3


# k_pre_uv_seg's share of pre_step3d's passes: u, v(nstp);
# u, v(indx) read and written; u, v(nnew) written; ru, rv; Hz, We, Wi, Akv.
# (The Hz_fwd / Hz_bak scratch it also reads is not a reference array: not counted.)
PRE_UV_SEG_PASSES = 14
# k_prsgrd_uv in whole steps (the prsgrd ru/rv kernel with the horizontal
# momentum r.h.s. of the following pre_step3d / step3d_uv1): z_r, rho1, qp1,
# Hz; u, v(nrhs), FlxU, FlxV read; ru, rv written.  The hydrostatic pressure
# P it also reads is prsgrd's own work array (prsgrd.F:200-330 forms it in
# the routine; here rho_eos's sweep stores it): not a model array, so it is
# not counted -- the bytes it costs lower the fraction.
PRSGRD_UV_PASSES = 10
# k_uv1_segb is all of step3d_uv1 (14 passes)
UV1_SEG_PASSES = 14
# roofline.traffic is not measured in the bench run: it is read from the PMC
# table tools/gpu.sh pmc wrote (a separate rocprofv3 --pmc pass per counter)
PMC_SOURCE_C3 = "stored: profiles/pmc_traffic_c3.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE passes; tools/gpu.sh pmc)"
PMC_SOURCE_C2 = "stored: profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE passes; tools/gpu.sh pmc)"


# set_HUV's Hz_u/Hz_v (set_depth.F:220,227) feed only extract_data.F; whole
# steps store them only on request (ROMS_GPU_HZ_UV=1, include/roms_gpu.h), so
# set_HUV's pass count is 5 (Hz, u, v read; FlxU, FlxV written), else 7
HZ_UV_PASSES = 2 if os.environ.get("ROMS_GPU_HZ_UV") == "1" else 0


def routine_passes(NT_, NT_TS_, lmd=False):
    """unique 3-D array passes per call; step2d counts 35 2-D
    passes per fast step (flagged with None).  lmd: the C3 switch set
    (NONLIN+SPLIT EOS, SALINITY, LMD/KPP), P3D = 150 + 10*NT."""
    huv = 5 + HZ_UV_PASSES
    if lmd:
        return {"rho_eos": 7, "set_HUV": huv, "omega": 6, "prsgrd": 6, "pre_step3d": 18 + 4 * NT_, "set_HUV1": 7,
                "step3d_uv1": 14, "visc3d": 7, "step2d": None, "step3d_uv2": 11, "step3d_t": 9 + 3 * NT_,
                "t3dmix": 1 + 3 * NT_, "lmd_vmix": 11}
    return {"rho_eos": 2 + NT_TS_, "set_HUV": huv, "omega": 6, "prsgrd": 5, "pre_step3d": 16 + NT_TS_ + 4 * NT_,
            "set_HUV1": 7, "step3d_uv1": 14, "visc3d": 7, "step2d": None, "step3d_uv2": 11,
            "step3d_t": 5 + NT_TS_ + 3 * NT_, "t3dmix": 1 + 3 * NT_, "lmd_vmix": 0}


def step_bytes(I, J, N, NT_, NT_TS_, nfast, lmd=False):
    """B_step = 8*(P3D*I*J*N + 35*nfast*I*J),
    P3D = 105+5*NT_TS+10*NT (Filament) or 150+10*NT (C3 switches), less the
    one rho_eos call per step the library does not repeat and the Hz_u/Hz_v
    stores whole steps skip (see above)."""
    P3D = (150 + 10 * NT_) if lmd else (105 + 5 * NT_TS_ + 10 * NT_)
    P3D -= routine_passes(NT_, NT_TS_, lmd)["rho_eos"]
    P3D -= 2 - HZ_UV_PASSES
    return 8.0 * (P3D * I * J * N + 35.0 * nfast * I * J)


def proc_grid(n):
    npx = 1
    while npx * npx < n:
        npx *= 2
    npx = min(npx, n)
    while n % npx:
        npx -= 1
    return npx, n // npx


# ---------------------------------------------------------------------------
# CPU baseline: P oracle processes, one per core
# ---------------------------------------------------------------------------
def _cpu_worker(kind, L, M, nsteps):
    """Child process: one oracle instance on an LxM cut; waits for GO on stdin
    after init so all P processes step together; prints the step time."""
    import oracle
    if kind == "c2":
        cfg = oracle.filament_cfg(LLm=L, MMm=M, N=C2_N, NT=NT, salinity=True, sizex=C2_DX * L, sizey=C2_DY * M,
                                  np_xi=1, np_eta=1)
    else:
        cfg = oracle.OrCfg()
        cfg.LLm, cfg.MMm, cfg.N, cfg.NT = L, M, C3_N, 2
        cfg.ew_periodic = cfg.ns_periodic = 0
        cfg.salinity, cfg.nonlin_eos, cfg.lmd = 1, 1, oracle.LMD_ICELAND
        cfg.case_id = oracle.CASE_BASIN
        cfg.dt, cfg.ndtfast = C3_DT, NDTFAST
        cfg.theta_s, cfg.theta_b, cfg.hc, cfg.rho0 = 6.0, 2.0, 250.0, 1027.5
        cfg.rdrg, cfg.rdrg2, cfg.Zob = 0.0, 1.0e-3, 1.0e-2
        cfg.Akv_bak = 1.0e-4
        cfg.Akt_bak[0] = cfg.Akt_bak[1] = 1.0e-5
        cfg.Tcoef, cfg.T0, cfg.Scoef, cfg.S0 = 0.20, 1.0, 0.822, 1.0
        cfg.sizex, cfg.sizey = C3_DX * L, C3_DX * M
        cfg.diag_np_xi = cfg.diag_np_eta = 1
    o = oracle.Oracle(cfg)
    o.init()
    print("READY", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    o.step(nsteps)
    print(json.dumps({"wall": time.perf_counter() - t0}), flush=True)


def host_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")   # the GPU box exports its CPU share (16) here
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline(kind):
    """P = host cores oracle processes, each stepping its own cut of the
    workload grid (independent subdomains: no halo exchange between them),
    started together; value = all cell updates / the slowest process's time."""
    P = host_cores()
    if kind == "c2":
        L, M, nsteps, N, dt, full = C2_L, max(8, C2_L // P), 5, C2_N, C2_DT, C2_L * C2_L * C2_N
    else:
        L, M, nsteps, N, dt, full = C3_L, 32, 2, C3_N, C3_DT, C3_L * C3_L * C3_N
    env = dict(os.environ, OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", kind, str(L), str(M),
                            str(nsteps)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
          for _ in range(P)]
    try:
        for p in ps:
            if p.stdout.readline().strip() != "READY":
                raise RuntimeError("cpu baseline worker failed")
        for p in ps:
            p.stdin.write("GO\n")
            p.stdin.flush()
        walls = [json.loads(p.stdout.readline())["wall"] for p in ps]
    finally:
        for p in ps:
            try:
                p.wait(timeout=120)
            except subprocess.TimeoutExpired:
                p.kill()
    wall = max(walls)
    cells = P * L * M * N * nsteps
    v = cells / wall
    what = ("C2 Filament+S, %d periodic %dx%dx%d cuts" % (P, L, M, N) if kind == "c2" else
            "C3 basin (NONLIN+SPLIT EOS, LMD/KPP), %d closed %dx%dx%d cuts" % (P, L, M, N))
    return {"value": v, "unit": "cell-updates/s", "cores": P, "kind": "port",
            "layout": "%d processes x 1 thread (nproc %d)" % (P, os.cpu_count() or 0),
            "sample": "%d roms_step of %s on the oracle (oracle/, gcc -O2 plain-C restatement), one process per core, "
                      "no halo exchange between the cuts; slowest process %.1f s" % (nsteps, what, wall),
            "model_seconds_per_wallclock_sec": v / full * dt}


# ---------------------------------------------------------------------------
# multi-rank launch
# ---------------------------------------------------------------------------
def launch_ranks(args, argv):
    """Start args.gpus ranks of this script (one process per GPU) and relay
    rank 0's JSON line.  Runs before anything touches the GPU."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        ps.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                   stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = ps[0].stdout.read().decode()
    rcs = [p.wait() for p in ps]
    sys.stdout.write(out)
    sys.stdout.flush()
    return max(abs(rc) for rc in rcs)


# ---------------------------------------------------------------------------
# one workload on this rank
# ---------------------------------------------------------------------------
def run_workload(kind, romsgpu, comm, rank, world, local_rank, steps, warmup, timing_steps, barrier, allmax,
                 step_only=False, gather=None):
    npx, npe = proc_grid(world)
    c3 = kind == "c3"
    if c3:
        m = romsgpu.Model.from_case(romsgpu.CASE_BASIN, C3_L, C3_L, C3_N, NT, salinity=True, nonlin_eos=True,
                                    lmd=romsgpu.LMD_ICELAND, dt=C3_DT, ndtfast=NDTFAST, sizex=C3_DX * C3_L,
                                    sizey=C3_DX * C3_L, device=local_rank, np_xi=npx, np_eta=npe, comm=comm, rank=rank)
        Lr, Mr, Nz, dt_step = m.Lm, m.Mm, C3_N, C3_DT
        total_cells = C3_L * C3_L * C3_N
    else:
        m = romsgpu.Model.from_case(romsgpu.CASE_FILAMENT, C2_L * npx, C2_L * npe, C2_N, NT, salinity=True, dt=C2_DT,
                                    ndtfast=NDTFAST, sizex=C2_DX * C2_L * npx, sizey=C2_DY * C2_L * npe,
                                    device=local_rank, np_xi=npx, np_eta=npe, comm=comm, rank=rank)
        assert (m.Lm, m.Mm) == (C2_L, C2_L)
        Lr, Mr, Nz, dt_step = C2_L, C2_L, C2_N, C2_DT
        total_cells = world * C2_L * C2_L * C2_N
    nfast = m.t.nfast
    m.step(warmup)
    m.sync()
    barrier()
    t0 = time.perf_counter()
    ev_ms = m.time_steps(steps)  # HIP events on the library stream around K steps
    m.sync()
    wall = time.perf_counter() - t0
    barrier()
    elapsed = allmax(max(wall, ev_ms / 1e3))
    overlap = m.halo_overlap() if comm is not None else False
    s2d_window = m.s2d_window()
    if step_only:   # the whole-step time alone (the exchange-overlap A/B of a multi-rank run)
        m.close()
        return {"ms_per_step": 1e3 * elapsed / steps, "value": total_cells * steps / elapsed,
                "steps": steps, "overlap": overlap}
    halo_time = None
    if comm is not None:
        # the halo path per rank: HIP events around every exchange's pack,
        # transport (IPC: signal + arrival wait, which also absorbs the other
        # ranks' skew; RCCL: the send/recv group) and unpack over eager steps,
        # where each exchange runs in place (timing any kernel turns the
        # deferral off), so these are the costs the deferred order hides
        mine = []
        for ph in ("pack", "wait", "unpack"):
            hms, hn = m.time_routine("k_halo_" + ph, timing_steps)
            mine += [1e3 * hms * hn / timing_steps, float(hn) / timing_steps]
        per = gather(mine) if gather is not None else [mine]
        halo_time = {"source": "HIP events on the halo path, %d eager steps per phase, exchanges in place" % timing_steps,
                     "exchanges_per_step": [r[1] for r in per]}
        for q, ph in enumerate(("pack", "wait", "unpack")):
            halo_time[ph + "_us_per_step"] = [r[2 * q] for r in per]

    # per-routine rooflines: HIP events around each routine's launches
    cells3 = Lr * Mr * Nz
    passes = routine_passes(NT, NT_TS, lmd=c3)
    routines = {}
    for r in romsgpu.ROUTINES:
        if passes.get(r, 0) == 0:   # kernel-level ids and routines off in this workload
            continue
        avg, n = m.time_routine(r, timing_steps)
        per_step = n / timing_steps
        nbytes = 35.0 * 8 * Lr * Mr if passes[r] is None else 8.0 * passes[r] * cells3
        gbs = nbytes / (avg * 1e-3) / 1e9 if avg > 0 else 0.0
        routines[r] = {"ms_per_call": avg, "calls_per_step": per_step, "ms_per_step": avg * per_step,
                       "bytes_per_call": nbytes, "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}
        if r == "prsgrd":
            # whole steps run the horizontal momentum r.h.s. of the following
            # pre_step3d / step3d_uv1 inside prsgrd's kernel (k_prsgrd_uv<true>):
            # its time is in this routine; bytes_per_call stays prsgrd's own
            # passes, the *_with_rhs figures add the r.h.s. inputs u, v(nrhs),
            # FlxU, FlxV (4 passes) that the fused kernel reads
            wb = nbytes + 8.0 * 4 * cells3
            routines[r].update({"includes": "uv horizontal r.h.s. of pre_step3d and step3d_uv1",
                                "bytes_per_call_with_rhs": wb,
                                "frac_with_rhs": (wb / (avg * 1e-3) / 1e9 if avg > 0 else 0.0) / HBM_PEAK_GBS})
    dom = max(routines, key=lambda k: routines[k]["ms_per_step"])
    D = routines[dom]
    # the north_star's roofline target: "the step2d_FB + step3d_uv/t fused
    # loop" = the fast loop + step3d_uv1 + step3d_uv2 + step3d_t, their
    # SURVEY.md 8(d) algorithmic bytes per step over their summed event time
    loop = ("step2d", "step3d_uv1", "step3d_uv2", "step3d_t")
    lb = sum(routines[r]["bytes_per_call"] * routines[r]["calls_per_step"] for r in loop)
    lms = sum(routines[r]["ms_per_step"] for r in loop)
    lg = lb / (lms * 1e-3) / 1e9 if lms > 0 else 0.0
    north_star_loop = {"bound": "hbm", "achieved": lg, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": lg / HBM_PEAK_GBS,
                       "target_frac": 0.40, "bytes_per_step": lb, "ms_per_step": lms, "routines": list(loop),
                       "per_routine_frac": {r: routines[r]["frac"] for r in loop}}
    # the fused barotropic kernel alone: 35 2-D passes per fast step over its
    # launch time (one event interval per fast loop on a single rank)
    fb_ms, fb_n = m.time_routine("k_s2d_fb", timing_steps)
    fb_bytes = 35.0 * 8 * Lr * Mr
    fb_gbs = fb_bytes / (fb_ms * 1e-3) / 1e9 if fb_ms > 0 else 0.0
    kernel_fb = {"kernel": "k_s2d_fb", "ms_per_launch": fb_ms, "launches_per_step": fb_n / timing_steps,
                 "ms_per_step": fb_ms * fb_n / timing_steps, "bytes_per_launch": fb_bytes,
                 "achieved_GBs": fb_gbs, "frac": fb_gbs / HBM_PEAK_GBS}
    if c3:
        # C3: every kernel with a kernel-level event timer and a fixed
        # per-launch pass count (k_prsgrd_uv, k_pre_uv_seg, k_uv1_seg,
        # k_s2d_fb -- the four largest per step in the committed C3 trace);
        # the dominant kernel is the largest time per step among them, and
        # trace_check names the committed trace's own maximum beside it
        c3k = {}
        for kname, npass in (("k_pre_uv_seg", PRE_UV_SEG_PASSES), ("k_prsgrd_uv", PRSGRD_UV_PASSES),
                             ("k_uv1_seg", UV1_SEG_PASSES), ("k_s2d_fb", None)):
            if kname == "k_s2d_fb":
                kms, kn, kb = fb_ms, fb_n, fb_bytes
            else:
                kms, kn = m.time_routine(kname, timing_steps)
                kb = 8.0 * npass * cells3
            kg = kb / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
            names = PMC_KERNELS[kname]
            kt = pmc_group(names, _pmc(True), "traffic_bytes")
            c3k[kname] = {"bound": "hbm", "achieved": kg, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": kg / HBM_PEAK_GBS, "traffic": kt, "traffic_source": PMC_SOURCE_C3,
                          "kernel": " + ".join(n for n in names if pmc_group([n], _pmc(True), "traffic_bytes")) or
                                    kname,
                          "bytes_per_launch": kb, "ms_per_launch": kms,
                          "launches_per_step": kn / timing_steps, "ms_per_step": kms * kn / timing_steps,
                          "passes": npass if npass is not None else "35 2-D"}
            c3k[kname].update(valu_issue(names, kms))
    transport = m.halo_transport() if comm is not None else "none (single rank)"
    # exchanges per step (the fast loop's zeta/ubar/vbar swap every K fast steps)
    exch, fast_k = m.halo_exchanges() if comm is not None else (0, 1)
    norms = m.diag()   # blow-up check as diag.F does (collective)
    if not all(x == x and abs(x) < 1e30 for x in norms):
        raise SystemExit("bench: non-finite diag norms %r" % norms)
    ms_step = 1e3 * elapsed / steps
    B = step_bytes(Lr, Mr, Nz, NT, NT_TS, nfast, lmd=c3)
    step_gbs = B / (ms_step * 1e-3) / 1e9
    m.close()
    if not c3:
        # dominant kernel by time per step in the C2 kernel trace
        # (profiles/r2_*_c2_per_step.txt): the fused barotropic kernel
        roofline = {"bound": "hbm", "achieved": fb_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": fb_gbs / HBM_PEAK_GBS, "traffic": pmc_kernel_traffic("k_s2d_fb"),
                    "traffic_source": PMC_SOURCE_C2,
                    "kernel": "k_s2d_fb", "bytes_per_launch": fb_bytes, "ms_per_launch": fb_ms,
                    # the 73 MB fast-time working set stays in the 256 MiB Infinity
                    # Cache across the 82 launches; c3.kernel_s2d_fb is the same
                    # kernel's HBM-resident figure (294 MB per launch)
                    "cache_resident": True}
    else:
        dom_k = max(c3k, key=lambda k: c3k[k]["ms_per_step"])
        roofline = dict(c3k[dom_k])
        roofline["other_kernels"] = {k: v for k, v in c3k.items() if k != dom_k}
        roofline["trace_check"] = trace_top_kernel()
    return {
        "value": total_cells * steps / elapsed,
        "ms_per_step": ms_step,
        "model_seconds_per_wallclock_sec": steps * dt_step / elapsed,
        "config": {"workload": ("C3: basin 1024x1024x100, NONLIN+SPLIT EOS, T+S, LMD KPP/BKPP/RIMIX/NONLOCAL, "
                                "dt=300s, ndtfast=60 (nfast=%d)" % nfast) if c3 else
                               "C2: Filament+S 512x512x50 per GPU, NT=2, dt=5s, ndtfast=60 (nfast=%d)" % nfast,
                   "grid_per_gpu": [Lr, Mr, Nz], "proc_grid": [npx, npe], "NT": NT, "dt": dt_step, "nfast": nfast,
                   "parallelism": "domain decomposition %dx%d" % (npx, npe), "halo_transport": transport,
                   "halo_exchanges_per_step": exch, "fast_exchange_interval": fast_k,
                   "exchange_order": ("deferred (3-D exchanges beside the next routine)" if overlap else
                                      "in place" if comm is not None else "none (single rank)"),
                   "halo_time_per_rank": halo_time,
                   "s2d_window": s2d_window},
        "scaling": "strong" if c3 else "weak",
        "steps": steps, "warmup": warmup,
        "roofline": roofline,
        "north_star_loop": north_star_loop,
        "roofline_routine": {"bound": "hbm", "achieved": D["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": D["frac"], "traffic": pmc_traffic(dom, c3),
                             "routine": dom + (" (one fast step: k_s2d_fb + edges + halo)" if dom == "step2d" else ""),
                             "bytes_per_launch": D["bytes_per_call"], "ms_per_launch": D["ms_per_call"]},
        "roofline_step": {"bound": "hbm", "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": step_gbs / HBM_PEAK_GBS, "bytes_per_step": B},
        "routines": routines,
        "kernel_s2d_fb": kernel_fb,
    }


def _pmc(c3=False):
    p = os.path.join(ROOT, "profiles", "pmc_traffic_c3.json" if c3 else "pmc_traffic.json")
    if not os.path.exists(p):
        return {}
    try:
        return json.load(open(p))
    except ValueError:
        return {}


def pmc_kernel_traffic(kernel, c3=False):
    """HBM bytes per dispatch of one kernel from profiles/pmc_traffic.json
    (C2) or pmc_traffic_c3.json (2*FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md),
    or None when absent."""
    try:
        k = _pmc(c3).get("kernels", {}).get(kernel)
        return None if k is None else float(k["traffic_bytes"]) / float(k["dispatches"])
    except (KeyError, TypeError, ZeroDivisionError, ValueError):
        return None


# the kernels each timed interval of the C3 candidates launches (PMC table names)
PMC_KERNELS = {"k_prsgrd_uv": ["k_prsgrd_strip", "k_prsgrd_uv"], "k_pre_uv_seg": ["k_pre_uv_segb", "k_pre_uv_seg"],
               "k_uv1_seg": ["k_uv1_segb", "k_uv1_seg"], "k_s2d_fb": ["k_s2d_fb"]}
VALU_SOURCE = ("stored: profiles/pmc_valu_c3.json (rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_*_F64; "
               "tools/gpu.sh valu)")
SIMDS, CLK_GHZ = 1024, 2.4   # MI355X: 256 CUs x 4 SIMDs; peak engine clock


def pmc_group(names, table, key):
    """Per-launch sum of `key` over the kernels one timed interval launches:
    the first name present sets the launch count (its dispatches), every
    present kernel's total is divided by it; None if none is present."""
    ks = table.get("kernels", {}) if table else {}
    present = [n for n in names if n in ks]
    if not present:
        return None
    try:
        n0 = float(ks[present[0]]["dispatches"])
        if key == "traffic_bytes":
            return sum(float(ks[n]["traffic_bytes"]) for n in present) / n0
        return sum(float(ks[n][key]) * float(ks[n]["dispatches"]) for n in present) / n0
    except (KeyError, TypeError, ZeroDivisionError, ValueError):
        return None


def valu_issue(names, ms):
    """roofline.valu_frac: the VALU issue time of one launch (a wave64 FP64
    instruction holds a SIMD 4 cycles -- FP64 78.6 TF = 16 lanes per cycle per
    SIMD -- every other VALU instruction 2) over the measured launch time."""
    p = os.path.join(ROOT, "profiles", "pmc_valu_c3.json")
    try:
        t = json.load(open(p))
    except (OSError, ValueError):
        return {}
    valu, f64 = pmc_group(names, t, "valu"), pmc_group(names, t, "valu_f64")
    if valu is None or f64 is None or not ms or ms <= 0:
        return {}
    cyc = 4.0 * f64 + 2.0 * (valu - f64)
    issue_ms = cyc / SIMDS / (CLK_GHZ * 1e9) * 1e3
    return {"valu_frac": issue_ms / ms, "valu_issue_ms": issue_ms, "valu_insts": valu, "valu_f64_insts": f64,
            "valu_source": VALU_SOURCE}


def trace_top_kernel():
    """The largest kernel per step in the committed C3 kernel trace of the
    current tree (profiles/current_c3_per_step.txt, a copy of the newest
    tools/prof_summary.py table), or None."""
    f = os.path.join(ROOT, "profiles", "current_c3_per_step.txt")
    try:
        rows = [ln for ln in open(f).read().splitlines()[1:] if ln.strip() and not ln.startswith("busy")]
        name = rows[0].rsplit(None, 4)[0]
        return {"trace": os.path.relpath(f, ROOT), "top_kernel": name, "us_per_step": float(rows[0].split()[-3])}
    except (OSError, IndexError, ValueError):
        return None


def pmc_traffic(routine, c3=False):
    try:
        r = _pmc(c3).get("routines", {}).get(routine)
        return None if r is None else float(r["bytes_per_launch"])
    except (KeyError, TypeError, ValueError):
        return None


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":
        _cpu_worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
        return 0
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--timing-steps", type=int, default=3, help="eager steps per routine for the event timings")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("c2", "c3"), default="c3", help="the workload of the primary line")
    ap.add_argument("--no-secondary", "--no-c3", dest="no_secondary", action="store_true",
                    help="skip the secondary workload's object (c2 under the default c3 line)")
    args = ap.parse_args()
    secondary = "c2" if args.workload == "c3" else "c3"
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        return launch_ranks(args, sys.argv[1:])
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # more ranks than GPUs (a rehearsal on a smaller box): ranks share devices
        import torch
        ndev = torch.cuda.device_count()   # does not initialise the GPU
        if ndev > 0:
            local_rank = local_rank % ndev

    # CPU baseline first, before this process touches the GPU
    cpu = {}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu[args.workload] = cpu_baseline(args.workload)
        if not args.no_secondary:
            cpu[secondary] = cpu_baseline(secondary)

    # the JSON line is the only thing on stdout: libraries (RCCL prints a
    # version banner at init) write to fd 1, so point it at stderr for the run
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import romsgpu

    dist = None
    comm = None
    bootstrap = "none (single rank)"
    # ROMS_BENCH_FORCE_COMM=1: take the multi-rank path even at world size 1
    # (RCCL comm + self-addressed exchanges; rehearses the N>1 plumbing)
    force = os.environ.get("ROMS_BENCH_FORCE_COMM") == "1"

    def rccl_comm():
        # the library's own RCCL communicator, its id broadcast through
        # torch.distributed; halos then move by IPC peer writes when the
        # library's init self-test passes, else by RCCL send/recv
        import torch
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(romsgpu.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        return romsgpu.comm_create(bytes(uid.numpy().tobytes()), world, rank, local_rank)

    if world > 1 or force:
        if force:
            os.environ.setdefault("ROMS_GPU_RCCL_SELF", "1")
            if world_env is None:   # a plain single-process run: a world of one over loopback
                import socket
                with socket.socket() as so:
                    so.bind(("127.0.0.1", 0))
                    port = so.getsockname()[1]
                for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"),
                             ("MASTER_PORT", str(port))):
                    os.environ.setdefault(k, v)
        import torch
        import torch.distributed as dist
        # torch.distributed is host plumbing only here (barrier, max over
        # ranks, the communicators' bootstrap): gloo on the CPU; the halo
        # traffic is the library's own (IPC peer writes or RCCL)
        dist.init_process_group("gloo", init_method="env://")
        if force or os.environ.get("ROMS_BENCH_COMM") == "rccl":
            comm, bootstrap = rccl_comm(), "rccl"
        else:
            # default: the host-channel communicator (roms_gpu_comm_create_host),
            # the deployment a Fortran host uses with its MPI_Allgather and the
            # transport the multi-process tests exercise: every halo exchange is
            # an IPC peer write, RCCL is not in the library at all
            def allgather(data):
                t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
                parts = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(parts, t)
                return [bytes(p.numpy().tobytes()) for p in parts]

            comm, bootstrap = romsgpu.comm_create_host(world, rank, allgather, local_rank), "host allgather (gloo)"

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize(local_rank)
            dist.barrier()

    def allmax(x):
        if dist is None:
            return x
        import torch
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def gather(vec):   # every rank's vector, rank order
        if dist is None:
            return [list(vec)]
        import torch
        tt = torch.tensor(vec, dtype=torch.float64)
        parts = [torch.empty_like(tt) for _ in range(world)]
        dist.all_gather(parts, tt)
        return [p.tolist() for p in parts]

    try:
        prim = run_workload(args.workload, romsgpu, comm, rank, world, local_rank, args.steps, args.warmup,
                            args.timing_steps, barrier, allmax, gather=gather)
    except romsgpu.RomsGpuError as e:
        # the host channel carries no RCCL fallback: when the IPC transport
        # fails its set-up or self-test (a collective verdict, so every rank
        # lands here) the ranks re-bootstrap over RCCL, which falls back to
        # RCCL send/recv by itself
        if not bootstrap.startswith("host") or "IPC" not in str(e):
            raise
        romsgpu.comm_destroy(comm)
        comm, bootstrap = rccl_comm(), "rccl (host-channel IPC self-test failed: %s)" % str(e)[:120]
        prim = run_workload(args.workload, romsgpu, comm, rank, world, local_rank, args.steps, args.warmup,
                            args.timing_steps, barrier, allmax, gather=gather)
    prim["config"]["comm_bootstrap"] = bootstrap
    if comm is not None and world > 1 and os.environ.get("ROMS_GPU_XOVERLAP") is None:
        # the deferred-exchange overlap (each producer's 3-D exchange beside
        # the next routine that reads none of its halo; the library's default
        # when every rank has its own GPU, in place when ranks share one,
        # DESIGN.md section 5): the other order A/B'd in the same job
        dflt = prim["config"]["exchange_order"].startswith("deferred")
        os.environ["ROMS_GPU_XOVERLAP"] = "0" if dflt else "1"
        try:
            alt = run_workload(args.workload, romsgpu, comm, rank, world, local_rank, args.steps, args.warmup,
                               args.timing_steps, barrier, allmax, step_only=True)
        finally:
            del os.environ["ROMS_GPU_XOVERLAP"]
        on, off = (prim, alt) if dflt else (alt, prim)
        prim["config"]["exchange_overlap"] = {
            "default": ("on (ranks on distinct GPUs; ROMS_GPU_XOVERLAP=0 keeps every exchange in place)" if dflt else
                        "off (ranks share a GPU; ROMS_GPU_XOVERLAP=1 defers the 3-D exchanges)"),
            "ms_per_step_off": off["ms_per_step"], "ms_per_step_on": on["ms_per_step"],
            "value_on": on["value"], "value_off": off["value"]}
    out = {
        "metric": "grid-cell-updates/sec",
        "value": prim["value"],
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": prim["ms_per_step"],
        "higher_is_better": True,
        "scaling": prim["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (analytic closed basin, SURVEY.md 8(d) C3)" if args.workload == "c3" else
                 "synthetic (analytic Filament+S initial state, ana_grid/ana_init of tests/Filament)"),
        "config": prim["config"],
        "model_seconds_per_wallclock_sec": prim["model_seconds_per_wallclock_sec"],
    }
    for k in ("roofline", "north_star_loop", "roofline_routine", "roofline_step", "routines", "kernel_s2d_fb"):
        out[k] = prim[k]
    if args.workload in cpu:
        out["cpu_baseline"] = cpu[args.workload]
    if not args.no_secondary:
        # the other BASELINE configuration, fewer steps when it is C3 (61 ms each on one GPU)
        c3s = secondary == "c3"
        sec = run_workload(secondary, romsgpu, comm, rank, world, local_rank, min(args.steps, 10) if c3s else args.steps,
                           min(args.warmup, 2) if c3s else args.warmup, min(args.timing_steps, 2) if c3s else
                           args.timing_steps, barrier, allmax, gather=gather)
        sec["metric"] = "grid-cell-updates/sec"
        sec["unit"] = "cell-updates/s"
        sec["data"] = ("synthetic (analytic closed basin, SURVEY.md 8(d) C3)" if c3s else
                       "synthetic (analytic Filament+S initial state, ana_grid/ana_init of tests/Filament)")
        if secondary in cpu:
            sec["cpu_baseline"] = cpu[secondary]
        out[secondary] = sec
    if comm is not None:
        romsgpu.comm_destroy(comm)
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
