"""Per-GPU compute of the C3 basin at the subdomain sizes of bench.py's strong
scaling (1024x1024, 512x1024, 512x512, 256x512 for N = 1, 2, 4, 8 GPUs),
each run as a single-rank closed basin on one GPU: no exchange, so the
figures bound what N GPUs can reach from kernel efficiency alone.  Prints one
JSON line per size: ms per step (graph replay), the routine times, and the
compute-only efficiency t(1024^2) / (N x t(size)).
usage: python tools/subdomain_probe.py [STEPS [NGPU]] (NGPU: that size only)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ucla-roms_amd"))
import romsgpu  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N, DT, DX, NDTFAST, NT = 100, 300.0, 2.0e3, 60, 2
sizes = [(1024, 1024, 1), (512, 1024, 2), (512, 512, 4), (256, 512, 8)]
if len(sys.argv) > 2:
    sizes = [z for z in sizes if z[2] == int(sys.argv[2])]
t1 = None
for L, M, ngpu in sizes:
    m = romsgpu.Model.from_case(romsgpu.CASE_BASIN, L, M, N, NT, salinity=True, nonlin_eos=True,
                                lmd=romsgpu.LMD_ICELAND, dt=DT, ndtfast=NDTFAST, sizex=DX * L, sizey=DX * M)
    m.step(2)
    m.sync()
    ms = m.time_steps(STEPS) / STEPS
    rout = {}
    for r in ("rho_eos", "omega", "prsgrd", "pre_step3d", "step3d_uv1", "step2d", "step3d_t", "lmd_vmix"):
        t, n = m.time_routine(r, 1)
        rout[r] = round(t * n, 3)   # ms per step
    m.close()
    if t1 is None:
        t1 = ms
    print(json.dumps({"grid": [L, M, N], "gpus_of_1024sq": ngpu, "ms_per_step": round(ms, 3),
                      "compute_only_efficiency": round(t1 / (ngpu * ms), 3), "routine_ms_per_step": rout}), flush=True)
