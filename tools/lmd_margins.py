"""Print the measured margins behind tests/test_gpu_lmd.py (GPU box)."""
import json, os, sys, threading
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ucla-roms_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import oracle, romsgpu
from test_gpu_lmd import make_pair, _cfg, LMD_OUT
from test_gpu_parity import copy_state, interior, relerr
keys = ("ke", "ke2b", "cu_adv", "cu_w")
gnu = json.load(open(os.path.join(ROOT, "tests/golden/pipes_ana_github_gnu.json")))["rows"]
cfg = _cfg("pipes"); o, m = make_pair(cfg)
for s in range(1, 21):
    o.step(); m.step(); d = m.diag(); on = o.norms()
    rg = max(abs(v - float(gnu[s][k])) / abs(float(gnu[s][k])) for k, v in zip(keys, d) if float(gnu[s][k]) != 0)
    ro = max(abs(v - w) / abs(w) for v, w in zip(d, on) if w != 0)
    print("step %2d  gpu-vs-gnu %.2e  gpu-vs-oracle(3x2 diag) %.2e" % (s, rg, ro))
for f in LMD_OUT + ["u", "t", "zeta"]:
    print("%-6s rel %.2e" % (f, relerr(interior(m.get(f), 100, 100), interior(o.field(f), 100, 100))))
print("hbls range", float(o.field("hbls").max()), "ghat min", float(o.field("ghat").min()))
m.close()
for case in ("basin_lmd", "pipes"):
    cfg = _cfg(case); o, m = make_pair(cfg); o.step(4)
    iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
    o.set_tindex([iic, kstp, knew, nstp, nstp, 3]); copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nstp, 3, nfast=o.nfast())
    o.L.or_lmd_vmix(o.h, nstp); m.lmd_vmix(nstp); m.sync()
    print(case, {f: "%.1e" % relerr(interior(m.get(f), cfg.LLm, cfg.MMm), interior(o.field(f), cfg.LLm, cfg.MMm)) for f in LMD_OUT})
    m.close()
# 3x2 GPU run vs golden digits
case = dict(case_id=2, LLm=100, MMm=100, N=10, NT=2, salinity=True, nonlin_eos=True, dt=60.0, ndtfast=30,
            sizex=30e3, sizey=30e3, lmd=True)
norms, errs = [], []
def work(rank):
    try:
        h = romsgpu.comm_create_local(77, 6, rank)
        mm = romsgpu.Model.from_case(np_xi=3, np_eta=2, comm=h, rank=rank, **case)
        d = mm.diag()
        if rank == 0: norms.append(d)
        for _ in range(20):
            mm.step(); d = mm.diag()
            if rank == 0: norms.append(d)
        mm.close(); romsgpu.comm_destroy(h)
    except Exception as e:
        errs.append(repr(e))
th = [threading.Thread(target=work, args=(r,)) for r in range(6)]
[t.start() for t in th]; [t.join(240) for t in th]
print("errs", errs)
ndig = 0
for s, (r, g) in enumerate(zip(gnu, norms)):
    have = [("%23.16E" % v).strip() for v in g]; want = [r[k] for k in keys]
    same = sum(a == b for a, b in zip(have, want)); ndig += same
    if s in (0, 1, 5, 10, 20): print(s, have, want)
print("3x2 exact-match cells: %d / %d" % (ndig, 4 * len(norms)))
