"""Rivers_ana on the reference's 3x2 rank grid on one GPU (in-process
subdomains): per-step diag norms against the golden logs.  Prints the
relative deviation per step (informational; see DESIGN.md rivers note)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ucla-roms_amd"))
sys.path.insert(0, ROOT)
from test_gpu_multirank import run_decomposed  # noqa: E402

keys = ("ke", "ke2b", "cu_adv", "cu_w")
gnu = json.load(open(os.path.join(ROOT, "tests", "golden", "rivers_ana_github_gnu.json")))["rows"]
case = dict(case_id=3, LLm=100, MMm=100, N=10, NT=2, salinity=True, nonlin_eos=True, dt=20.0, ndtfast=30,
            sizex=10e3, sizey=10e3, lmd=True)
npx, npe = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (3, 2)))
_, norms = run_decomposed(case, npx, npe, 20, fields=("zeta",), diag=True)
for s, (g, n) in enumerate(zip(gnu, norms)):
    print(s, " ".join("%s %.2e" % (k, abs(v - float(g[k])) / abs(float(g[k])) if float(g[k]) else abs(v))
                      for k, v in zip(keys, n)))
