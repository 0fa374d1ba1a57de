"""Debug: which routine makes the GPU's t ghost ring differ from the oracle (OBC basin)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "..", "ucla-roms_amd")]
import numpy as np
import oracle, romsgpu
from test_gpu_obc import obc_cfg, make_pair
from test_gpu_parity import copy_state

def where(a, b):
    d = np.abs(a - b)
    if d.max() == 0: return "equal"
    idx = np.argwhere(d > 1e-12 * max(1, np.abs(b).max()))
    return "n=%d first=%s max=%.3e" % (len(idx), idx[:4].tolist(), d.max())

cfg = obc_cfg()
o, m = make_pair(cfg)
print("init t:", where(m.get("t"), o.field("t")))
for s in range(3):
    o.step(1); m.step(1); m.sync()
    print("step", s + 1, "t:", where(m.get("t"), o.field("t")))
m.close()
# routine level from the oracle's state after 3 steps
o, m = make_pair(cfg)
o.step(3)
iic, kstp, knew, nstp, nrhs, nnew = o.tindex()
for routine, corr in [("pre_step3d", 0), ("step3d_t", 1), ("t3dmix", 1)]:
    if corr: nr, nn = 3, 3 - nstp
    else: nr, nn = nstp, 3
    o.set_tindex([iic, kstp, knew, nstp, nr, nn])
    copy_state(o, m)
    m.set_tindex(iic, kstp, knew, nstp, nr, nn, nfast=o.nfast())
    o.call(routine); getattr(m, routine)(); m.sync()
    print(routine, "t:", where(m.get("t"), o.field("t")))
m.close()
