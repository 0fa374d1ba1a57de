"""Per-block phase timeline of the fused fast step (k_s2d_fb) on a C3-like
closed basin of L x M x 100: needs a library built with -DROMS_S2D_PROBE
(tools/build_variant.sh s2dprobe -DROMS_S2D_PROBE, loaded with ROMS_GPU_LIB),
whose kernel stores the shader clock at each phase boundary into ptide.
Prints the median and 90th-percentile cycles of every phase over the blocks
of the last fast step.  usage: python tools/s2d_phase_probe.py L M"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ucla-roms_amd"))
import romsgpu
L, M = int(sys.argv[1]), int(sys.argv[2])
m = romsgpu.Model.from_case(romsgpu.CASE_BASIN, L, M, 100, 2, salinity=True, nonlin_eos=True, lmd=romsgpu.LMD_ICELAND,
                            dt=300.0, ndtfast=60, sizex=2e3 * L, sizey=2e3 * M)
m.step(2)
m.sync()
p = m.get("ptide").ravel()
m.close()
nb = ((L + 2 + 15) // 64 + 1) * ((M + 2 + 3) // 4 + 1)
t = p[:nb * 8].reshape(nb, 8)
ok = (t[:, 0] > 0) & (t[:, 7] > 0)
t = t[ok]
d = np.diff(t, axis=1)
names = ["loads issued", "loads landed + window in LDS", "DU/DV", "zeta part", "zetabc", "P3 (stores issued)", "fold + drain"]
print("blocks", int(ok.sum()), "of", nb, "total cycles median %.0f p10 %.0f p90 %.0f" % tuple(np.percentile(t[:, 7] - t[:, 0], [50, 10, 90])))
for k, n in enumerate(names):
    print("%-32s median %7.0f p90 %7.0f cycles" % (n, np.median(d[:, k]), np.percentile(d[:, k], 90)))
