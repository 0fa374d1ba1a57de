"""Allocation-race probe (roms_gpu_selftest_zero_fill) on the current or an
A/B library (ROMS_GPU_LIB): bad element counts per repetition."""
import romsgpu
m = romsgpu.Model.from_case(0, 32, 24, 16, sizex=12.8e3, sizey=3.2e3)
for n, c in ((1 << 18, 256), (1 << 16, 512), (1 << 20, 64), (1 << 14, 1024)):
    print(n, c, [m.selftest_zero_fill(n, c) for _ in range(10)], flush=True)
m.close()
