import sys, romsgpu
m = romsgpu.Model.from_case(0, 32, 24, 16, sizex=12.8e3, sizey=3.2e3)
for n, c in ((1 << 27, 1), (1 << 22, 32), (1 << 18, 256), (1 << 20, 64)):
    print(n, c, [m.selftest_zero_fill(n, c) for _ in range(3)], flush=True)
m.close()
