// Row-alignment probe: a 64x4-tiled 5-point stencil over C3-sized FP64
// arrays (1024 x 1024 interior, 100 levels; 4 inputs, 2 outputs), as the
// per-level model kernels read them, for three device layouts:
//   pitch 1028, offset 0   the reference layout (row j of element i at
//                          (i+1) + (j+1)*1028): i = 1 sits 16 B into a row
//                          whose start moves 32 B per row against 128-B lines
//   pitch 1040, offset 0   rows padded to 128 B, i = 1 still 16 B in
//   pitch 1040, offset 14  rows padded and the base shifted: i = 1 on a line
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) sten(const double* __restrict__ a, const double* __restrict__ b,
                                            const double* __restrict__ c, const double* __restrict__ d,
                                            double* __restrict__ o1, double* __restrict__ o2, int L, int M, int P, long n2) {
  const int i = 1 + blockIdx.x * 64 + threadIdx.x, j = 1 + blockIdx.y * 4 + threadIdx.y;
  if (i > L || j > M) return;
  const long o = (long)(i + 1) + (long)(j + 1) * P + (long)blockIdx.z * n2;
  const double x = a[o - 1] + a[o] + a[o + 1] + a[o - P] + a[o + P];
  const double y = b[o - 1] + b[o] + b[o + 1] + b[o - P] + b[o + P];
  const double z = c[o] * d[o] + c[o + 1] * d[o + P];
  o1[o] = x * z + y;
  o2[o] = y * z - x;
}
// one lane per (i,j) column walking 100 levels (the column kernels' shape)
__global__ void __launch_bounds__(64) col(const double* __restrict__ a, const double* __restrict__ b,
                                          const double* __restrict__ c, const double* __restrict__ d,
                                          double* __restrict__ o1, int L, int M, int P, long n2, int N) {
  const int i = 1 + blockIdx.x * 64 + threadIdx.x, j = 1 + blockIdx.y;
  if (i > L || j > M) return;
  long o = (long)(i + 1) + (long)(j + 1) * P;
  double s = 0.0;
  for (int k = 0; k < N; k++, o += n2) {
    s = s * 0.5 + a[o] + b[o] * c[o] - d[o - P];
    o1[o] = s;
  }
}

int main() {
  const int L = 1024, M = 1024, N = 100;
  struct Lay { int P, off; const char* name; };
  const Lay lays[] = {{1028, 0, "pitch 1028 off 0 (current)"}, {1040, 0, "pitch 1040 off 0"}, {1040, 14, "pitch 1040 off 14 (i=1 aligned)"}};
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; rep++)
  for (const Lay& y : lays) {
    const long n2 = (long)y.P * (M + 4), n = n2 * N + 64;
    std::vector<double*> A(6), B(6);
    for (int q = 0; q < 6; q++) { CK(hipMalloc(&B[q], n * 8)); CK(hipMemset(B[q], 0, n * 8)); A[q] = B[q] + y.off; }
    auto time = [&](auto&& launch) -> float {
      launch(); launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; r++) launch();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      return ms / 10;
    };
    const float ts = time([&] { hipLaunchKernelGGL(sten, dim3(L / 64, M / 4, N), dim3(64, 4), 0, 0, A[0], A[1], A[2], A[3], A[4], A[5], L, M, y.P, n2); });
    const float tc = time([&] { hipLaunchKernelGGL(col, dim3(L / 64, M), dim3(64), 0, 0, A[0], A[1], A[2], A[3], A[4], L, M, y.P, n2, N); });
    const double alg = (double)L * M * N * 8;
    printf("%-34s stencil %7.3f ms (%6.0f GB/s alg.)   column %7.3f ms (%6.0f GB/s alg.)\n", y.name, ts, 6 * alg / ts / 1e6, tc, 5 * alg / tc / 1e6);
    for (double* p : B) CK(hipFree(p));
  }
  return 0;
}
