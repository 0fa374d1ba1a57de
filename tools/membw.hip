// Streaming-bandwidth probe on the box: what a plain FP64 kernel reaches for
// read-only, copy and 4-read/2-write mixes at 8 B and 16 B per lane, over
// arrays of the C3 size (1028*1028*100 doubles = 845 MB each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) rd4(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                                           const double* __restrict__ d, double* __restrict__ out, long n) {
  double s = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) s += a[i] + b[i] + c[i] + d[i];
  if (s == 1.2345) out[0] = s;
}
__global__ void __launch_bounds__(256) rd4v(const double2* __restrict__ a, const double2* __restrict__ b, const double2* __restrict__ c,
                                            const double2* __restrict__ d, double* __restrict__ out, long n) {
  double s = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
    const double2 x = a[i], y = b[i], z = c[i], w = d[i];
    s += x.x + x.y + y.x + y.y + z.x + z.y + w.x + w.y;
  }
  if (s == 1.2345) out[0] = s;
}
__global__ void __launch_bounds__(256) cp1(const double* __restrict__ a, double* __restrict__ o, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) o[i] = a[i] * 1.0001;
}
__global__ void __launch_bounds__(256) mix42(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                                             const double* __restrict__ d, double* __restrict__ o1, double* __restrict__ o2, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
    const double x = a[i], y = b[i], z = c[i], w = d[i];
    o1[i] = x * y + z;
    o2[i] = z * w - x;
  }
}
// one element per thread, no grid-stride loop (the model kernels' shape)
__global__ void __launch_bounds__(256) mix42_flat(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                                                  const double* __restrict__ d, double* __restrict__ o1, double* __restrict__ o2, long n) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n) return;
  const double x = a[i], y = b[i], z = c[i], w = d[i];
  o1[i] = x * y + z;
  o2[i] = z * w - x;
}

int main() {
  const long n = 1028L * 1028L * 100L;
  std::vector<double*> A(6);
  for (auto& p : A) { CK(hipMalloc(&p, n * 8)); CK(hipMemset(p, 0, n * 8)); }
  double* out; CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto&& launch) {
    launch(); launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 10;
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms / reps, bytes / (ms / reps * 1e-3) / 1e9);
    return 0;
  };
  for (int grid : {1024, 2048, 8192}) {
    char nm[64];
    snprintf(nm, 64, "rd4 8B/lane grid %d", grid);
    run(nm, 4.0 * n * 8, [&] { hipLaunchKernelGGL(rd4, dim3(grid), dim3(256), 0, 0, A[0], A[1], A[2], A[3], out, n); });
    snprintf(nm, 64, "rd4 16B/lane grid %d", grid);
    run(nm, 4.0 * n * 8, [&] { hipLaunchKernelGGL(rd4v, dim3(grid), dim3(256), 0, 0, (const double2*)A[0], (const double2*)A[1], (const double2*)A[2], (const double2*)A[3], out, n / 2); });
    snprintf(nm, 64, "copy 8B grid %d", grid);
    run(nm, 2.0 * n * 8, [&] { hipLaunchKernelGGL(cp1, dim3(grid), dim3(256), 0, 0, A[0], A[4], n); });
    snprintf(nm, 64, "mix 4r2w 8B grid %d", grid);
    run(nm, 6.0 * n * 8, [&] { hipLaunchKernelGGL(mix42, dim3(grid), dim3(256), 0, 0, A[0], A[1], A[2], A[3], A[4], A[5], n); });
  }
  run("mix 4r2w flat 1/thread", 6.0 * n * 8, [&] { hipLaunchKernelGGL(mix42_flat, dim3((n + 255) / 256), dim3(256), 0, 0, A[0], A[1], A[2], A[3], A[4], A[5], n); });
  return 0;
}
