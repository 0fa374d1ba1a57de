// PMC calibration for FETCH_SIZE / WRITE_SIZE with the access widths our
// kernels use (MI355X_MICROARCH.md: only 16-B/lane streams are calibrated).
// Each kernel reads exactly NB bytes and writes exactly NB bytes.
//   k_copy8:  one double per lane, grid-stride flat copy
//   k_copy16: one double2 per lane
//   k_col8:   one lane per (i,j) column, walks k with stride n2 (our column kernels)
// usage: ./pmc_calib  (prints the byte counts and per-kernel times)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_copy8(const double* __restrict__ a, double* __restrict__ b, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] + 1.0;
}
__global__ void k_copy16(const double2* __restrict__ a, double2* __restrict__ b, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) { double2 v = a[i]; v.x += 1.0; v.y += 1.0; b[i] = v; }
}
__global__ void k_col8(const double* __restrict__ a, double* __restrict__ b, long n2, int N) {
  long ij = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (ij >= n2) return;
#pragma unroll 8
  for (int k = 0; k < N; k++) b[ij + k * n2] = a[ij + k * n2] + 1.0;
}

int main() {
  const long n2 = 1024L * 1024L, N = 100, n = n2 * N;  // 800 MiB per array
  double *a, *b;
  if (hipMalloc(&a, n * 8) || hipMalloc(&b, n * 8)) { printf("alloc failed\n"); return 1; }
  hipMemset(a, 0, n * 8); hipMemset(b, 0, n * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; rep++) {
    float ms[3];
    hipEventRecord(e0); hipLaunchKernelGGL(k_copy8, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[0], e0, e1);
    hipEventRecord(e0); hipLaunchKernelGGL(k_copy16, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, (const double2*)a, (double2*)b, n / 2);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[1], e0, e1);
    hipEventRecord(e0); hipLaunchKernelGGL(k_col8, dim3((n2 + 63) / 64), dim3(64), 0, 0, a, b, n2, (int)N);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[2], e0, e1);
    printf("rep %d: bytes read %ld written %ld; copy8 %.3f ms (%.0f GB/s) copy16 %.3f ms (%.0f GB/s) col8 %.3f ms (%.0f GB/s)\n",
           rep, n * 8, n * 8, ms[0], 2e-6 * n * 8 / ms[0], ms[1], 2e-6 * n * 8 / ms[1], ms[2], 2e-6 * n * 8 / ms[2]);
  }
  hipFree(a); hipFree(b);
  return 0;
}
