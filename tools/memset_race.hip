// Is hipMemset (null stream) complete before a kernel on a non-blocking stream starts?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void fill(double* p, long n, double v) { for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256) p[q] = v; }
__global__ void count_nonzero(const double* p, long n, unsigned long long* c) {
  unsigned long long k = 0;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256) k += p[q] != 0.0;
  atomicAdd(c, k);
}
int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const long n = 1L << 27;   // 1 GiB
  unsigned long long* c; hipMalloc(&c, 8);
  int bad = 0;
  for (int it = 0; it < 20; it++) {
    double* p; hipMalloc(&p, n * 8);
    fill<<<4096, 256, 0, s>>>(p, n, 1.0); hipStreamSynchronize(s);
    hipMemset(p, 0, n * 8);                 // null stream
    hipMemsetAsync(c, 0, 8, s);
    count_nonzero<<<4096, 256, 0, s>>>(p, n, c);
    unsigned long long h = 0; hipMemcpyAsync(&h, c, 8, hipMemcpyDeviceToHost, s); hipStreamSynchronize(s);
    if (h) bad++;
    printf("iter %d nonzero after memset: %llu\n", it, h);
    hipFree(p);
  }
  printf("RESULT %d of 20 iterations saw stale data\n", bad);
  return 0;
}
