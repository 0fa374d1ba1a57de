// k_diag.hip -- diag_tile (diag.F:58-535) on the device: per-column terms
// (barotropic velocities ub,vb, kinetic energy, barotropic KE, free-surface
// volume, advective/vertical Courant numbers), the reduction by pairs of
// each sum and the first-maximum Courant scan (diag.F loop order j, k=N..1,
// i) in the reference's order, and a blow-up flag.  Five numbers and the
// flag come back to the host, which combines ranks in the reference's tree.
#include <utility>

#include "roms_dev.h"

namespace roms {

__device__ __forceinline__ double diag_ub(const Dev& d, int i, int j, int nstp) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  double ub = (F.Hz[ij + (N - 1) * n2] + F.Hz[ij - 1 + (N - 1) * n2]) * U[ij + (N - 1) * n2];
  for (int k = N - 1; k >= 2; k--) ub = ub + (F.Hz[ij + (k - 1) * n2] + F.Hz[ij - 1 + (k - 1) * n2]) * U[ij + (k - 1) * n2];
  return (ub + (F.Hz[ij] + F.Hz[ij - 1]) * U[ij]) /
         (F.z_w[ij + N * n2] + F.z_w[ij - 1 + N * n2] - F.z_w[ij] - F.z_w[ij - 1]);
}
__device__ __forceinline__ double diag_vb(const Dev& d, int i, int j, int nstp) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  double vb = (F.Hz[ij + (N - 1) * n2] + F.Hz[ij - sj + (N - 1) * n2]) * V[ij + (N - 1) * n2];
  for (int k = N - 1; k >= 2; k--) vb = vb + (F.Hz[ij + (k - 1) * n2] + F.Hz[ij - sj + (k - 1) * n2]) * V[ij + (k - 1) * n2];
  return (vb + (F.Hz[ij] + F.Hz[ij - sj]) * V[ij]) /
         (F.z_w[ij + N * n2] + F.z_w[ij - sj + N * n2] - F.z_w[ij] - F.z_w[ij - sj]);
}

__global__ void __launch_bounds__(256) k_diag(Dev d, Range R, int nstp) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  const double ub0 = diag_ub(d, i, j, nstp), ub1 = diag_ub(d, i + 1, j, nstp);
  const double vb0 = diag_vb(d, i, j, nstp), vb1 = diag_vb(d, i, j + 1, nstp);
  const double v2b = 0.5 * (ub0 * ub0 + ub1 * ub1 + vb0 * vb0 + vb1 * vb1);
  double ke = 0.0;
  double ke2b = 0.5 * (F.z_w[ij + N * n2] - F.z_w[ij]) * v2b;
  double cxm = 0.0, cwm = 0.0, km = -1.0;
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  for (int k = N; k >= 1; k--) {
    const long o = ij + (long)(k - 1) * n2, w = ij + (long)k * n2;
    const double u0 = U[o], u1 = U[o + 1], v0 = V[o], v1 = V[o + sj];
    const double v2 = 0.5 * (u0 * u0 + u1 * u1 + v0 * v0 + v1 * v1);
    const double ciV = d.p.dt * F.rmask[ij] * F.pm[ij] * F.pn[ij] / F.Hz[o];
    const double cw = ciV * (fmax0(F.We[w] + F.Wi[w]) - fmin0(F.We[w - n2] + F.Wi[w - n2]));
    const double cx = cw + ciV * (fmax0(F.FlxU[o + 1]) - fmin0(F.FlxU[o]) + fmax0(F.FlxV[o + sj]) - fmin0(F.FlxV[o]));
    if (cx > cxm) { cxm = cx; cwm = cw; km = (double)k; }
    ke = ke + 0.5 * v2 * F.Hz[o];
  }
  const double dA = F.rmask[ij] / (F.pm[ij] * F.pn[ij]);
  F.s0[ij] = dA * F.z_w[ij + N * n2];
  F.s1[ij] = dA * ke;
  F.s2[ij] = dA * ke2b;
  F.s3[ij] = cxm;
  F.s4[ij] = cwm;
  F.s5[ij] = km;
}

// ---- reduction by pairs on the device (diag.F:409-470 "reduction by
// pairs" of each rank's tile, restated as host pair_reduce in host_init.cpp):
// alternating j- and i-halving passes, each one launch that reads one buffer
// set and writes the other, so every partial sum is formed from the same two
// operands in the same order as the sequential in-place loops. ----
struct Trio {
  double* a[3];
};
__global__ void __launch_bounds__(256) k_pairs_j(const Bounds b, Trio src, Trio dst, int istr, int isize, int jstr,
                                                 int js, int extra) {
  const int i = istr + (int)(blockIdx.x * blockDim.x + threadIdx.x), j = (int)blockIdx.y;   // j = 0..js(+1)
  if (i > istr + isize) return;
  const long t = IJ(b, i, jstr + j);
  if (j <= js) {
    const long s0 = IJ(b, i, jstr + 2 * j), s1 = IJ(b, i, jstr + 2 * j + 1);
#pragma unroll
    for (int q = 0; q < 3; q++) dst.a[q][t] = src.a[q][s0] + src.a[q][s1];
  } else if (extra) {   // odd row count: the last row moves down unchanged
    const long s0 = IJ(b, i, jstr + 2 * j);
#pragma unroll
    for (int q = 0; q < 3; q++) dst.a[q][t] = src.a[q][s0];
  }
}
__global__ void __launch_bounds__(256) k_pairs_i(const Bounds b, Trio src, Trio dst, int istr, int is, int extra,
                                                 int jstr, int jsize) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x), j = jstr + (int)blockIdx.y;   // i = 0..is(+1)
  if (j > jstr + jsize) return;
  const long t = IJ(b, istr + i, j);
  if (i <= is) {
    const long s0 = IJ(b, istr + 2 * i, j), s1 = IJ(b, istr + 2 * i + 1, j);
#pragma unroll
    for (int q = 0; q < 3; q++) dst.a[q][t] = src.a[q][s0] + src.a[q][s1];
  } else if (i == is + 1 && extra) {
    const long s0 = IJ(b, istr + 2 * i, j);
#pragma unroll
    for (int q = 0; q < 3; q++) dst.a[q][t] = src.a[q][s0];
  }
}
// MAX_ADV_CFL first maximum in the reference's scan order (j, then k = N..1,
// then i; strict '>'): per row, the largest Cu; among equal values the
// larger k, then the smaller i.  One block per row, then one block over rows
// (first j on ties).  out[0..4] = Cu_adv, Cu_w, ... and a blow-up flag.
struct CflBest {
  double cx, cw, k;
  int i;
};
__device__ __forceinline__ bool cfl_better(const CflBest& a, const CflBest& b) {   // a precedes b in the scan
  if (a.cx != b.cx) return a.cx > b.cx;
  if (a.k != b.k) return a.k > b.k;
  return a.i < b.i;
}
__global__ void __launch_bounds__(256) k_cfl_rows(const Bounds b, const double* cx, const double* cw, const double* kx,
                                                  double* rcx, double* rcw) {
  __shared__ CflBest sh[256];
  const int j = 1 + (int)blockIdx.x;
  CflBest best{0.0, 0.0, -1.0, 1 << 30};
  for (int i = 1 + (int)threadIdx.x; i <= b.Lm; i += blockDim.x) {
    const long o = IJ(b, i, j);
    const CflBest c{cx[o], cw[o], kx[o], i};
    if (c.cx > 0.0 && (best.k < 0.0 || cfl_better(c, best))) best = c;
  }
  sh[threadIdx.x] = best;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const CflBest o = sh[threadIdx.x + w];
      if (o.k >= 0.0 && (sh[threadIdx.x].k < 0.0 || cfl_better(o, sh[threadIdx.x]))) sh[threadIdx.x] = o;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    rcx[j] = sh[0].k >= 0.0 ? sh[0].cx : 0.0;
    rcw[j] = sh[0].k >= 0.0 ? sh[0].cw : 0.0;
  }
}
__global__ void __launch_bounds__(256) k_diag_final(const Bounds b, const double* rcx, const double* rcw, Trio sums,
                                                    double* out) {
  __shared__ double scx[256], scw[256];
  __shared__ int sj[256];
  double bc = 0.0, bw = 0.0;
  int bj = 1 << 30;
  for (int j = 1 + (int)threadIdx.x; j <= b.Mm; j += blockDim.x)
    if (rcx[j] > bc || (rcx[j] == bc && rcx[j] > 0.0 && j < bj)) { bc = rcx[j]; bw = rcw[j]; bj = j; }
  scx[threadIdx.x] = bc; scw[threadIdx.x] = bw; sj[threadIdx.x] = bj;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const double c = scx[threadIdx.x + w];
      const int jj = sj[threadIdx.x + w];
      if (c > scx[threadIdx.x] || (c == scx[threadIdx.x] && c > 0.0 && jj < sj[threadIdx.x])) {
        scx[threadIdx.x] = c; scw[threadIdx.x] = scw[threadIdx.x + w]; sj[threadIdx.x] = jj;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const long o = IJ(b, 1, 1);
    out[0] = sums.a[0][o];   // avzeta (sum of dA*zeta)
    out[1] = sums.a[1][o];   // ke
    out[2] = sums.a[2][o];   // ke2b
    out[3] = scx[0];
    out[4] = scw[0];
    // blow-up: a non-finite norm is what diag.F's check_line scan catches
    // as "Abnormal termination: BLOWUP" (diag.F:621-633)
    bool bad = false;
    for (int q = 0; q < 5; q++) bad = bad || !(out[q] == out[q]) || fabs(out[q]) > 1.0e300;
    out[5] = bad ? 1.0 : 0.0;
  }
}

void launch_diag(const Dev& d, hipStream_t s, const Tlev& t, double* out) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  (void)hipMemsetAsync(F.s0, 0, (size_t)b.n2 * sizeof(double), s);
  (void)hipMemsetAsync(F.s1, 0, (size_t)b.n2 * sizeof(double), s);
  (void)hipMemsetAsync(F.s2, 0, (size_t)b.n2 * sizeof(double), s);
  Range R{1, b.Lm, 1, b.Mm};
  hipLaunchKernelGGL(k_diag, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nstp);
  if (!out) return;
  // per-row CFL maxima into s6 / s7 (index j), then the pair sums of s0..s2
  hipLaunchKernelGGL(k_cfl_rows, dim3(b.Mm), dim3(256), 0, s, b, F.s3, F.s4, F.s5, F.s6, F.s7);
  Trio A{{F.s0, F.s1, F.s2}}, B{{F.s8, F.s9, F.s3}};
  int istr = 1, jstr = 1, isize = b.Lm - 1, jsize = b.Mm - 1;
  Trio* cur = &A;
  Trio* nxt = &B;
  while (isize > 0 || jsize > 0) {
    if (jsize > 0) {
      int js = (jsize + 1) / 2 - 1;
      const int extra = 2 * js + 1 < jsize;
      hipLaunchKernelGGL(k_pairs_j, dim3((isize + 1 + 255) / 256, js + 1 + extra), dim3(256), 0, s, b, *cur, *nxt,
                         istr, isize, jstr, js, extra);
      std::swap(cur, nxt);
      jsize = js + extra;
    }
    if (isize > 0) {
      int is = (isize + 1) / 2 - 1;
      const int extra = 2 * is + 1 < isize;
      hipLaunchKernelGGL(k_pairs_i, dim3((is + 1 + extra + 255) / 256, jsize + 1), dim3(256), 0, s, b, *cur, *nxt,
                         istr, is, extra, jstr, jsize);
      std::swap(cur, nxt);
      isize = is + extra;
    }
  }
  hipLaunchKernelGGL(k_diag_final, dim3(1), dim3(256), 0, s, b, F.s6, F.s7, *cur, out);
}


// ---- library self-test (roms_gpu_selftest_zero_fill): how many of n doubles
// are not +0.0, counted on stream s (vector atomics) ----
__global__ void __launch_bounds__(256) k_count_nonzero(const double* __restrict__ p, long n,
                                                       unsigned long long* __restrict__ cnt, double v) {
  unsigned long long c = 0;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) c += p[q] != v;
  if (c) atomicAdd(cnt, c);
}
__global__ void __launch_bounds__(256) k_fill_ones(double* __restrict__ p, long n) {
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) p[q] = 1.0;
}
// rows of `width` doubles, `prow` rows per plane: row r of plane p sits at
// p*plane + r*pitch on either side (host planes: compact rows; device planes:
// nx2-pitched rows, plane stride n2 with the wide-halo rows, roms_dev.h)
__global__ void __launch_bounds__(256) k_rows_copy(double* __restrict__ dst, long dpitch, long dplane,
                                                   const double* __restrict__ src, long spitch, long splane,
                                                   long width, long rows, long prow) {
  const long n = width * rows;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) {
    const long r = q / width, c = q - r * width;
    const long pl = r / prow, rr = r - pl * prow;
    dst[pl * dplane + rr * dpitch + c] = src[pl * splane + rr * spitch + c];
  }
}
void launch_rows_copy(double* dst, long dpitch, long dplane, const double* src, long spitch, long splane, long width,
                      long rows, long prow, hipStream_t s) {
  const long n = width * rows, nb = (n + 255) / 256;
  if (n > 0)
    hipLaunchKernelGGL(k_rows_copy, dim3((unsigned)(nb < 65536 ? nb : 65536)), dim3(256), 0, s, dst, dpitch, dplane, src,
                       spitch, splane, width, rows, prow);
}
void launch_fill_ones(double* p, long n, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_ones, dim3(2048), dim3(256), 0, s, p, n);
}
void launch_count_nonzero(const double* p, long n, unsigned long long* cnt, hipStream_t s, double v) {
  hipLaunchKernelGGL(k_count_nonzero, dim3(2048), dim3(256), 0, s, p, n, cnt, v);
}
}  // namespace roms
