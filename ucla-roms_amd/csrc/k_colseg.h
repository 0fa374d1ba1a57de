// k_colseg.h -- segment-partitioned tridiagonal column solves.
//
// The reference solves every vertical system (spline reconstructions,
// implicit diffusion/viscosity: step3d_t_ISO.F:1044-1100, step3d_uv1.F:146-280,
// pre_step3d4S.F:214-263,362-488, compute_vert_*_fluxes.h) with a sequential
// Thomas sweep per column.  On MI355X a lane-per-column sweep over N levels
// is a serial chain of N dependent divisions whose coefficients do not fit in
// registers for deep grids (N = 100: 2 x 101 doubles per lane).
//
// Here a block of S wavefronts owns 64 neighbouring columns (lane = column,
// coalesced rows of 64 doubles per level) and wave s owns a contiguous
// segment of at most KR rows of every column's system:
//   1. each wave eliminates its rows with the segment's lower neighbour x_L
//      kept symbolic:  x_q = D_q + E_q x_L - C_q x_{q+1}      (registers)
//   2. it derives the end-row relations  x = y + alpha x_L + beta x_R  for
//      its first and last rows and publishes them in LDS (6 doubles/lane);
//   3. after one barrier every wave solves the small 2S-unknown reduced
//      system of segment end values for its lane (a two-term recurrence over
//      segments), obtaining its own x_L and x_R;
//   4. and back-substitutes its rows.
// The result equals the sequential solution up to rounding (the elimination
// order differs); for the diagonally dominant systems of the model the
// difference is at the 1e-15 relative level.  Used when N exceeds the
// bit-exact LDS solvers' design point (see roms_shim.cpp: colseg).
#pragma once
#include "k_common.h"

namespace roms {


// Lane mapping: a wavefront holds kSegCW columns x (64/kSegCW) segments, so
// one load instruction still covers 64/kSegCW full 128-B lines, and a block of
// blockDim.y wavefronts holds S = blockDim.y*64/kSegCW segments of kSegCW
// columns.  Small blocks (1-2 wavefronts for N = 50..100) keep several
// independent blocks per CU whose load and solve phases overlap.
constexpr int kSegCW = 16;
struct SegSpan {
  int s, S, c0, n;  // segment index, count, first cell (1-based), cells in segment
  int col;          // column of the lane within the block (0..kSegCW-1)
};
__device__ __forceinline__ SegSpan seg_span(int N) {
  SegSpan r;
  const int t = (int)(threadIdx.x + blockDim.x * threadIdx.y);
  r.col = t % kSegCW;
  r.s = t / kSegCW;
  r.S = (int)(blockDim.x * blockDim.y) / kSegCW;
  const int base = N / r.S, rem = N % r.S;
  r.c0 = 1 + r.s * base + min(r.s, rem);
  r.n = base + (r.s < rem ? 1 : 0);
  return r;
}
// wavefronts per block for N levels: S = ceil(N / kSegRows) rounded up to whole wavefronts
inline int seg_waves(int N) {
  const int per = kCX / kSegCW;
  const int S = (N + kSegRows - 1) / kSegRows;
  return (S + per - 1) / per;
}

// LDS exchange area of one block: 6 end-relation values per (segment, column)
struct SegXchg {
  double v[6][kSegMaxS][kSegCW];
};

template <int KR>
struct SegTri {
  double C[KR], D[KR], E[KR];
  // forward elimination of rows q = 0..n-1; row(q, a, b, c, d): a x_{q-1} + b x_q + c x_{q+1} = d
  template <class RowF>
  __device__ __forceinline__ void eliminate(int n, RowF row) {
    double Cp = 0.0, Dp = 0.0, Ep = 1.0;  // x_{-1} = x_L
#pragma unroll
    for (int q = 0; q < KR; q++) {
      if (q < n) {
        double a, b, c, d;
        row(q, a, b, c, d);
        const double rm = 1.0 / (b - a * Cp);
        C[q] = c * rm;
        D[q] = (d - a * Dp) * rm;
        E[q] = -a * Ep * rm;
        Cp = C[q]; Dp = D[q]; Ep = E[q];
      }
    }
  }
  // publish the first/last-row relations, barrier, reduced solve -> x_L, x_R
  __device__ __forceinline__ void couple(const SegSpan& sp, int n, SegXchg& X, double& xL, double& xR) {
    const int s = sp.s, S = sp.S, l = sp.col;
    double y = 0.0, al = 0.0, be = 0.0, yl = 0.0, all = 0.0, bel = 0.0;
#pragma unroll
    for (int q = KR - 1; q >= 0; q--) {
      if (q < n) {
        if (q == n - 1) { y = D[q]; al = E[q]; be = -C[q]; yl = y; all = al; bel = be; }
        else { y = D[q] - C[q] * y; al = E[q] - C[q] * al; be = -C[q] * be; }
      }
    }
    X.v[0][s][l] = y; X.v[1][s][l] = al; X.v[2][s][l] = be;
    X.v[3][s][l] = yl; X.v[4][s][l] = all; X.v[5][s][l] = bel;
    __syncthreads();
    // F_t = U_t + V_t F_{t+1} (first values), L_t = P_t + Q_t F_{t+1} (last values)
    double U[kSegMaxS], V[kSegMaxS];
    double Pp = 0.0, Qp = 0.0, Ps = 0.0, Qs = 0.0;
#pragma unroll
    for (int t = 0; t < kSegMaxS; t++) {
      if (t < S) {
        const double yf = X.v[0][t][l], af = X.v[1][t][l], bf = X.v[2][t][l];
        const double yL = X.v[3][t][l], aL = X.v[4][t][l], bL = X.v[5][t][l];
        const double rden = 1.0 / (1.0 - af * Qp);
        U[t] = (yf + af * Pp) * rden;
        V[t] = bf * rden;
        const double Pn = yL + aL * Pp + aL * Qp * U[t];
        Qp = aL * Qp * V[t] + bL;
        Pp = Pn;
        if (t == s - 1) { Ps = Pp; Qs = Qp; }
      }
    }
    double Fn = 0.0;  // F_{t+1}
    xL = 0.0; xR = 0.0;
#pragma unroll
    for (int t = kSegMaxS - 1; t >= 0; t--) {
      if (t < S) {
        if (t == s) xR = Fn;
        if (t == s - 1) xL = Ps + Qs * Fn;
        Fn = U[t] + V[t] * Fn;
      }
    }
  }
  // back-substitution; x_q is left in D[q]
  __device__ __forceinline__ void solve(int n, double xL, double xR) {
    double xn = xR;
#pragma unroll
    for (int q = KR - 1; q >= 0; q--) {
      if (q < n) {
        xn = D[q] + E[q] * xL - C[q] * xn;
        D[q] = xn;
      }
    }
  }
};

}  // namespace roms
