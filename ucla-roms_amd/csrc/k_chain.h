// k_chain.h -- column kernels whose vertical work is sums or scans over k
// (step3d_uv2, set_HUV1): one column is spread over 4 lanes.
//
// A wavefront holds 16 neighbouring columns x 4 vertical segments of KL
// levels (lane = 16*g + column, g = 0 the bottom segment), so every load
// instruction covers four 128-B rows, and a lane keeps its KL levels of the
// column's values in registers between the passes the reference makes over
// the column.  A vertical sum (or running sum) is a chain over the segments:
// the first segment in the reference's k order accumulates its levels in
// order, hands its running value to the next segment's lane by a shuffle,
// and so on, so every sum keeps the reference's operation order and the
// results are bit-identical to a one-lane-per-column sweep.  A 256-thread
// block is a 16 x 4 patch of columns.  The form pays where a column is swept
// several times with little arithmetic per level (uv2: four passes -> one);
// a chained running sum with several dependent adds per level at 2 waves per
// SIMD (omega, measured: 2.62 vs 1.50 ms at C3) does not.
#pragma once
#include "roms_dev.h"

namespace roms {

constexpr int kChainCW = 16;   // columns per wavefront
constexpr int kChainG = 4;     // segments (lanes) per column

struct ChainLane {
  int col, g;    // column in the wavefront's row, segment (0 = bottom)
  int i, j;      // the lane's column (unclamped)
  int lo, nk;    // first level of the segment and its number of levels
  bool in;       // i >= R.i0: the aligned first tile's lanes left of the range store nothing
};
template <int KL>
__device__ __forceinline__ ChainLane chain_lane(const Range& R, const uint3& bI, int N) {
  ChainLane c;
  const int l = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
  c.col = l & (kChainCW - 1);
  c.g = l / kChainCW;
  c.i = tile_i0(R.i0) + (int)bI.x * kChainCW + c.col;
  c.in = c.i >= R.i0;
  c.j = R.j0 + (int)bI.y * 4 + w;
  c.lo = 1 + c.g * KL;
  c.nk = max(0, min(N, c.lo + KL - 1) - c.lo + 1);
  return c;
}
inline dim3 chain_grid_of(const Range& R) {
  return dim3((R.i1 - tile_i0(R.i0) + kChainCW) / kChainCW, (R.j1 - R.j0 + 4) / 4);
}
// segment length for N levels: ceil(N / 4) rounded up to a compiled size
inline int chain_kl(int N) {
  const int kl = (N + kChainG - 1) / kChainG;
  return kl <= 5 ? 5 : kl <= 13 ? 13 : kl <= 25 ? 25 : 0;
}

// Top-down chain (k = N..1): segments g = 3..0 in turn run body(s1, s2) on
// the running values handed down from the segment above; on return every
// lane of the column holds the totals.
template <class Body>
__device__ __forceinline__ void chain_down(const ChainLane& c, double& s1, double& s2, Body&& body) {
  s1 = 0.0; s2 = 0.0;
#pragma unroll
  for (int st = kChainG - 1; st >= 0; st--) {
    const double in1 = __shfl_down(s1, kChainCW), in2 = __shfl_down(s2, kChainCW);
    if (c.g == st) {
      if (st < kChainG - 1) { s1 = in1; s2 = in2; }
      body(s1, s2);
    }
  }
  s1 = __shfl(s1, c.col);
  s2 = __shfl(s2, c.col);
}
// Bottom-up chain (k = 1..N): segments g = 0..3 in turn run body(s) on the
// running value handed up from the segment below; on return every lane of
// the column holds the total.
template <class Body>
__device__ __forceinline__ void chain_up(const ChainLane& c, double& s, Body&& body) {
  s = 0.0;
#pragma unroll
  for (int st = 0; st < kChainG; st++) {
    const double in = __shfl_up(s, kChainCW);
    if (c.g == st) {
      if (st > 0) s = in;
      body(s);
    }
  }
  s = __shfl(s, (kChainG - 1) * kChainCW + c.col);
}

}  // namespace roms
