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
struct SegSpan {
  int s, S, c0, n;  // segment index, count, first cell (1-based), cells in segment
  int col;          // column of the lane within the block row (0..kSegCW-1)
  int row;          // row j of the lane within the block (threadIdx.z)
  int l;            // the lane's column slot in the block's LDS exchange (col + kSegCW*row)
};
// CW: columns per segment (kSegCW for the column solvers; k_omega_seg has
// its own, ROMS_GPU_OMEGA_CW)
template <int CW = kSegCW>
__device__ __forceinline__ SegSpan seg_span(int N) {
  SegSpan r;
  const int t = (int)(threadIdx.x + blockDim.x * threadIdx.y);
  r.col = t % CW;
  r.row = (int)threadIdx.z;
  r.l = r.col + CW * r.row;
  r.s = t / CW;
  r.S = (int)(blockDim.x * blockDim.y) / CW;
  const int base = N / r.S, rem = N % r.S;
  r.c0 = 1 + r.s * base + min(r.s, rem);
  r.n = base + (r.s < rem ? 1 : 0);
  return r;
}
// With one segment per wavefront (CW = 64) the segment index, first cell
// and row count are wave-uniform: readfirstlane tells the compiler so, and
// the level offsets derived from them live in SGPRs (buffer-load soffsets).
template <int CW = kSegCW>
__device__ __forceinline__ void seg_uniform(SegSpan& r) {
  static_assert(CW == kCX, "seg_uniform needs one segment per wavefront");
  r.s = __builtin_amdgcn_readfirstlane(r.s);
  r.c0 = __builtin_amdgcn_readfirstlane(r.c0);
  r.n = __builtin_amdgcn_readfirstlane(r.n);
}
// wavefronts per block for N levels: S = ceil(N / kSegRows) rounded up to whole wavefronts
template <int CW = kSegCW>
inline int seg_waves(int N) {
  const int per = kCX / CW;
  const int S = (N + kSegRows - 1) / kSegRows;
  return (S + per - 1) / per;
}

// Logical block of a segment-solver launch.  ord 0: xcd_tile() order (x
// fastest); ord 1: z (direction / tracer) fastest, then y (j), then x, so the
// blocks that share a column's arrays (both directions, all tracers) and the
// j-neighbour rows run back to back on one XCD; ord 2: z, then x, then y;
// ord 3: z, then x within a group of xg blocks, then y, then the group, so the
// blocks resident on an XCD at one time cover xg x (resident/xg/gz) columns
// blocks of both directions and share their i- and j-neighbour lines in L2.
__device__ __forceinline__ uint3 seg_tile(int ord, int xg = 4) {
  uint3 t = xcd_tile();
  if (ord == 0) return t;
  const unsigned gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const unsigned L = t.x + gx * (t.y + gy * t.z);
  t.z = L % gz;
  if (ord == 1) { t.y = (L / gz) % gy; t.x = L / (gz * gy); }
  else if (ord == 2) { t.x = (L / gz) % gx; t.y = L / (gz * gx); }
  else {
    const unsigned G = (unsigned)xg < gx ? (unsigned)xg : gx;
    const unsigned Lp = L / gz, nfull = gx / G, inf = nfull * G * gy;
    if (Lp < inf) {
      const unsigned rem = Lp % (G * gy);
      t.x = (Lp / (G * gy)) * G + rem % G;
      t.y = rem / G;
    } else {
      const unsigned Gl = gx - nfull * G, rem = Lp - inf;
      t.x = nfull * G + rem % Gl;
      t.y = rem / Gl;
    }
  }
  return t;
}

// LDS exchange area of one block: 6 end-relation values per (segment, column)
struct SegXchg {
  double v[6][kSegMaxS][kSegCW * kSegJMax];
};

// Every per-row loop below is straight-line code over all KR rows: rows
// q >= n (the segment is shorter than KR) are computed on clamped inputs and
// discarded by selects, never skipped by a lane-dependent branch.  Branches
// split the unrolled loops into basic blocks, and the compiler then waited
// for every row's loads before the next row's (one s_waitcnt vmcnt(0) per
// load); straight-line rows let it issue the loads of many rows back to back.
// The live rows keep their expressions and order: results are unchanged.
// Every segment of a launch has at least kSegNMin rows (seg_rows_ok, checked
// on the host before a segment solver is chosen), so rows q < kSegNMin are
// live in every wave and their selects fold away at compile time; only the
// last rows pay for them.  With 16-column blocks the segment count is rounded
// up to a multiple of four (four segments per wavefront, seg_count): N = 88..104
// gives 8 segments of 11-13 rows; N = 64..87 would give 8 segments of 8-10
// rows, fails the check and runs the sequential column solvers on global
// scratch instead (ROMS_GPU_COLSEG=1 cannot force it).
__device__ __forceinline__ bool seg_live(int q, int n) { return q < kSegNMin || q < n; }
__device__ __forceinline__ bool seg_last(int q, int n) { return q >= kSegNMin - 1 && q == n - 1; }

// A load whose value feeds only one arm of a select is sunk by the compiler
// into a branch of its own, and every such branch waits for its load alone:
// 14 serialized round trips per segment in the tracer flux rows (measured in
// the disassembly).  Loading every row first and pinning the values after
// all loads are issued keeps them one batch; the select is unchanged.
__device__ __forceinline__ void pin(double& x) { __asm__ volatile("" : "+v"(x)); }

#ifndef ROMS_SEG_LOAD_GROUP
#define ROMS_SEG_LOAD_GROUP 5
#endif
constexpr int kSegLoadGroup = ROMS_SEG_LOAD_GROUP;
#ifndef ROMS_SEG_COUPLE_GROUP
#define ROMS_SEG_COUPLE_GROUP 8
#endif
constexpr int kSegCoupleGroup = ROMS_SEG_COUPLE_GROUP;

// 1/x in the elimination and coupling recurrences, the serial dependency
// chain of every segment solve (one reciprocal per row): the hardware
// reciprocal refined by two Newton steps -- 5 dependent FP64 operations
// against the IEEE division's 10 -- agrees with 1/x to the last bit or one
// ulp (the solvers already differ from the reference's sequential Thomas at
// ~1e-15, k_colseg.h header); C3 pre_step3d, step3d_uv1 and step3d_t
// 0.08-0.15 ms faster each (profiles/r6_rc_seg_rcp_ab.txt).
// -DROMS_SEG_FASTRCP=0 builds the IEEE division.
#ifndef ROMS_SEG_FASTRCP
#define ROMS_SEG_FASTRCP 1
#endif
__device__ __forceinline__ double seg_rcp(double x) {
#if ROMS_SEG_FASTRCP
  double y = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-x, y, 1.0);
  return __builtin_fma(y, e, y);
#else
  return 1.0 / x;
#endif
}

// the rows' diffusion coefficients 2 dt K / (Hz_k + Hz_k+1) (step3d_t_ISO.F
// :1044-1065, step3d_uv1.F:146-170, pre_step3d4S.F:214-230,362-380): a times
// seg_rcp(b), 6 instructions instead of the division's 10, within an ulp of
// a / b; C3 pre_step3d, step3d_uv1 and step3d_t 0.05-0.07 ms faster each
// (profiles/r6_rc_seg_rcp_ab.txt).  -DROMS_SEG_FASTDIV=0: a / b.
#ifndef ROMS_SEG_FASTDIV
#define ROMS_SEG_FASTDIV 1
#endif
#if ROMS_SEG_FASTDIV
#define SEG_DIV(a, b) ((a) * seg_rcp(b))
#else
#define SEG_DIV(a, b) ((a) / (b))
#endif

template <int KR>
struct SegTri {
  double C[KR], D[KR], E[KR];
  // forward elimination of rows q = 0..n-1; row(q, a, b, c, d): a x_{q-1} + b x_q + c x_{q+1} = d
  // (row() is called for every q < KR and must be free of side effects)
  template <int G = kSegLoadGroup, class RowF>
  __device__ __forceinline__ void eliminate(int n, RowF row) {
    double Cp = 0.0, Dp = 0.0, Ep = 1.0;  // x_{-1} = x_L
#pragma unroll
    for (int q = 0; q < KR; q++) {
      double a, b, c, d;
      row(q, a, b, c, d);
      const double rm = seg_rcp(b - a * Cp);
      const double Cq = c * rm, Dq = (d - a * Dp) * rm, Eq = -a * Ep * rm;
      const bool live = seg_live(q, n);
      C[q] = live ? Cq : 0.0;
      D[q] = live ? Dq : 0.0;
      E[q] = live ? Eq : 0.0;
      Cp = C[q]; Dp = D[q]; Ep = E[q];
      // rows' loads run at most a group ahead of the elimination (register pressure)
      if (q % G == G - 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
  // publish the first/last-row relations, barrier, reduced solve -> x_L, x_R
  __device__ __forceinline__ void couple(const SegSpan& sp, int n, SegXchg& X, double& xL, double& xR) {
    const int s = sp.s, S = sp.S, l = sp.l;
    double y = 0.0, al = 0.0, be = 0.0, yl = 0.0, all = 0.0, bel = 0.0;
#pragma unroll
    for (int q = KR - 1; q >= 0; q--) {
      const bool last = seg_last(q, n), live = seg_live(q, n);
      const double yn = D[q] - C[q] * y, aln = E[q] - C[q] * al, ben = -C[q] * be;
      y = last ? D[q] : (live ? yn : y);
      al = last ? E[q] : (live ? aln : al);
      be = last ? -C[q] : (live ? ben : be);
      yl = last ? D[q] : yl;
      all = last ? E[q] : all;
      bel = last ? -C[q] : bel;
    }
    X.v[0][s][l] = y; X.v[1][s][l] = al; X.v[2][s][l] = be;
    X.v[3][s][l] = yl; X.v[4][s][l] = all; X.v[5][s][l] = bel;
    __syncthreads();
    // F_t = U_t + V_t F_{t+1} (first values), L_t = P_t + Q_t F_{t+1} (last
    // values), F_S = 0.  Every lane of a column runs the same forward
    // recurrence; the segment's own (U_s, V_s) and the composition of the
    // maps of the segments above it, F_{s+1} = ga + gb F_{t+1}, are carried
    // as running values, so F_{s+1} = ga at the end and no S-long arrays of
    // U_t, V_t are live at the register peak (32 VGPRs at S = 8).
    double Pp = 0.0, Qp = 0.0, Ps = 0.0, Qs = 0.0, Us = 0.0, Vs = 0.0, ga = 0.0, gb = 1.0;
#pragma unroll
    for (int t = 0; t < kSegMaxS; t++) {
      if (t < S) {
        const double yf = X.v[0][t][l], af = X.v[1][t][l], bf = X.v[2][t][l];
        const double yL = X.v[3][t][l], aL = X.v[4][t][l], bL = X.v[5][t][l];
        const double rden = seg_rcp(1.0 - af * Qp);
        const double Ut = (yf + af * Pp) * rden;
        const double Vt = bf * rden;
        Us = t == s ? Ut : Us;
        Vs = t == s ? Vt : Vs;
        const double gan = ga + gb * Ut, gbn = gb * Vt;
        ga = t > s ? gan : ga;
        gb = t > s ? gbn : gb;
        const double Pn = yL + aL * Pp + aL * Qp * Ut;
        Qp = aL * Qp * Vt + bL;
        Pp = Pn;
        Ps = t == s - 1 ? Pp : Ps;
        Qs = t == s - 1 ? Qp : Qs;
      }
      // LDS reads of at most kSegCoupleGroup segments ahead (register peak)
      if (t % kSegCoupleGroup == kSegCoupleGroup - 1) __builtin_amdgcn_sched_barrier(0);
    }
    xR = ga;                        // F_{s+1}
    xL = Ps + Qs * (Us + Vs * ga);  // L_{s-1} from F_s
  }
  // back-substitution; x_q is left in D[q]
  __device__ __forceinline__ void solve(int n, double xL, double xR) {
    double xn = xR;
#pragma unroll
    for (int q = KR - 1; q >= 0; q--) {
      const double v = D[q] + E[q] * xL - C[q] * xn;
      const bool live = seg_live(q, n);
      xn = live ? v : xn;
      D[q] = live ? v : D[q];
    }
  }
};

// ---- parabolic-spline interface values FC(0:N) of one column, segment form
// (compute_vert_tracer_fluxes.h, compute_vert_rhs_uv_terms.h; sequential forms
// tracer_spline_lds / uv_vert_flux_lds).  Rows: FC(0)+FC(1) = 2 f(1);
// w(r+1) FC(r-1) + 2(w(r)+w(r+1)) FC(r) + w(r) FC(r+1) = 3(w(r) f(r+1) + w(r+1) f(r));
// FC(N-1)+FC(N) = 2 f(N).  On entry w[q], f[q] hold the layer weights (Hz, or
// the 4-point u/v average) and values at cell c0-1+q (clamped to 1..N),
// q = 0..n+1 and 0..n.  On exit fc[q] = FC(c0-1+q), q = 0..n. ----
template <int KR>
__device__ __forceinline__ void spline_fc_seg(const SegSpan& sg, int N, SegXchg& X, const double (&w)[KR + 1],
                                              const double (&f)[KR], double (&fc)[KR]) {
  const int c0 = sg.c0, n = sg.n;
  const int ns = n + (sg.s == sg.S - 1 ? 1 : 0);   // the last segment also owns interface N
  SegTri<KR> T;
  T.eliminate(ns, [&](int q, double& a, double& bb, double& c, double& dd) {
    const int r = c0 - 1 + q;
    const int q1 = q + 1 < KR ? q + 1 : KR - 1;   // f[q+1] of a row that can be live
    const double ai = w[q + 1], bi = 2.0 * (w[q] + w[q + 1]), ci = w[q];
    const double di = 3.0 * (w[q] * f[q1] + w[q + 1] * f[q]);
    a = r == 0 ? 0.0 : (r == N ? 1.0 : ai);
    bb = (r == 0 || r == N) ? 1.0 : bi;
    c = r == 0 ? 1.0 : (r == N ? 0.0 : ci);
    dd = r == 0 ? 2.0 * f[1] : (r == N ? 2.0 * f[q] : di);
  });
  double xL, xR;
  T.couple(sg, ns, X, xL, xR);
  T.solve(ns, xL, xR);
#pragma unroll
  for (int q = 0; q < KR; q++) fc[q] = seg_live(q, ns) ? T.D[q] : xR;
}

// SPLINE_UV advective flux of a u (dir 0) / v (dir 1) column at interfaces
// r = c0-1+q, q = 0..n (0 at the bottom and the surface): FC(r) * 0.5 * the
// 4-point We average with the reference's masked curvature correction.
// row(q, L, hz, hzm, u) is called in the load phase for q = 0..KR (cells
// c0-1+q clamped to 1..N; rows outside the segment are dead) with the
// column's Hz, its (i-1)/(j-1) neighbour's Hz and u(nrhs) there (0 at
// q = KR), unconditionally (a branch on n would split the straight-line
// loads).  k_pre_uv_seg forms its u(indx) terms from them, k_uv1_seg keeps
// the Hz pairs for its viscosity rows.  Without UV_ADV the hook is not called.
struct NoSplineRow {
  __device__ __forceinline__ void operator()(int, long, double, double, double) const {}
};
template <int KR, class RowF = NoSplineRow>
__device__ __forceinline__ void uv_spline_seg(const Dev& d, const SegSpan& sg, SegXchg& X, long ij, int nrhs, int dir,
                                              double (&fl)[KR], RowF row = RowF()) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, c0 = sg.c0, n = sg.n;
  if (!d.p.uv_adv) {  // no UV_ADV (uniform over the grid: the skipped coupling barrier is too)
#pragma unroll
    for (int q = 0; q < KR; q++) fl[q] = 0.0;
    return;
  }
  const long n2 = b.n2, s = dir == 0 ? 1 : b.nx2;
  const double* __restrict__ Uv = (dir == 0 ? F.u : F.v) + (long)(nrhs - 1) * b.n3 + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ We = F.We + ij;
  const double* mask = dir == 0 ? F.umask : F.vmask;
  double dc[KR + 1], uu[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {   // all rows (clamped levels): straight-line loads
    const long L = (long)(min(max(c0 - 1 + q, 1), N) - 1) * n2;
    const double h0 = Hz[L], h1 = Hz[L - s];
    dc[q] = 0.5625 * (h0 + h1) - 0.0625 * (Hz[L + s] + Hz[L - 2 * s]);
    if (q < KR) uu[q] = Uv[L];
    row(q, L, h0, h1, q < KR ? uu[q] : 0.0);
    // groups of kSegLoadGroup rows: their loads issue together, the next
    // group's wait (without the barrier all 5 (KR+1) loads were hoisted and spilled)
    if (q % kSegLoadGroup == kSegLoadGroup - 1) __builtin_amdgcn_sched_barrier(0);
  }
  spline_fc_seg<KR>(sg, N, X, dc, uu, fl);
  const double m1 = mask[ij + s], m0 = mask[ij - s];
  // every row's 4-point We average formed unconditionally, in load groups,
  // and pinned before the selects (see pin above: sunk into per-row
  // branches the 14 rows' loads were 14 serialized memory round trips)
  double wf[KR];
#pragma unroll
  for (int q = 0; q < KR; q++) {
    const long w = (long)min(max(c0 - 1 + q, 1), N - 1) * n2;
    wf[q] = We[w] + We[w - s] - 0.125 * ((We[w + s] - We[w]) * m1 - (We[w - s] - We[w - 2 * s]) * m0);
    if (q % kSegLoadGroup == kSegLoadGroup - 1) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int q = 0; q < KR; q++) pin(wf[q]);
#pragma unroll
  for (int q = 0; q < KR; q++) {
    const int r = c0 - 1 + q;
    fl[q] = (r == 0 || r == N) ? 0.0 : fl[q] * 0.5 * wf[q];
  }
}

// uv_spline_seg with buffer loads (the segment solvers' buffer forms): the
// lane's column and its (i-1)/(j-1), (i+1)/(j+1), (i-2)/(j-2) neighbours in
// four VGPR offsets, each row's level in an SGPR (seg_uniform).  row(q, so,
// h0, h1, u) gets the row's level byte offset in place of the element offset.
// Same expressions and order: bitwise equal to uv_spline_seg.
struct NoSplineRowB {
  __device__ __forceinline__ void operator()(int, unsigned, double, double, double) const {}
};
// UNI: the segment is wave-uniform (seg_uniform) and level offsets go in
// the SGPR soffset; else they are added to the VGPR offset.
template <int KR, bool UNI = true, class RowF = NoSplineRowB>
__device__ __forceinline__ void uv_spline_segb(const Dev& d, const SegSpan& sg, SegXchg& X, long ij, int nrhs, int dir,
                                               double (&fl)[KR], RowF row = RowF()) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, c0 = sg.c0, n = sg.n;
  if (!d.p.uv_adv) {
#pragma unroll
    for (int q = 0; q < KR; q++) fl[q] = 0.0;
    return;
  }
  const long s = dir == 0 ? 1 : b.nx2;
  const unsigned lv = (unsigned)b.n2 * 8u, vo = (unsigned)ij * 8u, ds = (unsigned)s * 8u;
  const unsigned vm = vo - ds, vp = vo + ds, vm2 = vo - 2u * ds;
  const BufF64 Uv((dir == 0 ? F.u : F.v) + (long)(nrhs - 1) * b.n3), Hz(F.Hz), We(F.We);
  const double* mask = dir == 0 ? F.umask : F.vmask;
  auto LD = [&](const BufF64& B, unsigned v, unsigned l) { return UNI ? B.ld(v, l) : B.ld(v + l, 0u); };
  double dc[KR + 1], uu[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {
    const unsigned L = (unsigned)(min(max(c0 - 1 + q, 1), N) - 1) * lv;
    const double h0 = LD(Hz, vo, L), h1 = LD(Hz, vm, L);
    dc[q] = 0.5625 * (h0 + h1) - 0.0625 * (LD(Hz, vp, L) + LD(Hz, vm2, L));
    if (q < KR) uu[q] = LD(Uv, vo, L);
    row(q, L, h0, h1, q < KR ? uu[q] : 0.0);
    if (q % kSegLoadGroup == kSegLoadGroup - 1) __builtin_amdgcn_sched_barrier(0);
  }
  spline_fc_seg<KR>(sg, N, X, dc, uu, fl);
  const double m1 = mask[ij + s], m0 = mask[ij - s];
  double wf[KR];
#pragma unroll
  for (int q = 0; q < KR; q++) {
    const unsigned w = (unsigned)min(max(c0 - 1 + q, 1), N - 1) * lv;
    const double we0 = LD(We, vo, w), wem = LD(We, vm, w);
    wf[q] = we0 + wem - 0.125 * ((LD(We, vp, w) - we0) * m1 - (wem - LD(We, vm2, w)) * m0);
    if (q % kSegLoadGroup == kSegLoadGroup - 1) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int q = 0; q < KR; q++) pin(wf[q]);
#pragma unroll
  for (int q = 0; q < KR; q++) {
    const int r = c0 - 1 + q;
    fl[q] = (r == 0 || r == N) ? 0.0 : fl[q] * 0.5 * wf[q];
  }
}

// SPLINE_TS advective flux FC(r)*We(r) of a tracer column at interfaces
// r = c0-1+q, q = 0..n (0 at the bottom and the surface); hz, tt as w, f of
// spline_fc_seg.
template <int KR>
__device__ __forceinline__ void tracer_spline_seg(const SegSpan& sg, int N, long n2, SegXchg& X,
                                                  const double (&hz)[KR + 1], const double (&tt)[KR],
                                                  const double* __restrict__ We, double (&fl)[KR]) {
  spline_fc_seg<KR>(sg, N, X, hz, tt, fl);
  double we[KR];
#pragma unroll
  for (int q = 0; q < KR; q++) we[q] = We[(long)min(max(sg.c0 - 1 + q, 1), N - 1) * n2];
#pragma unroll
  for (int q = 0; q < KR; q++) pin(we[q]);
#pragma unroll
  for (int q = 0; q < KR; q++) {
    const int r = sg.c0 - 1 + q;
    fl[q] = (r == 0 || r == N) ? 0.0 : fl[q] * we[q];
  }
}

// Block prologue of the momentum column kernels: grid z = direction (0: u at
// i >= istrU, 1: v at j >= jstrV), kSegCW columns x blockDim.z rows j per block.
// Lanes outside the column range (i or j) solve a clamped duplicate column
// (they take part in the barriers) and store nothing.
// v columns (Params::seg_vtile, kSegCW = 64): a wavefront's 64 lanes hold a
// 16 x 4 tile of columns instead of one row of 64.  The v stencils read the
// rows j-2..j+1 of Hz and We and j-1 of Hz_fwd/bak, Akv, Wi; with one row per
// wavefront every one of those rows is another block's row and comes from
// HBM again (no L2 reuse at ~1 MB of columns per block), with four rows per
// wavefront the tile's 7 (4) distinct rows serve its 16 (8) row reads.  A
// 16-wide row is one 128-B line at the device row pitch (roms_dev.h).  The
// blocks of the two directions enumerate their own tiles; a block whose
// tile lies outside the range is idle (returns before any barrier).
// (16 x 4 at 64 columns; the 8 x 4 tiles of 32-column segments measured
// much slower, C3 58.3 vs 53.9 ms, r5_r_vtile_cw32_ab.txt, so segments of 32
// columns keep their v columns in rows)
constexpr int kVTX = 16, kVTY = 4;
struct SegCol {
  int i, j, dir;
  bool act, idle;
};
__device__ __forceinline__ bool seg_vtile_on(const Dev& d) { return d.p.seg_vtile && kSegCW == kVTX * kVTY; }
__device__ __forceinline__ void seg_uv_col(const Dev& d, const Range& R, const uint3& bI, const SegSpan& sg,
                                           SegCol& c) {
  const Bounds& b = d.b;
  c.dir = (int)bI.z;
  const int ilo = c.dir == 0 ? b.istrU : b.istr;
  const int jlo = c.dir == 1 ? (b.jstrV > R.j0 ? b.jstrV : R.j0) : R.j0;
  int iu, ju;
  if (c.dir == 1 && seg_vtile_on(d)) {
    const int ti0 = tile_i0(R.i0);
    const int ntx = (R.i1 - ti0 + kVTX) / kVTX, nty = (R.j1 - R.j0 + kVTY) / kVTY;
    const int t = (int)bI.x + (int)gridDim.x * (int)bI.y;
    c.idle = t >= ntx * nty;
    iu = ti0 + (t % ntx) * kVTX + sg.col % kVTX;
    ju = R.j0 + (t / ntx) * kVTY + sg.col / kVTX;
  } else {
    iu = tile_i0(R.i0) + (int)bI.x * kSegCW + sg.col;
    ju = R.j0 + (int)bI.y * (int)blockDim.z + sg.row;
    c.idle = R.j0 + (int)bI.y * (int)blockDim.z > R.j1;
  }
  c.act = iu >= ilo && iu <= R.i1 && ju >= jlo && ju <= R.j1;
  c.i = iu < ilo ? ilo : (iu > R.i1 ? R.i1 : iu);
  c.j = ju < jlo ? jlo : (ju > R.j1 ? R.j1 : ju);
}
inline dim3 seg_grid_of(const Range& R, int nz, int jrows = 1) {
  return dim3((R.i1 - tile_i0(R.i0) + kSegCW) / kSegCW, (R.j1 - R.j0 + jrows) / jrows, nz);
}
// the momentum kernels' grid: enough blocks in (x, y) for the u rows and for
// the v tiles (seg_uv_col)
inline dim3 seg_uv_grid(const Dev& d, const Range& R, int jrows) {
  dim3 g = seg_grid_of(R, 2, jrows);
  if (d.p.seg_vtile && kSegCW == kVTX * kVTY && jrows == 1) {
    const long nvt = (long)((R.i1 - tile_i0(R.i0) + kVTX) / kVTX) * ((R.j1 - R.j0 + kVTY) / kVTY);
    const long gy = (nvt + g.x - 1) / g.x;
    if (gy > (long)g.y) g.y = (unsigned)gy;
  }
  return g;
}

}  // namespace roms
