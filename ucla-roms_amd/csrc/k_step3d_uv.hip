// k_step3d_uv.hip -- corrector momentum: step3d_uv1 (step3d_uv1.F:23-534),
// visc3d (visc3d_S.F:18-131) and the 2-D/3-D coupling step3d_uv2
// (step3d_uv2.F:18-786, IMPLICIT_BOTTOM_DRAG branch).
#include <vector>

#include "k_colseg.h"
#include "k_chain.h"

namespace roms {

void launch_uv_horiz(const Dev& d, hipStream_t s, int nrhs, int up);

#ifndef ROMS_UV1_PF
#define ROMS_UV1_PF 8
#endif
constexpr int kUv1PF = ROMS_UV1_PF;
// ---- step3d_uv1: implicit viscosity with implicit bottom drag r_D, result
// stored as Hz*u in u(nnew); rufrc = vertical integral of ru + stresses ----
template <class C>
__device__ __forceinline__ void uv1_col(const Dev& d, int i, int j, int dir, int nnew, int nrhs, const C& A,
                                        const C& B) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double dt = d.p.dt;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const long s = dir == 0 ? 1 : b.nx2;
  // spline sweeps with their prefetch rings, and a ring in the Thomas sweep
  // below: 1.16 -> 0.90 ms at C2 (profiles/r2_m_uv1_ring_ab.txt; the spline
  // rings alone 1.61 ms, the Thomas ring alone 0.96 at depth 4 and 1.39 at
  // depth 8).  ROMS_UV1_PF=0 builds the plain form.
  uv_vert_flux_lds<(kUv1PF > 0)>(d, ij, nrhs, dir, A, B);
  double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
  double* __restrict__ rr = (dir == 0 ? F.ru : F.rv) + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Akv = F.Akv + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = dt * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  auto hz = [&](int k) { return Hz[(long)(k - 1) * n2]; };
  auto hzm = [&](int k) { return Hz[(long)(k - 1) * n2 - s]; };
  auto rk = [&](int k) {  // final ru(k): vertical advection added, stored back
    const long o = (long)(k - 1) * n2;
    const double r = uv_rr_update(rr[o], A, k);
    rr[o] = r;
    return r;
  };
  double FCk = 2.0 * dt * (Akv[(long)(N - 1) * n2] + Akv[(long)(N - 1) * n2 - s]) /
               (hz(N) + hzm(N) + hz(N - 1) + hzm(N - 1));
  double WCk = DC0 * 0.5 * (Wi[(long)(N - 1) * n2] + Wi[(long)(N - 1) * n2 - s]);
  double cff = 1.0 / (0.5 * (hz(N) + hzm(N)) + FCk - fmin0(WCk));
  double CFk = cff * (FCk + fmax0(WCk));
  double DCk1 = cff * (Un[(long)(N - 1) * n2] + DC0 * rk(N) + dt * sstr);
  A[N] = DCk1;
  B[N - 1] = CFk;
#if ROMS_UV1_PF > 0
  // Forward elimination through a ring of kUv1PF iterations' raw loads,
  // refilled ahead of each iteration's ru store (the store of level k would
  // otherwise hold back the ru load of level k-1: same array, offsets the
  // compiler cannot separate); same expressions and order as the plain loop.
  struct Lv { double ak, aks, wi, wis, hl, hlm, un, r; };
  auto load = [&](int k) {   // iteration k: w-level k-1, rho levels k-1 (Hz) and k (u, ru)
    k = k < 2 ? 2 : k;
    const long o = (long)(k - 1) * n2, l = o - n2;
    return Lv{Akv[o], Akv[o - s], Wi[o], Wi[o - s], Hz[l], Hz[l - s], Un[o], rr[o]};
  };
  double hK = hz(N - 1), hKm = hzm(N - 1);
  auto iter = [&](int k, const Lv& v) {
    const double FCl = 2.0 * dt * (v.ak + v.aks) / (hK + hKm + v.hl + v.hlm);
    const double WCl = DC0 * 0.5 * (v.wi + v.wis);
    cff = 1.0 / (0.5 * (hK + hKm) + FCl - fmin0(WCl) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
    const double CFl = cff * (FCl + fmax0(WCl));
    const double r = uv_rr_update(v.r, A, k);
    rr[(long)(k - 1) * n2] = r;
    const double DCk = cff * (v.un + DC0 * r + DCk1 * (FCk - fmin0(WCk)));
    B[k - 1] = CFl;
    A[k] = DCk;
    DCk1 = DCk; FCk = FCl; WCk = WCl; CFk = CFl;
    hK = v.hl; hKm = v.hlm;
  };
  constexpr int PF = kUv1PF;
  Lv ring[PF];
#pragma unroll
  for (int q = 0; q < PF; q++) ring[q] = load(N - 1 - q);
  int k1 = N - 1;
  for (; k1 - PF + 1 >= 2; k1 -= PF) {
#pragma unroll
    for (int q = 0; q < PF; q++) {
      const Lv v = ring[q];
      ring[q] = load(k1 - q - PF);
      iter(k1 - q, v);
    }
  }
#pragma unroll
  for (int q = 0; q < PF; q++)
    if (k1 - q >= 2) iter(k1 - q, ring[q]);
#else
#pragma unroll 8
  for (int k = N - 1; k >= 2; k--) {
    const double FCl = 2.0 * dt * (Akv[(long)(k - 1) * n2] + Akv[(long)(k - 1) * n2 - s]) /
                       (hz(k) + hzm(k) + hz(k - 1) + hzm(k - 1));
    const double WCl = DC0 * 0.5 * (Wi[(long)(k - 1) * n2] + Wi[(long)(k - 1) * n2 - s]);
    cff = 1.0 / (0.5 * (hz(k) + hzm(k)) + FCl - fmin0(WCl) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
    const double CFl = cff * (FCl + fmax0(WCl));
    const double DCk = cff * (Un[(long)(k - 1) * n2] + DC0 * rk(k) + DCk1 * (FCk - fmin0(WCk)));
    B[k - 1] = CFl;
    A[k] = DCk;
    DCk1 = DCk; FCk = FCl; WCk = WCl; CFk = CFl;
  }
#endif
  const double rD = F.r_D[ij], rDm = F.r_D[ij - s];
  const double r1 = rk(1);
  double dc = (Un[0] + DC0 * r1 + DCk1 * (FCk - fmin0(WCk))) /
              (0.5 * (hz(1) + hzm(1)) + 0.5 * dt * (rD + rDm) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
  Un[0] = dc * 0.5 * (hz(1) + hzm(1));
  const double dmdn = dir == 0 ? F.dm_u[ij] * F.dn_u[ij] : F.dm_v[ij] * F.dn_v[ij];
  double frc = r1 + dmdn * (sstr - 0.5 * (rDm + rD) * dc);
#pragma unroll 8
  for (int k = 2; k <= N; k++) {
    dc = A[k] + B[k - 1] * dc;
    Un[(long)(k - 1) * n2] = dc * 0.5 * (hz(k) + hzm(k));
    frc = frc + rr[(long)(k - 1) * n2];
  }
  if (dir == 0) F.rufrc[ij] = frc;
  else F.rvfrc[ij] = frc;
}

template <class C>
__global__ void __launch_bounds__(64) k_uv1(Dev d, Range R, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<C>(2, d.b.N);
  const Bounds& b = d.b;
  const long ij = IJ(b, i, j);
  const C A = ColMake<C>::at(d, 0, (int)bI.z, ij), B = ColMake<C>::at(d, 1, (int)bI.z, ij);
  if (bI.z == 0) {
    if (i >= b.istrU && i <= b.iend) uv1_col(d, i, j, 0, nnew, nrhs, A, B);
  } else {
    if (j >= b.jstrV) uv1_col(d, i, j, 1, nnew, nrhs, A, B);
  }
}

// ---- register-resident variant of k_uv1 for a compile-time depth NN: one
// of the two coefficient columns (the spline FC / Thomas DC, NN+1 doubles per
// lane) lives in VGPRs, the other (CF) in LDS.  Every level loop is fully
// unrolled, so each column element is a fixed register.  Half the LDS per
// wave doubles the resident waves (6 per CU against 3 for the two-slot LDS
// form at N = 50; both columns in VGPRs would spill).  Same expressions and
// order as uv_vert_flux_lds<false> + uv1_col, so results are bit-identical. ----
constexpr int kUv1Chunk = 5;
template <int NN>
__global__ void __launch_bounds__(64, 2) k_uv1_reg(Dev d, Range R, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<ColLds>(1, NN);
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int dir = (int)bI.z;
  if (dir == 0 ? !(i >= b.istrU && i <= b.iend) : !(j >= b.jstrV)) return;
  constexpr int N = NN;
  const double dt = d.p.dt;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const long s = dir == 0 ? 1 : b.nx2;
  double A[N + 1];               // registers
  const ColLds B = col_lds(0, N);  // LDS: 26 KB per wave at N = 50
  uv_spline_reg<N>(d, ij, nrhs, dir, A, B);
  double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
  double* __restrict__ rr = (dir == 0 ? F.ru : F.rv) + ij;
  const double* Hz = F.Hz + ij;
  __asm__ volatile("" : "+v"(Hz));   // no reuse of the spline sweep's Hz loads
  const double* __restrict__ Akv = F.Akv + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = dt * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  auto hz = [&](int k) { return Hz[(long)(k - 1) * n2]; };
  auto hzm = [&](int k) { return Hz[(long)(k - 1) * n2 - s]; };
  // pre-pass, k ascending, in chunks whose loads all precede their ru stores
  // (inside the elimination every later ru load had to wait behind the
  // previous level's store, may-alias): final ru(k) stored back, the Thomas
  // right-hand side v(k) = u(nnew) + DC0*ru(k) kept in A[k-1] (A[k-1] is last
  // read by ru(k)); ru(1) kept for rufrc.
  double r1 = 0.0;
#pragma unroll
  for (int k0 = 1; k0 <= N; k0 += kUv1Chunk) {
    double r_[kUv1Chunk], un_[kUv1Chunk];
#pragma unroll
    for (int q = 0; q < kUv1Chunk; q++) {
      const long o = (long)(k0 + q - 1) * n2;
      r_[q] = rr[o]; un_[q] = Un[o];
    }
#pragma unroll
    for (int q = 0; q < kUv1Chunk; q++) {
      const int k = k0 + q;
      const double r = k == 1 ? r_[q] - A[1] : r_[q] - A[k] + A[k - 1];
      rr[(long)(k - 1) * n2] = r;
      if (k == 1) r1 = r;
      A[k - 1] = un_[q] + DC0 * r;
    }
  }
  double FCk = 2.0 * dt * (Akv[(long)(N - 1) * n2] + Akv[(long)(N - 1) * n2 - s]) /
               (hz(N) + hzm(N) + hz(N - 1) + hzm(N - 1));
  double WCk = DC0 * 0.5 * (Wi[(long)(N - 1) * n2] + Wi[(long)(N - 1) * n2 - s]);
  double cff = 1.0 / (0.5 * (hz(N) + hzm(N)) + FCk - fmin0(WCk));
  double CFk = cff * (FCk + fmax0(WCk));
  double DCk1 = cff * (A[N - 1] + dt * sstr);
  A[N] = DCk1;
  B[N - 1] = CFk;
#pragma unroll
  for (int k = N - 1; k >= 2; k--) {
    const double FCl = 2.0 * dt * (Akv[(long)(k - 1) * n2] + Akv[(long)(k - 1) * n2 - s]) /
                       (hz(k) + hzm(k) + hz(k - 1) + hzm(k - 1));
    const double WCl = DC0 * 0.5 * (Wi[(long)(k - 1) * n2] + Wi[(long)(k - 1) * n2 - s]);
    cff = 1.0 / (0.5 * (hz(k) + hzm(k)) + FCl - fmin0(WCl) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
    const double CFl = cff * (FCl + fmax0(WCl));
    const double DCk = cff * (A[k - 1] + DCk1 * (FCk - fmin0(WCk)));
    B[k - 1] = CFl;
    A[k] = DCk;
    DCk1 = DCk; FCk = FCl; WCk = WCl; CFk = CFl;
    ROMS_LEVEL_FENCE_AT(k);
  }
  const double rD = F.r_D[ij], rDm = F.r_D[ij - s];
  double dc = (A[0] + DCk1 * (FCk - fmin0(WCk))) /
              (0.5 * (hz(1) + hzm(1)) + 0.5 * dt * (rD + rDm) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
  Un[0] = dc * 0.5 * (hz(1) + hzm(1));
  const double dmdn = dir == 0 ? F.dm_u[ij] * F.dn_u[ij] : F.dm_v[ij] * F.dn_v[ij];
  double frc = r1 + dmdn * (sstr - 0.5 * (rDm + rD) * dc);
  // reload Hz and ru in the back-substitution instead of keeping the N levels
  // of the elimination sweep live in registers (laundered base pointers: the
  // compiler may not forward the earlier loads / stores across the sweep)
  const double* Hz2 = Hz;
  const double* rr2 = rr;
  __asm__ volatile("" : "+v"(Hz2), "+v"(rr2));
#pragma unroll
  for (int k = 2; k <= N; k++) {
    dc = A[k] + B[k - 1] * dc;
    const long o = (long)(k - 1) * n2;
    Un[o] = dc * 0.5 * (Hz2[o] + Hz2[o - s]);
    frc = frc + rr2[o];
    ROMS_LEVEL_FENCE_AT(k);
  }
  if (dir == 0) F.rufrc[ij] = frc;
  else F.rvfrc[ij] = frc;
}

// ---- segment-partitioned variant of k_uv1 (k_colseg.h) for deep grids:
// block = kSegCW columns x S segments, grid z = direction.  Spline advection and
// the implicit viscosity are each one partitioned tridiagonal system with the
// rows of uv1_col; the final ru(k) of every level go to LDS, from where the
// first segment forms rufrc/rvfrc in the reference's k = 1..N order. ----
// ru(k) of the block's columns for rufrc: dynamic LDS, level k-1 of lane
// slot l at roms_smem[(k-1)*ncol + l], ncol = kSegCW*blockDim.z.
//
// kLds (UV_ADV): the spline phase's Hz loads serve the viscosity rows too --
// the Hz of the column and of its (i-1)/(j-1) neighbour at the segment's
// cells c0-1..c0+KR-1, exactly the levels the viscosity rows read -- kept in
// dynamic LDS ([2][KR+1][threads], 123 KB at N = 100) instead of reloaded
// (at C3 these reloads missed L2: 2 of the v column's 17 array passes).  The
// ru(k) for rufrc then stay in the lane's registers and the sum runs as a
// chain through the waves in k order (wave s adds its levels to wave s-1's
// running sum, handed over in LDS between barriers): the reference's
// operations in its order, bit-identical.
template <bool kLds>
__global__ void __launch_bounds__(kSegBlock * kSegJMax, 2) k_uv1_seg(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  __shared__ double Lf[kLds ? kSegMaxS : 1][kSegCW * kSegJMax];   // kLds: rufrc running sums
  double* const Sr = roms_smem;   // !kLds (see above)
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double dt = d.p.dt;
  const SegSpan sg = seg_span(N);
  SegCol col;
  seg_uv_col(d, R, bI, sg, col);
  if (col.idle) return;   // uniform over the block
  const int ncol = kSegCW * (int)blockDim.z;
  const int dir = col.dir;
  const bool act = col.act;
  const long n2 = b.n2, ij = IJ(b, col.i, col.j), s = dir == 0 ? 1 : b.nx2;
  const int c0 = sg.c0, n = sg.n;
  auto cell = [&](int k) { return (long)(min(max(k, 1), N) - 1) * n2; };   // rho level k (clamped)
  const int nthr = (int)(blockDim.x * blockDim.y * blockDim.z);
  const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  double* const Sh = roms_smem + tid;                             // kLds: Hz(c0-1+q) at Sh[q*nthr]
  double* const Shm = roms_smem + (long)(KR + 1) * nthr + tid;    //       its neighbour's at Shm[q*nthr]
  double fl[KR];
  if constexpr (kLds) {
    uv_spline_seg<KR>(d, sg, X, ij, nrhs, dir, fl, [&](int q, long, double h0, double h1, double) {
      Sh[q * nthr] = h0;
      Shm[q * nthr] = h1;
    });
  } else {
    uv_spline_seg<KR>(d, sg, X, ij, nrhs, dir, fl);
  }
  __builtin_amdgcn_sched_barrier(0);   // the viscosity phase's loads stay out of the spline phase
  double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
  const double* __restrict__ rr = (dir == 0 ? F.ru : F.rv) + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Akv = F.Akv + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = dt * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  // right-hand sides first: ru(k) with the vertical advection (uv_rr_update)
  // for rufrc (LDS, or kLds: registers) -- the updated ru itself is dead
  // after this routine (the next step's prsgrd overwrites it, prsgrd.F:293),
  // so it is not stored -- and dd = u(nnew) + DC0*ru
  // (kLds: only ru(k) here; dd is formed in the elimination rows, u(nnew)
  // loaded there -- one register array less)
  double rhs[kLds ? 1 : KR], rk[kLds ? KR : 1];
#pragma unroll
  for (int p = 0; p < KR; p++) {
    const int k = c0 + p;
    const long o = cell(k);
    const double r = k == 1 ? rr[o] - fl[1] : rr[o] - fl[p + 1 < KR ? p + 1 : KR - 1] + fl[p];
    if constexpr (kLds) {
      rk[p] = r;
    } else {
      if (p < n) Sr[(k - 1) * ncol + sg.l] = r;
      const double v = Un[o] + DC0 * r;
      rhs[p] = k == N ? v + dt * sstr : v;
    }
  }
  double hz[kLds ? 1 : KR + 1], hzm[kLds ? 1 : KR + 1];   // !kLds: Hz(c0-1+q) of the column and of its (i-1) / (j-1) neighbour
  if constexpr (!kLds) {
#pragma unroll
    for (int q = 0; q < KR + 1; q++) {
      const long L = cell(c0 - 1 + q);
      hz[q] = Hz[L];
      hzm[q] = Hz[L - s];
    }
  }
  // kLds: the LDS reads go through an opaque offset, so the compiler cannot
  // forward the spline phase's stored values and keep them in registers
  // across the spline solve instead (it did: 256 VGPRs and spills)
  int tl = tid;
  __asm__ volatile("" : "+v"(tl));
  auto HZ = [&](int q) { if constexpr (kLds) return roms_smem[tl + q * nthr]; else return hz[q]; };
  auto HZM = [&](int q) { if constexpr (kLds) return roms_smem[(KR + 1 + q) * nthr + tl]; else return hzm[q]; };
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q (0 at the bottom and the surface)
    const int r = c0 - 1 + q;
    const long w = (long)min(max(r, 1), N - 1) * n2;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * dt * (Akv[w] + Akv[w - s]), HZ(qa) + HZM(qa) + HZ(q) + HZM(q));
    const double wv = DC0 * 0.5 * (Wi[w] + Wi[w - s]);
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  const double rD = F.r_D[ij], rDm = F.r_D[ij - s];
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.eliminate(n, [&](int p, double& a, double& bb, double& cc, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    const int k = c0 + p;
    a = -(fcl + fmax0(wcl));
    cc = -(fcu - fmin0(wcu));
    const double b1 = 0.5 * (HZ(p + 1) + HZM(p + 1)) + 0.5 * dt * (rD + rDm) + fcu + fmax0(wcu);
    const double bk = 0.5 * (HZ(p + 1) + HZM(p + 1)) + fcl - fmin0(wcl) + fcu + fmax0(wcu);
    bb = k == 1 ? b1 : bk;
    if constexpr (kLds) {
      const double v = Un[cell(k)] + DC0 * rk[p];
      dd = k == N ? v + dt * sstr : v;
    } else {
      dd = rhs[p];
    }
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);   // its barrier also publishes Sr
  T.solve(n, xL, xR);
  const double dmdn = dir == 0 ? F.dm_u[ij] * F.dn_u[ij] : F.dm_v[ij] * F.dn_v[ij];
  if constexpr (kLds) {
    // rufrc = ru(1) + dmdn*(sstr - r_D*u(1)) + ru(2) + ... + ru(N), wave by wave
    const int S = sg.S, sl = sg.l;
    for (int t = 0; t < S; t++) {
      if (sg.s == t) {
        double frc;
        if (t == 0) frc = rk[0] + dmdn * (sstr - 0.5 * (rDm + rD) * T.D[0]);
        else frc = Lf[t - 1][sl] + rk[0];
#pragma unroll
        for (int p = 1; p < KR; p++) frc = p < n ? frc + rk[p] : frc;
        Lf[t][sl] = frc;
      }
      __syncthreads();
    }
    if (!act) return;
#pragma unroll
    for (int p = 0; p < KR; p++)
      if (p < n) Un[cell(c0 + p)] = T.D[p] * 0.5 * (HZ(p + 1) + HZM(p + 1));
    if (sg.s == 0) {
      if (dir == 0) F.rufrc[ij] = Lf[S - 1][sl];
      else F.rvfrc[ij] = Lf[S - 1][sl];
    }
  } else {
    if (!act) return;
#pragma unroll
    for (int p = 0; p < KR; p++)
      if (p < n) Un[cell(c0 + p)] = T.D[p] * 0.5 * (hz[p + 1] + hzm[p + 1]);
    if (sg.s == 0) {
      double frc = Sr[sg.l] + dmdn * (sstr - 0.5 * (rDm + rD) * T.D[0]);
      for (int k = 2; k <= N; k++) frc = frc + Sr[(k - 1) * ncol + sg.l];
      if (dir == 0) F.rufrc[ij] = frc;
      else F.rvfrc[ij] = frc;
    }
  }
}

// ---- k_uv1_seg<true> with buffer loads/stores (Params::seg_buf bit 32):
// wave-uniform level offsets in SGPRs (seg_uniform), the lane's column and
// its neighbour in VGPR offsets; PF: u(nnew) of the segment's rows loaded
// with the spline phase's inputs.  Same expressions and order: bitwise equal
// to k_uv1_seg<true>. ----
// UNI false: the level offsets in the VGPR offset (no seg_uniform, no SGPR pressure)
template <bool PF, bool UNI = true>
__global__ void __launch_bounds__(kSegBlock * kSegJMax, 2) k_uv1_segb(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  __shared__ double Lf[kSegMaxS][kSegCW * kSegJMax];   // rufrc running sums
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double dt = d.p.dt;
  SegSpan sg = seg_span(N);
  constexpr bool kU = UNI && kSegCW == kCX;   // scalar level offsets need one segment per wavefront
  if constexpr (kU) seg_uniform(sg);
  SegCol col;
  seg_uv_col(d, R, bI, sg, col);
  if (col.idle) return;   // uniform over the block
  const int dir = col.dir;
  const bool act = col.act;
  const long n2 = b.n2, ij = IJ(b, col.i, col.j), s = dir == 0 ? 1 : b.nx2;
  const int c0 = sg.c0, n = sg.n;
  const unsigned lv = (unsigned)n2 * 8u, vo = (unsigned)ij * 8u, vm = vo - (unsigned)s * 8u;
  auto lev = [&](int k) { return (unsigned)(min(max(k, 1), N) - 1) * lv; };   // rho level k (clamped)
  const int nthr = (int)(blockDim.x * blockDim.y * blockDim.z);
  const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  double* const Sh = roms_smem + tid;                             // Hz(c0-1+q) at Sh[q*nthr]
  double* const Shm = roms_smem + (long)(KR + 1) * nthr + tid;    // its neighbour's at Shm[q*nthr]
  const BufF64 Un((dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3);
  auto LD = [&](const BufF64& B, unsigned v, unsigned l) { return kU ? B.ld(v, l) : B.ld(v + l, 0u); };
  double fl[KR], un[PF ? KR : 1];
  if constexpr (PF) {
#pragma unroll
    for (int p = 0; p < KR; p++) un[p] = LD(Un, vo, lev(c0 + p));
  }
  uv_spline_segb<KR, kU>(d, sg, X, ij, nrhs, dir, fl, [&](int q, unsigned, double h0, double h1, double) {
    Sh[q * nthr] = h0;
    Shm[q * nthr] = h1;
  });
  __builtin_amdgcn_sched_barrier(0);   // the viscosity phase's loads stay out of the spline phase
  const BufF64 rr(dir == 0 ? F.ru : F.rv), Akv(F.Akv), Wi(F.Wi);
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = dt * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  double rk[KR];
#pragma unroll
  for (int p = 0; p < KR; p++) {
    const int k = c0 + p;
    const double rro = LD(rr, vo, lev(k));
    rk[p] = k == 1 ? rro - fl[1] : rro - fl[p + 1 < KR ? p + 1 : KR - 1] + fl[p];
  }
  int tl = tid;
  __asm__ volatile("" : "+v"(tl));
  auto HZ = [&](int q) { return roms_smem[tl + q * nthr]; };
  auto HZM = [&](int q) { return roms_smem[(KR + 1 + q) * nthr + tl]; };
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q (0 at the bottom and the surface)
    const int r = c0 - 1 + q;
    const unsigned w = (unsigned)min(max(r, 1), N - 1) * lv;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * dt * (LD(Akv, vo, w) + LD(Akv, vm, w)), HZ(qa) + HZM(qa) + HZ(q) + HZM(q));
    const double wv = DC0 * 0.5 * (LD(Wi, vo, w) + LD(Wi, vm, w));
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  const double rD = F.r_D[ij], rDm = F.r_D[ij - s];
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.eliminate(n, [&](int p, double& a, double& bb, double& cc, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    const int k = c0 + p;
    a = -(fcl + fmax0(wcl));
    cc = -(fcu - fmin0(wcu));
    const double b1 = 0.5 * (HZ(p + 1) + HZM(p + 1)) + 0.5 * dt * (rD + rDm) + fcu + fmax0(wcu);
    const double bk = 0.5 * (HZ(p + 1) + HZM(p + 1)) + fcl - fmin0(wcl) + fcu + fmax0(wcu);
    bb = k == 1 ? b1 : bk;
    const double v = (PF ? un[p] : LD(Un, vo, lev(k))) + DC0 * rk[p];
    dd = k == N ? v + dt * sstr : v;
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  const double dmdn = dir == 0 ? F.dm_u[ij] * F.dn_u[ij] : F.dm_v[ij] * F.dn_v[ij];
  // rufrc = ru(1) + dmdn*(sstr - r_D*u(1)) + ru(2) + ... + ru(N), wave by wave
  const int S = sg.S, sl = sg.l;
  for (int t = 0; t < S; t++) {
    if (sg.s == t) {
      double frc;
      if (t == 0) frc = rk[0] + dmdn * (sstr - 0.5 * (rDm + rD) * T.D[0]);
      else frc = Lf[t - 1][sl] + rk[0];
#pragma unroll
      for (int p = 1; p < KR; p++) frc = p < n ? frc + rk[p] : frc;
      Lf[t][sl] = frc;
    }
    __syncthreads();
  }
  const unsigned vs = act ? vo : kBufOff;
#pragma unroll
  for (int p = 0; p < KR; p++)
    if (p < n) {
      if constexpr (kU) Un.st(T.D[p] * 0.5 * (HZ(p + 1) + HZM(p + 1)), vs, lev(c0 + p));
      else Un.st(T.D[p] * 0.5 * (HZ(p + 1) + HZM(p + 1)), act ? vo + lev(c0 + p) : kBufOff, 0u);
    }
  if (act && sg.s == 0) {
    if (dir == 0) F.rufrc[ij] = Lf[S - 1][sl];
    else F.rvfrc[ij] = Lf[S - 1][sl];
  }
}

void setup_column_kernels_uv1(size_t bytes) {
  (void)hipFuncSetAttribute((const void*)k_uv1<ColLds>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
// the ru levels of k_uv1_seg's rows-j blocks (up to kSegJMax rows, N <= kSegRows*kSegMaxS);
// kLds: the Hz pairs of every thread's KR+1 rows
static size_t uv1_seg_lds_bytes(unsigned nthr) { return (size_t)2 * (kSegRows + 2) * nthr * sizeof(double); }
void setup_uv1_seg() {
  (void)hipFuncSetAttribute((const void*)k_uv1_seg<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)((size_t)kSegRows * kSegMaxS * kSegCW * kSegJMax * sizeof(double)));
  (void)hipFuncSetAttribute((const void*)k_uv1_seg<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uv1_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_uv1_segb<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uv1_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_uv1_segb<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uv1_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_uv1_segb<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uv1_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_uv1_segb<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uv1_seg_lds_bytes(kSegBlock * kSegJMax));
}

void launch_step3d_uv1(const Dev& d, hipStream_t s, const Tlev& t, bool uv_done) {
  const Bounds& b = d.b;
  if (!uv_done) launch_uv_horiz(d, s, t.nrhs, 1);
  Range R{b.istr, b.iend, b.jstr, b.jend};
  dim3 g = gridc_of(R);
  g.z = 2;
  if ((d.p.colreg & 1) && b.N == 50)
    hipLaunchKernelGGL(k_uv1_reg<50>, g, dim3(kCX), col_lds_bytes(1, 50), s, d, R, t.nnew, t.nrhs);
  else if (d.p.colseg) {
    const dim3 gs = seg_uv_grid(d, R, d.p.seg_jrows), bs(kCX, seg_waves(b.N), d.p.seg_jrows);
    ktimer_mark(s, kTimedUv1Seg, 0);
    if (d.p.uv1_lds && d.p.uv_adv && (d.p.seg_buf & 32) && (d.p.seg_buf & 512) && (d.p.seg_buf & 64))
      hipLaunchKernelGGL((k_uv1_segb<true, false>), gs, bs, uv1_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, R, t.nnew,
                         t.nrhs);
    else if (d.p.uv1_lds && d.p.uv_adv && (d.p.seg_buf & 32) && (d.p.seg_buf & 512))
      hipLaunchKernelGGL((k_uv1_segb<false, false>), gs, bs, uv1_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, R, t.nnew,
                         t.nrhs);
    else if (d.p.uv1_lds && d.p.uv_adv && (d.p.seg_buf & 32) && (d.p.seg_buf & 64))
      hipLaunchKernelGGL(k_uv1_segb<true>, gs, bs, uv1_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, R, t.nnew, t.nrhs);
    else if (d.p.uv1_lds && d.p.uv_adv && (d.p.seg_buf & 32))
      hipLaunchKernelGGL(k_uv1_segb<false>, gs, bs, uv1_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, R, t.nnew, t.nrhs);
    else if (d.p.uv1_lds && d.p.uv_adv)
      hipLaunchKernelGGL(k_uv1_seg<true>, gs, bs, uv1_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, R, t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL(k_uv1_seg<false>, gs, bs, (size_t)b.N * kSegCW * d.p.seg_jrows * sizeof(double), s, d, R,
                         t.nnew, t.nrhs);
    ktimer_mark(s, kTimedUv1Seg, 1, 1);
  }
  else if (d.f.colscr)
    hipLaunchKernelGGL(k_uv1<ColGlb>, g, dim3(kCX), 0, s, d, R, t.nnew, t.nrhs);
  else
    hipLaunchKernelGGL(k_uv1<ColLds>, g, dim3(kCX), col_lds_bytes(2, b.N), s, d, R, t.nnew, t.nrhs);
}

// ---- visc3d: harmonic viscosity along S; adds dt*cff to u,v(indx) (Hz*u)
// and cff to rufrc,rvfrc.  Each lane forms the two rho-point and two
// psi-point stress components around its u (v) point. ----
__device__ __forceinline__ void visc_rho(const Dev& d, int i, int j, int k, int nstp, double& UFx, double& VFe) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), o = ij + (long)(k - 1) * b.n2, l = (long)(nstp - 1) * b.n3;
  const double* pm = F.pm;
  const double* pn = F.pn;
  const long sj = b.nx2;
  const double cff = 0.5 * F.Hz[o] * F.visc2_r[ij] *
                     (F.dn_r[ij] * pm[ij] * ((pn[ij] + pn[ij + 1]) * F.u[o + 1 + l] - (pn[ij - 1] + pn[ij]) * F.u[o + l]) -
                      F.dm_r[ij] * pn[ij] * ((pm[ij] + pm[ij + sj]) * F.v[o + sj + l] - (pm[ij - sj] + pm[ij]) * F.v[o + l]));
  UFx = cff * F.dn_r[ij] * F.dn_r[ij];
  VFe = -cff * F.dm_r[ij] * F.dm_r[ij];
}
__device__ __forceinline__ void visc_psi(const Dev& d, int i, int j, int k, int nstp, double& UFe, double& VFx) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long sj = b.nx2;
  const long ij = IJ(b, i, j), o = ij + (long)(k - 1) * b.n2, l = (long)(nstp - 1) * b.n3;
  const double* pm = F.pm;
  const double* pn = F.pn;
  const double cff =
      0.125 * (F.Hz[o - 1] + F.Hz[o] + F.Hz[o - 1 - sj] + F.Hz[o - sj]) * F.visc2_p[ij] *
      (0.25 * (pm[ij - 1] + pm[ij] + pm[ij - 1 - sj] + pm[ij - sj]) * F.dn_p[ij] *
           ((pn[ij - sj] + pn[ij]) * F.v[o + l] - (pn[ij - 1 - sj] + pn[ij - 1]) * F.v[o - 1 + l]) +
       0.25 * (pn[ij - 1] + pn[ij] + pn[ij - 1 - sj] + pn[ij - sj]) * F.dm_p[ij] *
           ((pm[ij - 1] + pm[ij]) * F.u[o + l] - (pm[ij - 1 - sj] + pm[ij - sj]) * F.u[o - sj + l])) *
      F.pmask[ij];
  UFe = cff * F.dm_p[ij] * F.dm_p[ij];
  VFx = cff * F.dn_p[ij] * F.dn_p[ij];
}

// Whole-column tiles: a block owns a 64x4 tile of (i,j) for all levels
// k = 1..N.  The 2-D metric factors of every stress point and divergence
// point are formed once per block (registers) instead of once per level,
// and each lane sums its own stress divergence over k in the reference's
// k = 1..N order, so rufrc/rvfrc need no column scratch or second kernel.
// Per level, the rho-point (UFx,VFe) and psi-point (UFe,VFx) stresses of
// the tile (rho points with a low-side, psi points with a high-side halo)
// are evaluated once into LDS, then each lane forms its divergences.
// Operation order is the reference's (visc3d_S.F:60-136), so results are
// bit-identical to the per-level form.
constexpr int kVW = kBX + 1, kVN = kVW * (kBY + 1), kVQ = (kVN + kBX * kBY - 1) / (kBX * kBY);
struct ViscRho {  // metric factors of one rho point
  double v2, X, sx1, sx0, Y, sy1, sy0, dn, dm;
  long ij;
  bool on;
};
struct ViscPsi {  // metric factors of one psi point
  double v2, P1, P2, a1, a0, b1, b0, msk, dm, dn;
  long ij;
  bool on;
};
__global__ void __launch_bounds__(256) k_visc3d(Dev d, Range R, int nstp) {
  const uint3 bI = xcd_tile();
  __shared__ double sUFx[kVN], sVFe[kVN], sUFe[kVN], sVFx[kVN];
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int indx = 3 - nstp;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const long sj = b.nx2;
  const double* pm = F.pm;
  const double* pn = F.pn;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  ViscRho gr[kVQ];
  ViscPsi gp[kVQ];
#pragma unroll
  for (int m = 0; m < kVQ; m++) {
    const int q = tid + m * kBX * kBY;
    const int li = q % kVW, lj = q / kVW;
    const int ir = i0 - 1 + li, jr = j0 - 1 + lj;  // rho point
    ViscRho& r = gr[m];
    r.on = q < kVN && ir >= 0 && ir <= b.Lm + 1 && jr >= 0 && jr <= b.Mm + 1;
    r.ij = IJ(b, ir, jr);
    if (r.on) {
      const long ij = r.ij;
      r.v2 = F.visc2_r[ij];
      r.X = F.dn_r[ij] * pm[ij]; r.sx1 = pn[ij] + pn[ij + 1]; r.sx0 = pn[ij - 1] + pn[ij];
      r.Y = F.dm_r[ij] * pn[ij]; r.sy1 = pm[ij] + pm[ij + sj]; r.sy0 = pm[ij - sj] + pm[ij];
      r.dn = F.dn_r[ij]; r.dm = F.dm_r[ij];
    }
    const int ip = i0 + li, jp = j0 + lj;  // psi point
    ViscPsi& p = gp[m];
    p.on = q < kVN && ip >= 0 && ip <= b.Lm + 2 && jp >= 0 && jp <= b.Mm + 2;
    p.ij = IJ(b, ip, jp);
    if (p.on) {
      const long ij = p.ij;
      p.v2 = F.visc2_p[ij];
      p.P1 = 0.25 * (pm[ij - 1] + pm[ij] + pm[ij - 1 - sj] + pm[ij - sj]) * F.dn_p[ij];
      p.a1 = pn[ij - sj] + pn[ij]; p.a0 = pn[ij - 1 - sj] + pn[ij - 1];
      p.P2 = 0.25 * (pn[ij - 1] + pn[ij] + pn[ij - 1 - sj] + pn[ij - sj]) * F.dm_p[ij];
      p.b1 = pm[ij - 1] + pm[ij]; p.b0 = pm[ij - 1 - sj] + pm[ij - sj];
      p.msk = F.pmask[ij]; p.dm = F.dm_p[ij]; p.dn = F.dn_p[ij];
    }
  }
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, i, j);
  const bool du = act && i >= b.istrU && i <= b.iend, dv = act && j >= b.jstrV && j <= b.jend;
  double cum = 0.0, cun = 0.0, cvm = 0.0, cvn = 0.0, fu = 0.0, fv = 0.0;
  if (du) { cum = pm[ij - 1] + pm[ij]; cun = pn[ij - 1] + pn[ij]; fu = F.rufrc[ij]; }
  if (dv) { cvm = pm[ij] + pm[ij - sj]; cvn = pn[ij] + pn[ij - sj]; fv = F.rvfrc[ij]; }
  const double cu0 = 0.125 * cum * cun, cv0 = 0.125 * cvm * cvn;
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  double* Ui = F.u + (long)(indx - 1) * b.n3;
  double* Vi = F.v + (long)(indx - 1) * b.n3;
  const int qr = (threadIdx.x + 1) + (threadIdx.y + 1) * kVW;  // rho (i,j); -1: (i-1,j); -kVW: (i,j-1)
  const int qp = threadIdx.x + threadIdx.y * kVW;              // psi (i,j); +1: (i+1,j); +kVW: (i,j+1)
  for (int k = 1; k <= b.N; k++) {
    const long kk = (long)(k - 1) * b.n2;
    const double* Hk = F.Hz + kk;
    const double* Uk = U + kk;
    const double* Vk = V + kk;
    // the lane's u/v(indx) of this level, loaded with the stress inputs (one
    // memory wait per level instead of a second one after the barriers)
    const double ui = du ? Ui[ij + kk] : 0.0, vi = dv ? Vi[ij + kk] : 0.0;
    if (k > 1) __syncthreads();  // previous level's stresses consumed
#pragma unroll
    for (int m = 0; m < kVQ; m++) {
      const int q = tid + m * kBX * kBY;
      if (q >= kVN) break;
      double ufx = 0.0, vfe = 0.0, ufe = 0.0, vfx = 0.0;
      const ViscRho& r = gr[m];
      if (r.on) {
        const long o = r.ij;
        const double cff = 0.5 * Hk[o] * r.v2 * (r.X * (r.sx1 * Uk[o + 1] - r.sx0 * Uk[o]) -
                                                 r.Y * (r.sy1 * Vk[o + sj] - r.sy0 * Vk[o]));
        ufx = cff * r.dn * r.dn;
        vfe = -cff * r.dm * r.dm;
      }
      const ViscPsi& p = gp[m];
      if (p.on) {
        const long o = p.ij;
        const double cff = 0.125 * (Hk[o - 1] + Hk[o] + Hk[o - 1 - sj] + Hk[o - sj]) * p.v2 *
                           (p.P1 * (p.a1 * Vk[o] - p.a0 * Vk[o - 1]) + p.P2 * (p.b1 * Uk[o] - p.b0 * Uk[o - sj])) *
                           p.msk;
        ufe = cff * p.dm * p.dm;
        vfx = cff * p.dn * p.dn;
      }
      sUFx[q] = ufx; sVFe[q] = vfe; sUFe[q] = ufe; sVFx[q] = vfx;
    }
    __syncthreads();
    const long o = ij + kk;
    if (du) {
      const double cff = cu0 * (cun * (sUFx[qr] - sUFx[qr - 1]) + cum * (sUFe[qp + kVW] - sUFe[qp]));
      Ui[o] = ui + d.p.dt * cff;
      fu = fu + cff;
    }
    if (dv) {
      const double cff = cv0 * (cvn * (sVFx[qp + 1] - sVFx[qp]) + cvm * (sVFe[qr] - sVFe[qr - kVW]));
      Vi[o] = vi + d.p.dt * cff;
      fv = fv + cff;
    }
  }
  if (du) F.rufrc[ij] = fu;
  if (dv) F.rvfrc[ij] = fv;
}

// The same with each level's raw u, v(nstp) and Hz windows staged in LDS
// once per block (u over i0-1..i0+65 x j0-1..j0+4, v over i0-1..i0+64 x
// j0-1..j0+5, Hz over i0-1..i0+64 x j0-1..j0+4: about 5 loads per lane per
// level instead of about 22), the next level's window in registers while
// this one is consumed.  Two barriers per level, as above.  Bit-identical.
constexpr int kVUW = kBX + 3, kVUN = kVUW * (kBY + 2);   // u window
constexpr int kVVW = kBX + 2, kVVN = kVVW * (kBY + 3);   // v window
constexpr int kVHW = kBX + 2, kVHN = kVHW * (kBY + 2);   // Hz window
constexpr int kVSN = kVUN + kVVN + kVHN, kVSQ = (kVSN + kBX * kBY - 1) / (kBX * kBY);
__global__ void __launch_bounds__(256, 3) k_visc3d_stg(Dev d, Range R, int nstp) {
  const uint3 bI = xcd_tile();
  __shared__ double sUFx[kVN], sVFe[kVN], sUFe[kVN], sVFx[kVN];
  __shared__ double sRaw[kVSN];
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int indx = 3 - nstp;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const long sj = b.nx2;
  const double* pm = F.pm;
  const double* pn = F.pn;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  ViscRho gr[kVQ];
  ViscPsi gp[kVQ];
#pragma unroll
  for (int m = 0; m < kVQ; m++) {
    const int q = tid + m * kBX * kBY;
    const int li = q % kVW, lj = q / kVW;
    const int ir = i0 - 1 + li, jr = j0 - 1 + lj;  // rho point
    ViscRho& r = gr[m];
    r.on = q < kVN && ir >= 0 && ir <= b.Lm + 1 && jr >= 0 && jr <= b.Mm + 1;
    r.ij = IJ(b, ir, jr);
    if (r.on) {
      const long ij = r.ij;
      r.v2 = F.visc2_r[ij];
      r.X = F.dn_r[ij] * pm[ij]; r.sx1 = pn[ij] + pn[ij + 1]; r.sx0 = pn[ij - 1] + pn[ij];
      r.Y = F.dm_r[ij] * pn[ij]; r.sy1 = pm[ij] + pm[ij + sj]; r.sy0 = pm[ij - sj] + pm[ij];
      r.dn = F.dn_r[ij]; r.dm = F.dm_r[ij];
    }
    const int ip = i0 + li, jp = j0 + lj;  // psi point
    ViscPsi& p = gp[m];
    p.on = q < kVN && ip >= 0 && ip <= b.Lm + 2 && jp >= 0 && jp <= b.Mm + 2;
    p.ij = IJ(b, ip, jp);
    if (p.on) {
      const long ij = p.ij;
      p.v2 = F.visc2_p[ij];
      p.P1 = 0.25 * (pm[ij - 1] + pm[ij] + pm[ij - 1 - sj] + pm[ij - sj]) * F.dn_p[ij];
      p.a1 = pn[ij - sj] + pn[ij]; p.a0 = pn[ij - 1 - sj] + pn[ij - 1];
      p.P2 = 0.25 * (pn[ij - 1] + pn[ij] + pn[ij - 1 - sj] + pn[ij - sj]) * F.dm_p[ij];
      p.b1 = pm[ij - 1] + pm[ij]; p.b0 = pm[ij - 1 - sj] + pm[ij - sj];
      p.msk = F.pmask[ij]; p.dm = F.dm_p[ij]; p.dn = F.dn_p[ij];
    }
  }
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  // this thread's raw window entries: field (0 u, 1 v, 2 Hz, -1 none) and 2-D offset
  long wo[kVSQ];
  int wf[kVSQ];
#pragma unroll
  for (int m = 0; m < kVSQ; m++) {
    const int q = tid + m * kBX * kBY;
    int ii = 0, jj = 0, f = -1;
    if (q < kVUN) { f = 0; ii = i0 - 1 + q % kVUW; jj = j0 - 1 + q / kVUW; }
    else if (q < kVUN + kVVN) { const int qq = q - kVUN; f = 1; ii = i0 - 1 + qq % kVVW; jj = j0 - 1 + qq / kVVW; }
    else if (q < kVSN) { const int qq = q - kVUN - kVVN; f = 2; ii = i0 - 1 + qq % kVHW; jj = j0 - 1 + qq / kVHW; }
    if (f >= 0 && !(ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2)) f = -1;
    wf[m] = f;
    wo[m] = f >= 0 ? IJ(b, ii, jj) : 0;
  }
  auto ldraw = [&](int k, double (&x)[kVSQ]) {
    const long kk = (long)(k - 1) * b.n2;
#pragma unroll
    for (int m = 0; m < kVSQ; m++)
      x[m] = wf[m] == 0 ? U[wo[m] + kk] : wf[m] == 1 ? V[wo[m] + kk] : wf[m] == 2 ? F.Hz[wo[m] + kk] : 0.0;
  };
  auto Uw = [&](int ii, int jj) { return sRaw[(ii - (i0 - 1)) + (jj - (j0 - 1)) * kVUW]; };
  auto Vw = [&](int ii, int jj) { return sRaw[kVUN + (ii - (i0 - 1)) + (jj - (j0 - 1)) * kVVW]; };
  auto Hw = [&](int ii, int jj) { return sRaw[kVUN + kVVN + (ii - (i0 - 1)) + (jj - (j0 - 1)) * kVHW]; };
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, i, j);
  const bool du = act && i >= b.istrU && i <= b.iend, dv = act && j >= b.jstrV && j <= b.jend;
  double cum = 0.0, cun = 0.0, cvm = 0.0, cvn = 0.0, fu = 0.0, fv = 0.0;
  if (du) { cum = pm[ij - 1] + pm[ij]; cun = pn[ij - 1] + pn[ij]; fu = F.rufrc[ij]; }
  if (dv) { cvm = pm[ij] + pm[ij - sj]; cvn = pn[ij] + pn[ij - sj]; fv = F.rvfrc[ij]; }
  const double cu0 = 0.125 * cum * cun, cv0 = 0.125 * cvm * cvn;
  double* Ui = F.u + (long)(indx - 1) * b.n3;
  double* Vi = F.v + (long)(indx - 1) * b.n3;
  const int qr = (threadIdx.x + 1) + (threadIdx.y + 1) * kVW;  // rho (i,j); -1: (i-1,j); -kVW: (i,j-1)
  const int qp = threadIdx.x + threadIdx.y * kVW;              // psi (i,j); +1: (i+1,j); +kVW: (i,j+1)
  double raw[kVSQ];
  ldraw(1, raw);
  // u, v(indx) of the lane's cell: level k+1's loaded with level k+1's
  // window, before level k's stores (which vmcnt counts with the loads)
  double nui = du ? Ui[ij] : 0.0, nvi = dv ? Vi[ij] : 0.0;
  for (int k = 1; k <= b.N; k++) {
    const long kk = (long)(k - 1) * b.n2;
    const double ui = nui, vi = nvi;
    // every lane finished the previous level's stress reads of sRaw before
    // its second barrier, so the raw window can be overwritten here
#pragma unroll
    for (int m = 0; m < kVSQ; m++) {
      const int q = tid + m * kBX * kBY;
      if (q < kVSN) sRaw[q] = raw[m];
    }
    if (k < b.N) {
      ldraw(k + 1, raw);
      nui = du ? Ui[ij + kk + b.n2] : 0.0;
      nvi = dv ? Vi[ij + kk + b.n2] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kVQ; m++) {
      const int q = tid + m * kBX * kBY;
      if (q >= kVN) break;
      const int li = q % kVW, lj = q / kVW;
      double ufx = 0.0, vfe = 0.0, ufe = 0.0, vfx = 0.0;
      const ViscRho& r = gr[m];
      if (r.on) {
        const int ir = i0 - 1 + li, jr = j0 - 1 + lj;
        const double cff = 0.5 * Hw(ir, jr) * r.v2 * (r.X * (r.sx1 * Uw(ir + 1, jr) - r.sx0 * Uw(ir, jr)) -
                                                      r.Y * (r.sy1 * Vw(ir, jr + 1) - r.sy0 * Vw(ir, jr)));
        ufx = cff * r.dn * r.dn;
        vfe = -cff * r.dm * r.dm;
      }
      const ViscPsi& p = gp[m];
      if (p.on) {
        const int ip = i0 + li, jp = j0 + lj;
        const double cff = 0.125 * (Hw(ip - 1, jp) + Hw(ip, jp) + Hw(ip - 1, jp - 1) + Hw(ip, jp - 1)) * p.v2 *
                           (p.P1 * (p.a1 * Vw(ip, jp) - p.a0 * Vw(ip - 1, jp)) +
                            p.P2 * (p.b1 * Uw(ip, jp) - p.b0 * Uw(ip, jp - 1))) *
                           p.msk;
        ufe = cff * p.dm * p.dm;
        vfx = cff * p.dn * p.dn;
      }
      sUFx[q] = ufx; sVFe[q] = vfe; sUFe[q] = ufe; sVFx[q] = vfx;
    }
    __syncthreads();
    const long o = ij + kk;
    if (du) {
      const double cff = cu0 * (cun * (sUFx[qr] - sUFx[qr - 1]) + cum * (sUFe[qp + kVW] - sUFe[qp]));
      Ui[o] = ui + d.p.dt * cff;
      fu = fu + cff;
    }
    if (dv) {
      const double cff = cv0 * (cvn * (sVFx[qp + 1] - sVFx[qp]) + cvm * (sVFe[qr] - sVFe[qr - kVW]));
      Vi[o] = vi + d.p.dt * cff;
      fv = fv + cff;
    }
  }
  if (du) F.rufrc[ij] = fu;
  if (dv) F.rvfrc[ij] = fv;
}

void launch_visc3d(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  if (d.p.visc_stg)
    hipLaunchKernelGGL(k_visc3d_stg, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nstp);
  else
    hipLaunchKernelGGL(k_visc3d, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nstp);
}

// Columns that k_uv2_fused owns: the coupling range without the rows (u) /
// columns (v) next to a closed edge, whose coupled values u3dbc/v3dbc copy
// into the ghost rows before the flux correction.
__host__ __device__ __forceinline__ bool uv2_fused_in(const Bounds& b, int dir, int i, int j) {
  if (dir == 0)
    return i >= b.istrU && i <= b.iend && j >= b.jstr + (b.south_edge ? 1 : 0) && j <= b.jend - (b.north_edge ? 1 : 0);
  return i >= b.istr + (b.west_edge ? 1 : 0) && i <= b.iend - (b.east_edge ? 1 : 0) && j >= b.jstrV && j <= b.jend;
}

// ---- step3d_uv2 part 1: convert Hz*u to u and remove the mismatch against
// the fast-time-averaged barotropic flux DU_avg1 (at n+1 depths) ----
__global__ void __launch_bounds__(256) k_uv2_couple(Dev d, Range R, int nnew, int edges) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  for (int dir = 0; dir < 2; dir++) {
    if (dir == 0 && !(i >= b.istrU)) continue;
    if (dir == 1 && !(j >= b.jstrV)) continue;
    if (edges && uv2_fused_in(b, dir, i, j)) continue;   // edge mode: what k_uv2_fused leaves out
    const long s = dir == 0 ? 1 : b.nx2;
    double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
    const double* __restrict__ Hz = F.Hz + ij;
    const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
    const double avg1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
    const double msk = dir == 0 ? F.umask[ij] : F.vmask[ij];
    // sums first (read-only, so the loads of all levels pipeline), then the
    // per-level quotient and correction in chunks whose loads precede their
    // stores: the reference's values (step3d_uv2.F:103-133) without a
    // may-alias wait per level (edge columns walk alone: their latency is the
    // kernel's)
    long o = (long)(N - 1) * n2;
    double CF0 = 0.5 * (Hz[o] + Hz[o - s]);
    double DC0 = Un[o];
#pragma unroll 8
    for (int k = N - 1; k >= 1; k--) {
      o = (long)(k - 1) * n2;
      CF0 = CF0 + 0.5 * (Hz[o] + Hz[o - s]);
      DC0 = DC0 + Un[o];
    }
    DC0 = (DC0 * dn - avg1) / (CF0 * dn);
    constexpr int CH = 8;
    for (int k0 = 1; k0 <= N; k0 += CH) {
      double uc[CH], cc[CH];
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const long oq = (long)(min(k0 + q, N) - 1) * n2;
        uc[q] = Un[oq];
        cc[q] = 0.5 * (Hz[oq] + Hz[oq - s]);
      }
#pragma unroll
      for (int q = 0; q < CH; q++)
        if (k0 + q <= N) Un[(long)(k0 + q - 1) * n2] = (uc[q] / cc[q] - DC0) * msk;
    }
  }
}

// ---- step3d_uv2 part 2: ubar,vbar(knew) from DU_avg1; corrected fluxes
// FlxU = DELTA*FlxU + EPSIL*Hz_u*dn_u*(u(nstp)+u(nnew)), mismatch vs DU_avg2 ----
__global__ void __launch_bounds__(256) k_uv2_flux(Dev d, Range R, int nnew, int nstp, int knew, int iu0, int iu1, int iv0,
                                                  int iv1, int edges) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double DELTA = 0.28, EPSIL = 0.36;
  for (int dir = 0; dir < 2; dir++) {
    if (dir == 0 && !(i >= iu0 && i <= iu1)) continue;
    if (dir == 1 && !(i >= iv0 && i <= iv1 && j >= b.jstr)) continue;
    // edge mode: only the columns k_uv2_fused leaves out (outside the coupling range)
    if (edges && uv2_fused_in(b, dir, i, j)) continue;
    const long s = dir == 0 ? 1 : b.nx2;
    double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
    const double* __restrict__ Us = (dir == 0 ? F.u : F.v) + (long)(nstp - 1) * b.n3 + ij;
    double* __restrict__ Flx = (dir == 0 ? F.FlxU : F.FlxV) + ij;
    const double* __restrict__ Hz = F.Hz + ij;
    double* __restrict__ CFs = F.c0 + ij;
    const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
    const double avg1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
    const double avg2 = dir == 0 ? F.DU_avg2[ij] : F.DV_avg2[ij];
    const double msk = dir == 0 ? F.umask[ij] : F.vmask[ij];
    auto DCk = [&](int k) { const long o = (long)(k - 1) * n2; return 0.5 * (Hz[o] + Hz[o - s]) * dn; };
    long o = (long)(N - 1) * n2;
    const double dcN = DCk(N);
    double DC0 = dcN, FC0 = dcN * Un[o];
#pragma unroll 8
    for (int k = N - 1; k >= 1; k--) {
      o = (long)(k - 1) * n2;
      const double dck = DCk(k);
      DC0 = DC0 + dck;
      FC0 = FC0 + dck * Un[o];
    }
    DC0 = 1.0 / DC0;
    if (dir == 0) F.ubar[IJL(b, i, j, knew)] = DC0 * avg1;
    else F.vbar[IJL(b, i, j, knew)] = DC0 * avg1;
    FC0 = DC0 * (FC0 - avg1);
    double CF0 = 0.0;
    // chunks of levels whose loads precede their stores (see k_uv2_couple)
    constexpr int CH = 8;
    for (int k0 = N; k0 >= 1; k0 -= CH) {
      double uc[CH], fc[CH], sc[CH], dc[CH];
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int k = max(k0 - q, 1);
        const long oq = (long)(k - 1) * n2;
        uc[q] = Un[oq]; fc[q] = Flx[oq]; sc[q] = Us[oq]; dc[q] = DCk(k);
      }
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int k = k0 - q;
        if (k >= 1) {
          const long oq = (long)(k - 1) * n2;
          const double un = (uc[q] - FC0) * msk;
          Un[oq] = un;
          const double cfk = DELTA * fc[q] + EPSIL * dc[q] * (sc[q] + un);
          CFs[(long)k * n2] = cfk;
          CF0 = CF0 + cfk;
        }
      }
    }
    CF0 = DC0 * (CF0 - avg2);
#pragma unroll 8
    for (int k = 1; k <= N; k++) {
      o = (long)(k - 1) * n2;
      Flx[o] = CFs[(long)k * n2] - DCk(k) * CF0;
    }
  }
}

// ---- step3d_uv2, fused form: k_uv2_couple and k_uv2_flux for every column
// of the coupling range in one pass, for both directions.  A wavefront holds
// 16 columns x 4 vertical segments (lane = 16*g + column, g = 0 the bottom
// segment of KL levels), so every load covers four 128-B rows; a block is a
// 16 x 4 patch of columns.  The column's values stay in the lane's registers
// between the reference's three vertical passes, and the four vertical sums
// (sum of Hz_u, of Hz_u*u, of Hz_u*dn_u, of the corrected fluxes) run as a
// chain down the segments, top lane first, handing the running sum to the
// lane below with a shuffle, so every sum keeps the reference's k = N..1
// order and the results are bit-identical to the two kernels
// (step3d_uv2.F:18-786).  The open-edge columns outside the coupling range
// (walls, ghost rows) follow u3dbc/v3dbc through k_uv2_flux (edge mode). ----
// KL > 13 (N > 52): the lane's KL Hz_u levels sit in LDS (hc[] below) -- in
// registers beside the KL u levels they spilled (29 VGPRs at KL = 25); three
// 256-thread blocks per CU keep the same occupancy
// FULL: N == 4*KL, every segment holds KL levels (C3's N = 100), so the
// per-level guards fold away and the level loops are straight-line code
template <int KL, bool FULL = false>
__global__ void __launch_bounds__(256, KL > 13 ? 3 : 4) k_uv2_fused(Dev d, Range R, int nnew, int nstp, int knew) {
  constexpr bool kHcLds = KL > 13;
  __shared__ double sHc[kHcLds ? KL * 256 : 1];
  const uint3 bI = xcd_tile();
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double DELTA = 0.28, EPSIL = 0.36;
  const ChainLane cl = chain_lane<KL>(R, bI, N);
  const int i = cl.i, j = cl.j, g = cl.g, lo = cl.lo, nk = FULL ? KL : cl.nk;
  const long n2 = b.n2;
  auto chain2 = [&](double& s1, double& s2, auto&& body) { chain_down(cl, s1, s2, body); };
  const int d0 = gridDim.z == 2 ? (int)bI.z : 0, d1 = gridDim.z == 2 ? d0 + 1 : 2;   // grid z = 2: a direction per block
  for (int dir = d0; dir < d1; dir++) {
    // the lane's column, clamped into the coupling range (lanes outside
    // k_uv2_fused's columns compute on a valid column so the shuffles see
    // defined values, and store nothing)
    const int ilo = dir == 0 ? b.istrU : b.istr, jlo = dir == 0 ? b.jstr : b.jstrV;
    const int ic = min(max(i, ilo), b.iend), jc = min(max(j, jlo), b.jend);
    const bool act = ic == i && jc == j && cl.in && uv2_fused_in(b, dir, i, j);
    const long ij = IJ(b, ic, jc), s = dir == 0 ? 1 : b.nx2;
    const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
    const double avg1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
    const double avg2 = dir == 0 ? F.DU_avg2[ij] : F.DV_avg2[ij];
    const double msk = dir == 0 ? F.umask[ij] : F.vmask[ij];
    // The level loops' memory operations are raw-buffer accesses: the lane's
    // column offset in a VGPR, the level's in an SGPR (no 64-bit address per
    // level held in registers across the passes; they spilled ~200 VGPRs).
    // A level the lane does not own (q >= nk: past N in the top segment)
    // and every store of an inactive lane take the offset kBufOff, outside
    // the extent: the load returns 0 and the store is dropped -- straight-line
    // level loops without branches.  The sums skip those levels by selects.
    const double* const Ub = (dir == 0 ? F.u : F.v);
    const BufF64 bUn(Ub + (long)(nnew - 1) * b.n3, b.n3), bUs(Ub + (long)(nstp - 1) * b.n3, b.n3), bHz(F.Hz, b.n3),
        bFl(dir == 0 ? F.FlxU : F.FlxV, b.n3);
    const unsigned vo = (unsigned)((ij + (long)(lo - 1) * n2) * 8), vom = vo - (unsigned)(s * 8);
    auto so = [&](int q) { return (unsigned)((long)q * n2 * 8); };
    auto vq = [&](int q) { return q < nk ? vo : kBufOff; };              // loads of level lo+q
    auto vqm = [&](int q) { return q < nk ? vom : kBufOff; };            // ... of its (i-1) / (j-1) neighbour
    auto vsq = [&](int q) { return act && q < nk ? vo : kBufOff; };      // stores
    double un[KL];
    double hcr[kHcLds ? 1 : KL];
    struct HcRef {   // hc[q]: Hz_u of the lane's level lo+q, in LDS (kHcLds) or registers
      double* l;
      double* r;
      __device__ __forceinline__ double& operator[](int q) const { return kHcLds ? l[q * 256] : r[q]; }
    } const hc{sHc + threadIdx.x, hcr};
#pragma unroll
    for (int q = 0; q < KL; q++) {
      un[q] = bUn.ld(vq(q), so(q));
      hc[q] = 0.5 * (bHz.ld(vq(q), so(q)) + bHz.ld(vqm(q), so(q)));
      // the loads of 8 levels in flight at a time (all 25 hoisted spilled)
      if (q % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    }
    // k_uv2_couple: CF0 = sum Hz_u, DC0 = sum Hz*u (k = N..1); u = Hz*u/Hz_u
    double CF0, DC0;
    chain2(CF0, DC0, [&](double& a, double& c) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--) {
        a = q < nk ? a + hc[q] : a;
        c = q < nk ? c + un[q] : c;
      }
    });
    DC0 = (DC0 * dn - avg1) / (CF0 * dn);
#pragma unroll
    for (int q = 0; q < KL; q++) un[q] = (un[q] / hc[q] - DC0) * msk;   // (dead levels: never used)
    // k_uv2_flux: D = sum Hz_u*dn, FC = sum Hz_u*dn*u (k = N..1)
    double DS, FC0;
    chain2(DS, FC0, [&](double& a, double& c) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--) {
        const double dck = hc[q] * dn;
        a = q < nk ? a + dck : a;
        c = q < nk ? c + dck * un[q] : c;
      }
    });
    const double DCi = 1.0 / DS;
    if (act && g == 0) {
      if (dir == 0) F.ubar[IJL(b, i, j, knew)] = DCi * avg1;
      else F.vbar[IJL(b, i, j, knew)] = DCi * avg1;
    }
    FC0 = DCi * (FC0 - avg1);
    // corrected u and the fluxes; un[] becomes the flux cfk (the level loop's
    // loads of u(nstp) and Flx stay here, not hoisted above the chains)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < KL; q++) {
      const double u1 = (un[q] - FC0) * msk;
      bUn.st(u1, vsq(q), so(q));
      un[q] = DELTA * bFl.ld(vq(q), so(q)) + EPSIL * (hc[q] * dn) * (bUs.ld(vq(q), so(q)) + u1);
      if (q % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    }
    double CS, unused;
    chain2(CS, unused, [&](double& a, double& c) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--) a = q < nk ? a + un[q] : a;
    });
    const double CF1 = DCi * (CS - avg2);
#pragma unroll
    for (int q = 0; q < KL; q++) bFl.st(un[q] - (hc[q] * dn) * CF1, vsq(q), so(q));
  }
}

// ---- step3d_uv2 on the closed-edge columns that k_uv2_fused leaves out,
// in k_uv2_fused's chain layout (16 columns x 4 vertical segments per
// wavefront) over a list of (dir, i, j) columns: kCouple = k_uv2_couple's
// pass (the coupling range's edge rows / columns), else k_uv2_flux's (those
// plus the wall faces and ghost rows u3dbc/v3dbc set in between).  The same
// operations in the same order as k_uv2_couple / k_uv2_flux (and as the
// fused kernel's two halves), bit-identical; a column's dependent level walk
// is a quarter of theirs, which is what the one-lane-per-column edge mode's
// time was (each level a page away: a TLB miss per load). ----
template <int KL, bool kCouple>
__global__ void __launch_bounds__(256) k_uv2_edge(Dev d, const int* __restrict__ cols, int ncol, int nnew, int nstp,
                                                  int knew) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double DELTA = 0.28, EPSIL = 0.36;
  const int l = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
  ChainLane cl;
  cl.col = l & (kChainCW - 1);
  cl.g = l / kChainCW;
  cl.lo = 1 + cl.g * KL;
  cl.nk = max(0, min(N, cl.lo + KL - 1) - cl.lo + 1);
  const int c = ((int)blockIdx.x * 4 + w) * kChainCW + cl.col;
  const bool act = c < ncol;
  const int cc = act ? c : ncol - 1;   // idle lanes repeat the last column (shuffles see defined values)
  const int dir = cols[3 * cc], i = cols[3 * cc + 1], j = cols[3 * cc + 2];
  cl.i = i; cl.j = j; cl.in = true;
  const long n2 = b.n2, ij = IJ(b, i, j), s = dir == 0 ? 1 : b.nx2;
  auto chain2 = [&](double& s1, double& s2, auto&& body) { chain_down(cl, s1, s2, body); };
  double* __restrict__ Un = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
  const double avg1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
  const double msk = dir == 0 ? F.umask[ij] : F.vmask[ij];
  double un[KL], hc[KL];
#pragma unroll
  for (int q = 0; q < KL; q++) {
    if (q < cl.nk) {
      const long o = (long)(cl.lo + q - 1) * n2;
      un[q] = Un[o];
      hc[q] = 0.5 * (Hz[o] + Hz[o - s]);
    }
  }
  if constexpr (kCouple) {
    double CF0, DC0;
    chain2(CF0, DC0, [&](double& a, double& c2) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--)
        if (q < cl.nk) { a = a + hc[q]; c2 = c2 + un[q]; }
    });
    DC0 = (DC0 * dn - avg1) / (CF0 * dn);
    if (act) {
#pragma unroll
      for (int q = 0; q < KL; q++)
        if (q < cl.nk) Un[(long)(cl.lo + q - 1) * n2] = (un[q] / hc[q] - DC0) * msk;
    }
  } else {
    const double* __restrict__ Us = (dir == 0 ? F.u : F.v) + (long)(nstp - 1) * b.n3 + ij;
    double* __restrict__ Flx = (dir == 0 ? F.FlxU : F.FlxV) + ij;
    const double avg2 = dir == 0 ? F.DU_avg2[ij] : F.DV_avg2[ij];
    double DS, FC0;
    chain2(DS, FC0, [&](double& a, double& c2) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--)
        if (q < cl.nk) { const double dck = hc[q] * dn; a = a + dck; c2 = c2 + dck * un[q]; }
    });
    const double DCi = 1.0 / DS;
    if (act && cl.g == 0) {
      if (dir == 0) F.ubar[IJL(b, i, j, knew)] = DCi * avg1;
      else F.vbar[IJL(b, i, j, knew)] = DCi * avg1;
    }
    FC0 = DCi * (FC0 - avg1);
#pragma unroll
    for (int q = 0; q < KL; q++) {
      if (q < cl.nk) {
        const long o = (long)(cl.lo + q - 1) * n2;
        const double u1 = (un[q] - FC0) * msk;
        if (act) Un[o] = u1;
        un[q] = DELTA * Flx[o] + EPSIL * (hc[q] * dn) * (Us[o] + u1);
      }
    }
    double CS, unused;
    chain2(CS, unused, [&](double& a, double& c2) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--)
        if (q < cl.nk) a = a + un[q];
    });
    const double CF1 = DCi * (CS - avg2);
    if (act) {
#pragma unroll
      for (int q = 0; q < KL; q++)
        if (q < cl.nk) Flx[(long)(cl.lo + q - 1) * n2] = un[q] - (hc[q] * dn) * CF1;
    }
  }
}

// The (dir, i, j) lists of k_uv2_edge: the columns k_uv2_couple (couple) and
// k_uv2_flux (flux) visit in edge mode, in their ranges and order.
void uv2_edge_lists(const Bounds& b, std::vector<int>& couple, std::vector<int>& flux) {
  couple.clear();
  flux.clear();
  if (!(b.west_edge || b.east_edge || b.south_edge || b.north_edge)) return;
  const int iu0 = b.istr, iu1 = b.ew_periodic ? b.iend : b.iendR;
  const int iv0 = b.ew_periodic ? b.istr : b.istrR, iv1 = b.ew_periodic ? b.iend : b.iendR;
  const int j0 = b.ns_periodic ? b.jstr : b.jstrR, j1 = b.ns_periodic ? b.jend : b.jendR;
  for (int dir = 0; dir < 2; dir++)
    for (int j = b.jstr; j <= b.jend; j++)
      for (int i = b.istr; i <= b.iend; i++) {
        if (dir == 0 && !(i >= b.istrU)) continue;
        if (dir == 1 && !(j >= b.jstrV)) continue;
        if (uv2_fused_in(b, dir, i, j)) continue;
        couple.insert(couple.end(), {dir, i, j});
      }
  for (int dir = 0; dir < 2; dir++)
    for (int j = j0; j <= j1; j++)
      for (int i = (iv0 < iu0 ? iv0 : iu0); i <= (iu1 > iv1 ? iu1 : iv1); i++) {
        if (dir == 0 && !(i >= iu0 && i <= iu1)) continue;
        if (dir == 1 && !(i >= iv0 && i <= iv1 && j >= b.jstr)) continue;
        if (uv2_fused_in(b, dir, i, j)) continue;
        flux.insert(flux.end(), {dir, i, j});
      }
}

void launch_step3d_uv2(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R1{b.istr, b.iend, b.jstr, b.jend};
  const int iu0 = b.istr, iu1 = b.ew_periodic ? b.iend : b.iendR;
  const int iv0 = b.ew_periodic ? b.istr : b.istrR, iv1 = b.ew_periodic ? b.iend : b.iendR;
  const int j0 = b.ns_periodic ? b.jstr : b.jstrR, j1 = b.ns_periodic ? b.jend : b.jendR;
  Range R2{iv0 < iu0 ? iv0 : iu0, iu1 > iv1 ? iu1 : iv1, j0, j1};
  const int kl = (b.N + 3) / 4;
  if (!d.p.obc && d.p.uv2_fused && kl <= 25) {
    dim3 gf = chain_grid_of(R1);
    gf.z = d.p.chain_dirz ? 2 : 1;
    if (kl <= 5) hipLaunchKernelGGL(k_uv2_fused<5>, gf, dim3(256), 0, s, d, R1, t.nnew, t.nstp, t.knew);
    else if (kl <= 13) hipLaunchKernelGGL(k_uv2_fused<13>, gf, dim3(256), 0, s, d, R1, t.nnew, t.nstp, t.knew);
    else if (b.N == 100) hipLaunchKernelGGL((k_uv2_fused<25, true>), gf, dim3(256), 0, s, d, R1, t.nnew, t.nstp, t.knew);
    else hipLaunchKernelGGL(k_uv2_fused<25>, gf, dim3(256), 0, s, d, R1, t.nnew, t.nstp, t.knew);
    if (d.f.uv2e_couple && d.p.uv2e_nc > 0 && d.p.uv2e_nf > 0) {   // closed edges: chain form over the column lists
      const int nc = d.p.uv2e_nc, nf = d.p.uv2e_nf;
      const dim3 gc((nc + 63) / 64), gf2((nf + 63) / 64);
      if (kl <= 5) hipLaunchKernelGGL((k_uv2_edge<5, true>), gc, dim3(256), 0, s, d, d.f.uv2e_couple, nc, t.nnew, t.nstp, t.knew);
      else if (kl <= 13) hipLaunchKernelGGL((k_uv2_edge<13, true>), gc, dim3(256), 0, s, d, d.f.uv2e_couple, nc, t.nnew, t.nstp, t.knew);
      else hipLaunchKernelGGL((k_uv2_edge<25, true>), gc, dim3(256), 0, s, d, d.f.uv2e_couple, nc, t.nnew, t.nstp, t.knew);
      launch_u3dbc(d, s, t);
      launch_v3dbc(d, s, t);
      if (kl <= 5) hipLaunchKernelGGL((k_uv2_edge<5, false>), gf2, dim3(256), 0, s, d, d.f.uv2e_flux, nf, t.nnew, t.nstp, t.knew);
      else if (kl <= 13) hipLaunchKernelGGL((k_uv2_edge<13, false>), gf2, dim3(256), 0, s, d, d.f.uv2e_flux, nf, t.nnew, t.nstp, t.knew);
      else hipLaunchKernelGGL((k_uv2_edge<25, false>), gf2, dim3(256), 0, s, d, d.f.uv2e_flux, nf, t.nnew, t.nstp, t.knew);
    } else if (b.west_edge || b.east_edge || b.south_edge || b.north_edge) {   // columns next to closed edges: couple, u3dbc/v3dbc, flux
      hipLaunchKernelGGL(k_uv2_couple, grid_of(R1), dim3(kBX, kBY), 0, s, d, R1, t.nnew, 1);
      launch_u3dbc(d, s, t);
      launch_v3dbc(d, s, t);
      hipLaunchKernelGGL(k_uv2_flux, grid_of(R2), dim3(kBX, kBY), 0, s, d, R2, t.nnew, t.nstp, t.knew, iu0, iu1, iv0,
                         iv1, 1);
    }
  } else {
    hipLaunchKernelGGL(k_uv2_couple, grid_of(R1), dim3(kBX, kBY), 0, s, d, R1, t.nnew, 0);
    launch_u3dbc(d, s, t);
    launch_v3dbc(d, s, t);
    hipLaunchKernelGGL(k_uv2_flux, grid_of(R2), dim3(kBX, kBY), 0, s, d, R2, t.nnew, t.nstp, t.knew, iu0, iu1, iv0, iv1,
                       0);
  }
  // ADV_ISONEUTRAL: diff3u/v and idRz from the corrected u,v(nnew), before the river faces
  if (d.p.iso) launch_iso_diff3(d, s, t, iu0, iu1, iv0, iv1, j0, j1);
  launch_river_uv(d, s, t.nnew, 0);   // step3d_uv2.F:689-717
  if (d.p.iso) launch_iso_exch_diff3(d, s);
  launch_exchange_list(d, s, ExchList{{d.f.FlxU, d.f.u + (long)(t.nnew - 1) * b.n3, d.f.ubar + (long)(t.knew - 1) * b.n2,
                                        d.f.FlxV, d.f.v + (long)(t.nnew - 1) * b.n3, d.f.vbar + (long)(t.knew - 1) * b.n2},
                                       {b.N, b.N, 1, b.N, b.N, 1}, 6});
}

}  // namespace roms
