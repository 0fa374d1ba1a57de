// k_pre_step3d.hip -- pre_step3d_tile (pre_step3d4S.F:23-742): LF-AM3
// predictor for tracers and momentum to n+1/2, and the bottom-drag
// coefficient r_D (compute_rd_bott_drag.h).  Also hosts the horizontal
// momentum r.h.s. kernel shared with step3d_uv1 (UPSTREAM_UV flag).
#include "k_colseg.h"

namespace roms {

struct PreCoef {
  double dtau, cf_stp, cf_bak;
};

// ---- tracers, horizontal part: one thread per (i,j,k) cell, all tracers:
// t(nnew) = Hz_bak*(cf_stp*t(nstp)+cf_bak*t(indx)) - dtau*pm*pn*div(FX,FE),
// t(indx) = Hz*t(nstp). ----
__global__ void __launch_bounds__(256) k_pre_tracer_h(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  const uint3 bI = xcd_tile();
  __shared__ TracerWin W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z, indx = 3 - nstp;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2;
  tracer_win_fill(b, F, W, ib, jb, kk, nullptr);
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, i, j), o = ij + kk;
  double hb = 0.0;
  if (act) {
    double hf;
    hz_bak_fwd(d, i, j, k, 0.5 * c.dtau, hb, hf);
    F.c2[o] = hf;  // Hz_fwd, Hz_bak kept for the column solves (range istr-1.., jstr-1..)
    F.c3[o] = hb;
  }
  const bool in = act && i >= b.istr && j >= b.jstr;
  const double hz = in ? F.Hz[o] : 0.0;
  const AccTL a{W.T, W.UM, W.VM, W.FU, W.FV, ib, jb};
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    const long tb = (long)(itrc - 1) * 3 * b.n3;
    const double* Tr = F.t + (long)(nrhs - 1) * b.n3 + tb;
    __syncthreads();  // previous tracer's window fully consumed
    tracer_win_fill(b, F, W, ib, jb, kk, Tr);
    __syncthreads();
    if (!in) continue;
    double* Tn = F.t + (long)(nnew - 1) * b.n3 + tb;
    double* Ti = F.t + (long)(indx - 1) * b.n3 + tb;
    const double* Ts = F.t + (long)(nstp - 1) * b.n3 + tb;
    double FX0 = tracer_fx(b, a, i, j, false), FX1 = tracer_fx(b, a, i + 1, j, false);
    double FE0 = tracer_fe(b, a, i, j, false), FE1 = tracer_fe(b, a, i, j + 1, false);
    if (d.p.nriv > 0) {   // river inflow faces (compute_horiz_tracer_fluxes.h:217-246)
      river_tracer_flux(d, 0, i, j, k, itrc, FX0); river_tracer_flux(d, 0, i + 1, j, k, itrc, FX1);
      river_tracer_flux(d, 1, i, j, k, itrc, FE0); river_tracer_flux(d, 1, i, j + 1, k, itrc, FE1);
    }
    const double tsk = Ts[o];
    Tn[o] = hb * (c.cf_stp * tsk + c.cf_bak * Ti[o]) - c.dtau * F.pm[ij] * F.pn[ij] * (FX1 - FX0 + FE1 - FE0);
    Ti[o] = hz * tsk;
  }
}

// ---- the same for NTT <= 2 tracers with every global load issued at entry:
// the windows (masks, FlxU/FlxV, each tracer) and the lane's own inputs
// (pseudo-continuity terms, t(nstp), t(indx)) land together, so a block waits
// for memory once instead of once per phase.  The per-phase form above waits
// 2 + 2 NT times and, with ~7 blocks per CU, was bound by those round trips,
// not by bandwidth.  Same expressions in the same order: bit-identical. ----
template <int NTT, int TY>
struct TracerWinN {
  static constexpr int kN = kUVW * (TY + 4);
  double UM[kN], VM[kN], FU[kN], FV[kN], T[NTT][kN];
};
// kHB: the interior cells' Hz_bak / Hz_fwd are already in c3 / c2 (the
// predictor's k_omega_seg<true> formed them with this expression); those
// cells load Hz_bak instead of the fluxes and We/Wi, the ring i = istr-1 /
// j = jstr-1 still forms both.
template <int NTT, int TY, bool kHB>
__global__ void __launch_bounds__(kBX * TY) k_pre_tracer_h1(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  const uint3 bI = h_tile(d.p.tile_grp);
  __shared__ TracerWinN<NTT, TY> W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z, indx = 3 - nstp;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * TY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2, n2 = b.n2;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  constexpr int NW = kUVW * (TY + 4), NR = (NW + kBX * TY - 1) / (kBX * TY);
  double wUM[NR], wVM[NR], wFU[NR], wFV[NR], wT[NTT][NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q = tid + r * kBX * TY;
    const int i = ib + q % kUVW, j = jb + q / kUVW;
    const bool ok = q < NW && i >= -1 && i <= b.Lm + 2 && j >= -1 && j <= b.Mm + 2;
    const long o = ok ? IJ(b, i, j) : 0;
    wUM[r] = ok ? F.umask[o] : 0.0;
    wVM[r] = ok ? F.vmask[o] : 0.0;
    wFU[r] = ok ? F.FlxU[o + kk] : 0.0;
    wFV[r] = ok ? F.FlxV[o + kk] : 0.0;
#pragma unroll
    for (int t = 0; t < NTT; t++)
      wT[t][r] = ok ? F.t[(long)(nrhs - 1) * b.n3 + (long)t * 3 * b.n3 + o + kk] : 0.0;
  }
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const bool in = act && i >= b.istr && j >= b.jstr;
  const long ij = act ? IJ(b, i, j) : IJ(b, R.i0, R.j0), o = ij + kk, w = ij + (long)k * n2;
  // hz_bak_fwd's inputs (pre_step3d4S.F:136-148) and the tracer time levels
  const bool formed = kHB && in;   // Hz_bak/fwd from omega
  double fu0 = 0.0, fu1 = 0.0, fv0 = 0.0, fv1 = 0.0, we1 = 0.0, wi1 = 0.0, we0 = 0.0, wi0 = 0.0, hbo = 0.0;
  if (formed) {
    hbo = F.c3[o];
  } else {
    fu0 = F.FlxU[o]; fu1 = F.FlxU[o + 1]; fv0 = F.FlxV[o]; fv1 = F.FlxV[o + b.nx2];
    we1 = F.We[w]; wi1 = F.Wi[w]; we0 = F.We[w - n2]; wi0 = F.Wi[w - n2];
  }
  const double pm = F.pm[ij], pn = F.pn[ij], hzo = F.Hz[o];
  double ts[NTT], ti[NTT];
#pragma unroll
  for (int t = 0; t < NTT; t++) {
    const long tb = (long)t * 3 * b.n3;
    ts[t] = F.t[(long)(nstp - 1) * b.n3 + tb + o];
    ti[t] = F.t[(long)(indx - 1) * b.n3 + tb + o];
  }
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q = tid + r * kBX * TY;
    if (q < NW) {
      W.UM[q] = wUM[r]; W.VM[q] = wVM[r]; W.FU[q] = wFU[r]; W.FV[q] = wFV[r];
#pragma unroll
      for (int t = 0; t < NTT; t++) W.T[t][q] = wT[t][r];
    }
  }
  __syncthreads();
  if (!act) return;
  double hb;
  if (formed) {
    hb = hbo;
  } else {
    const double cff = 0.5 * c.dtau;
    const double FlxDiv = cff * pm * pn * (fu1 - fu0 + fv1 - fv0 + we1 + wi1 - we0 - wi0);
    hb = hzo + FlxDiv;
    const double hf = hzo - FlxDiv;
    F.c2[o] = hf;  // Hz_fwd, Hz_bak kept for the column solves (range istr-1.., jstr-1..)
    F.c3[o] = hb;
  }
  if (!in) return;
  const double hz = hzo;
#pragma unroll
  for (int t = 0; t < NTT; t++) {
    const int itrc = t + 1;
    const AccTL a{W.T[t], W.UM, W.VM, W.FU, W.FV, ib, jb};
    double FX0 = tracer_fx(b, a, i, j, false), FX1 = tracer_fx(b, a, i + 1, j, false);
    double FE0 = tracer_fe(b, a, i, j, false), FE1 = tracer_fe(b, a, i, j + 1, false);
    if (d.p.nriv > 0) {   // river inflow faces (compute_horiz_tracer_fluxes.h:217-246)
      river_tracer_flux(d, 0, i, j, k, itrc, FX0); river_tracer_flux(d, 0, i + 1, j, k, itrc, FX1);
      river_tracer_flux(d, 1, i, j, k, itrc, FE0); river_tracer_flux(d, 1, i, j + 1, k, itrc, FE1);
    }
    const long tb = (long)t * 3 * b.n3;
    const double tsk = ts[t];
    F.t[(long)(nnew - 1) * b.n3 + tb + o] =
        hb * (c.cf_stp * tsk + c.cf_bak * ti[t]) - c.dtau * pm * pn * (FX1 - FX0 + FE1 - FE0);
    F.t[(long)(indx - 1) * b.n3 + tb + o] = hz * tsk;
  }
}

// ---- j-marching form of k_pre_tracer_h1 (Params::h_jc): a block of 64 x 4
// threads walks a 64-wide strip through jc rows of one level, 4 rows per
// step.  The windows (masks, FlxU/FlxV, each tracer) live in an 8-row LDS ring
// (AccTR): each step brings in only the 4 rows the next tile needs beyond the
// ones already there, loaded into registers while the current tile computes
// (with the next tile's lane inputs), so every window row is read from HBM
// once per strip instead of twice (the 64 x 4 tiles' 4-row j-halo: 8 window
// rows per 4 tile rows).  Same expressions, same order: bit-identical. ----
template <int NTT>
struct TracerRing {
  double UM[kRingH * kUVW], VM[kRingH * kUVW], FU[kRingH * kUVW], FV[kRingH * kUVW], T[NTT][kRingH * kUVW];
};
// window rows [r0, r0 + nr) of the ring fields: entry q of the row block is
// register m of thread tid (q = tid + m*256)
template <int NTT, int NR>
struct TracerRows {
  double um[NR], vm[NR], fu[NR], fv[NR], t[NTT][NR];
  __device__ __forceinline__ void load(const Bounds& b, const Fields& F, int tid, int ib, int r0, int nr, long kk,
                                       long tlev) {
#pragma unroll
    for (int m = 0; m < NR; m++) {
      const int q = tid + m * kBX * kBY;
      const int i = ib + q % kUVW, j = r0 + q / kUVW;
      const bool ok = q < nr * kUVW && i >= -1 && i <= b.Lm + 2 && j >= -1 && j <= b.Mm + 2;
      const long o = ok ? IJ(b, i, j) : 0;
      um[m] = ok ? F.umask[o] : 0.0;
      vm[m] = ok ? F.vmask[o] : 0.0;
      fu[m] = ok ? F.FlxU[o + kk] : 0.0;
      fv[m] = ok ? F.FlxV[o + kk] : 0.0;
#pragma unroll
      for (int t = 0; t < NTT; t++) this->t[t][m] = ok ? F.t[tlev + (long)t * 3 * b.n3 + o + kk] : 0.0;
    }
  }
  __device__ __forceinline__ void store(TracerRing<NTT>& W, int tid, int r0, int nr, int jb) const {
#pragma unroll
    for (int m = 0; m < NR; m++) {
      const int q = tid + m * kBX * kBY;
      if (q < nr * kUVW) {
        const int s = (q % kUVW) + ((r0 + q / kUVW - jb) & (kRingH - 1)) * kUVW;
        W.UM[s] = um[m]; W.VM[s] = vm[m]; W.FU[s] = fu[m]; W.FV[s] = fv[m];
#pragma unroll
        for (int t = 0; t < NTT; t++) W.T[t][s] = this->t[t][m];
      }
    }
  }
};
template <int NTT, bool kHB>
__global__ void __launch_bounds__(kBX * kBY) k_pre_tracer_hj(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs,
                                                           int jc) {
  const uint3 bI = xcd_tile();
  __shared__ TracerRing<NTT> W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z, indx = 3 - nstp;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, jc0 = R.j0 + (int)bI.y * jc;
  const int jend = min(jc0 + jc - 1, R.j1);
  const int ib = i0 - 2, jb = jc0 - 2;
  const long kk = (long)(k - 1) * b.n2, n2 = b.n2, tlev = (long)(nrhs - 1) * b.n3;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  constexpr int NT = kBX * kBY;
  constexpr int NR0 = (kRingH * kUVW + NT - 1) / NT, NR4 = (kBY * kUVW + NT - 1) / NT;
  // the lane's own inputs of tile row j (hz_bak_fwd's, pre_step3d4S.F:136-148, and the time levels)
  struct Lane {
    double fu0, fu1, fv0, fv1, we1, wi1, we0, wi0, hbo, pm, pn, hzo, ts[NTT], ti[NTT];
  };
  const int i = i0 + (int)threadIdx.x;
  auto load_lane = [&](Lane& L, int j) {
    const bool act = i >= R.i0 && i <= R.i1 && j <= jend;
    const bool formed = kHB && act && i >= b.istr && j >= b.jstr;
    const long ij = act ? IJ(b, i, j) : IJ(b, R.i0, R.j0), o = ij + kk, w = ij + (long)k * n2;
    L.fu0 = L.fu1 = L.fv0 = L.fv1 = L.we1 = L.wi1 = L.we0 = L.wi0 = L.hbo = 0.0;
    if (formed) {
      L.hbo = F.c3[o];
    } else {
      L.fu0 = F.FlxU[o]; L.fu1 = F.FlxU[o + 1]; L.fv0 = F.FlxV[o]; L.fv1 = F.FlxV[o + b.nx2];
      L.we1 = F.We[w]; L.wi1 = F.Wi[w]; L.we0 = F.We[w - n2]; L.wi0 = F.Wi[w - n2];
    }
    L.pm = F.pm[ij]; L.pn = F.pn[ij]; L.hzo = F.Hz[o];
#pragma unroll
    for (int t = 0; t < NTT; t++) {
      const long tb = (long)t * 3 * b.n3;
      L.ts[t] = F.t[(long)(nstp - 1) * b.n3 + tb + o];
      L.ti[t] = F.t[(long)(indx - 1) * b.n3 + tb + o];
    }
  };
  // prologue: the first tile's window (8 rows) and lane inputs
  Lane L;
  {
    TracerRows<NTT, NR0> X;
    X.load(b, F, tid, ib, jb, kRingH, kk, tlev);
    load_lane(L, jc0 + (int)threadIdx.y);
    X.store(W, tid, jb, kRingH, jb);
  }
  __syncthreads();
  const AccTR a0{nullptr, W.UM, W.VM, W.FU, W.FV, ib, jb};
  for (int j0 = jc0; j0 <= jend; j0 += kBY) {
    const bool more = j0 + kBY <= jend;
    TracerRows<NTT, NR4> X;
    Lane Ln;
    if (more) {   // the next tile's 4 new window rows and lane inputs, in flight during this tile
      X.load(b, F, tid, ib, j0 + kBY + 2, kBY, kk, tlev);
      load_lane(Ln, j0 + kBY + (int)threadIdx.y);
    }
    const int j = j0 + (int)threadIdx.y;
    const bool act = i >= R.i0 && i <= R.i1 && j <= jend;
    const bool in = act && i >= b.istr && j >= b.jstr;
    if (act) {
      const long ij = IJ(b, i, j), o = ij + kk;
      double hb;
      if (kHB && in) {
        hb = L.hbo;
      } else {
        const double cff = 0.5 * c.dtau;
        const double FlxDiv = cff * L.pm * L.pn * (L.fu1 - L.fu0 + L.fv1 - L.fv0 + L.we1 + L.wi1 - L.we0 - L.wi0);
        hb = L.hzo + FlxDiv;
        const double hf = L.hzo - FlxDiv;
        F.c2[o] = hf;  // Hz_fwd, Hz_bak kept for the column solves (range istr-1.., jstr-1..)
        F.c3[o] = hb;
      }
      if (in) {
        const double hz = L.hzo;
#pragma unroll
        for (int t = 0; t < NTT; t++) {
          const int itrc = t + 1;
          AccTR a = a0;
          a.T = W.T[t];
          double FX0 = tracer_fx(b, a, i, j, false), FX1 = tracer_fx(b, a, i + 1, j, false);
          double FE0 = tracer_fe(b, a, i, j, false), FE1 = tracer_fe(b, a, i, j + 1, false);
          if (d.p.nriv > 0) {   // river inflow faces (compute_horiz_tracer_fluxes.h:217-246)
            river_tracer_flux(d, 0, i, j, k, itrc, FX0); river_tracer_flux(d, 0, i + 1, j, k, itrc, FX1);
            river_tracer_flux(d, 1, i, j, k, itrc, FE0); river_tracer_flux(d, 1, i, j + 1, k, itrc, FE1);
          }
          const long tb = (long)t * 3 * b.n3;
          const double tsk = L.ts[t];
          F.t[(long)(nnew - 1) * b.n3 + tb + o] =
              hb * (c.cf_stp * tsk + c.cf_bak * L.ti[t]) - c.dtau * L.pm * L.pn * (FX1 - FX0 + FE1 - FE0);
          F.t[(long)(indx - 1) * b.n3 + tb + o] = hz * tsk;
        }
      }
    }
    if (!more) break;
    __syncthreads();   // this tile's reads of the 4 oldest rows are done
    X.store(W, tid, j0 + kBY + 2, kBY, jb);
    L = Ln;
    __syncthreads();
  }
}

// ---- tracers, vertical part per column: spline advection on t(nrhs), then
// implicit diffusion with Wi up-winding on Hz_fwd (LDS slots A, B). ----
template <class C>
__global__ void __launch_bounds__(64) k_pre_tracer_v(Dev d, Range R, PreCoef c, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<C>(2, d.b.N);
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ We = F.We + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const C A = ColMake<C>::at(d, 0, (int)bI.z, ij), B = ColMake<C>::at(d, 1, (int)bI.z, ij);
  const double* __restrict__ Hf = F.c2 + ij;
  auto hfwd = [&](int k) { return Hf[(long)(k - 1) * n2]; };
  {
    const int itrc = 1 + (int)bI.z;
    const long tb = (long)(itrc - 1) * 3 * b.n3;
    const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + tb + ij;
    double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + tb + ij;
    tracer_spline_lds(N, n2, Hz, Tr, We, A, B);
    auto tval_of = [&](int k, double tnk) {
      return tnk - c.dtau * F.pm[ij] * F.pn[ij] * (A[k] - A[k - 1]);
    };
    auto tval = [&](int k) { return tval_of(k, Tn[(long)(k - 1) * n2]); };
    const int iAkt = itrc < b.nTS ? itrc : b.nTS;
    const double* __restrict__ Akt = F.Akt + (long)(iAkt - 1) * b.n3w + ij;
    const double DC0 = c.dtau * F.pm[ij] * F.pn[ij];
    const double hf1 = hfwd(1);
    double hfk = hfwd(2);
    double FCk = 2.0 * c.dtau * Akt[n2] / (hfk + hf1);
    double WCk = DC0 * Wi[n2];
    double cff = 1.0 / (hf1 + FCk + fmax0(WCk));
    double CFk = cff * (FCk - fmin0(WCk));
    double DCk = cff * tval(1);
    B[1] = CFk;
    A[0] = DCk;
    {
      auto thomas = [&](int k, double hfk1, double akt, double wi, double tn) {
        const double FCn = 2.0 * c.dtau * akt / (hfk1 + hfk);
        const double WCn = DC0 * wi;
        cff = 1.0 / (hfk + FCn + fmax0(WCn) + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
        const double CFn = cff * (FCn - fmin0(WCn));
        const double DCn = cff * (tval_of(k, tn) + DCk * (FCk + fmax0(WCk)));
        B[k] = CFn;
        A[k - 1] = DCn;
        FCk = FCn; WCk = WCn; CFk = CFn; DCk = DCn; hfk = hfk1;
      };
      double rhf[kPF], ra[kPF], rwi[kPF], rtn[kPF];  // Hz_fwd(k+1), Akt(k), Wi(k), Tn(k) of level k
#pragma unroll
      for (int q = 0; q < kPF; q++) {
        const int k = min(2 + q, N - 1);
        rhf[q] = Hf[(long)k * n2]; ra[q] = Akt[(long)k * n2]; rwi[q] = Wi[(long)k * n2];
        rtn[q] = Tn[(long)(k - 1) * n2];
      }
      int k2 = 2;
      for (; k2 + kPF - 1 <= N - 1; k2 += kPF) {
#pragma unroll
        for (int q = 0; q < kPF; q++) {
          const double hf1 = rhf[q], akt = ra[q], wi = rwi[q], tn = rtn[q];
          const int kn = min(k2 + q + kPF, N - 1);
          rhf[q] = Hf[(long)kn * n2]; ra[q] = Akt[(long)kn * n2]; rwi[q] = Wi[(long)kn * n2];
          rtn[q] = Tn[(long)(kn - 1) * n2];
          thomas(k2 + q, hf1, akt, wi, tn);
        }
      }
      for (int k = k2; k <= N - 1; k++) thomas(k, Hf[(long)k * n2], Akt[(long)k * n2], Wi[(long)k * n2], Tn[(long)(k - 1) * n2]);
    }
    const long oN = (long)(N - 1) * n2;
    double tt = (tval(N) + DCk * (FCk + fmax0(WCk))) / (hfk + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
    Tn[oN] = tt;
#pragma unroll 8
    for (int k = N - 1; k >= 1; k--) {
      tt = A[k - 1] + B[k] * tt;
      Tn[(long)(k - 1) * n2] = tt;
    }
  }
}

// ---- register-resident k_pre_tracer_v for a compile-time depth NN: the
// FC/DC column in VGPRs, CF in one LDS slot (26 KB per wave at N = 50, six
// waves per CU instead of three); fully unrolled, same expressions and order,
// bit-identical. ----
template <int NN>
__global__ void __launch_bounds__(64, 2) k_pre_tracer_v_reg(Dev d, Range R, PreCoef c, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<ColLds>(1, NN);
  const Bounds& b = d.b;
  const Fields& F = d.f;
  constexpr int N = NN;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ We = F.We + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double* __restrict__ Hf = F.c2 + ij;
  const ColLds B = col_lds(0, N);
  double A[N + 1];
  const int itrc = 1 + (int)bI.z;
  const long tb = (long)(itrc - 1) * 3 * b.n3;
  const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + tb + ij;
  double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + tb + ij;
  tracer_spline_reg<N>(n2, Hz, Tr, We, A, B);
  const double pm = F.pm[ij], pn = F.pn[ij];
  auto tval = [&](int k) { return Tn[(long)(k - 1) * n2] - c.dtau * pm * pn * (A[k] - A[k - 1]); };
  const int iAkt = itrc < b.nTS ? itrc : b.nTS;
  const double* __restrict__ Akt = F.Akt + (long)(iAkt - 1) * b.n3w + ij;
  const double DC0 = c.dtau * pm * pn;
  const double hf1 = Hf[0];
  double hfk = Hf[n2];
  double FCk = 2.0 * c.dtau * Akt[n2] / (hfk + hf1);
  double WCk = DC0 * Wi[n2];
  double cff = 1.0 / (hf1 + FCk + fmax0(WCk));
  double CFk = cff * (FCk - fmin0(WCk));
  double DCk = cff * tval(1);
  B[1] = CFk;
  A[0] = DCk;
#pragma unroll
  for (int k = 2; k <= N - 1; k++) {
    const double hfk1 = Hf[(long)k * n2];
    const double FCn = 2.0 * c.dtau * Akt[(long)k * n2] / (hfk1 + hfk);
    const double WCn = DC0 * Wi[(long)k * n2];
    cff = 1.0 / (hfk + FCn + fmax0(WCn) + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
    const double CFn = cff * (FCn - fmin0(WCn));
    const double DCn = cff * (tval(k) + DCk * (FCk + fmax0(WCk)));
    B[k] = CFn;
    A[k - 1] = DCn;
    FCk = FCn; WCk = WCn; CFk = CFn; DCk = DCn; hfk = hfk1;
  }
  const long oN = (long)(N - 1) * n2;
  double tt = (tval(N) + DCk * (FCk + fmax0(WCk))) / (hfk + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
  Tn[oN] = tt;
#pragma unroll
  for (int k = N - 1; k >= 1; k--) {
    tt = A[k - 1] + B[k] * tt;
    Tn[(long)(k - 1) * n2] = tt;
  }
}

// ---- horizontal momentum r.h.s., one (i,j,k) cell per thread; u, v,
// FlxU, FlxV of the block's 64x4 tile plus a 2-cell halo staged in LDS ----
__global__ void __launch_bounds__(256) k_uv_horiz(Dev d, Range R, int nrhs, UVBounds ub, int up) {
  const uint3 bI = xcd_tile();
  __shared__ double sU[kUVN], sV[kUVN], sFU[kUVN], sFV[kUVN];
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2;
  const double* U = F.u + (long)(nrhs - 1) * b.n3 + kk;
  const double* V = F.v + (long)(nrhs - 1) * b.n3 + kk;
  const double* FU = F.FlxU + kk;
  const double* FV = F.FlxV + kk;
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  for (int q = threadIdx.x + kBX * threadIdx.y; q < kUVN; q += kBX * kBY) {
    const int ii = ib + q % kUVW, jj = jb + q / kUVW;
    if (ii < -1 || ii > b.Lm + 2 || jj < -1 || jj > b.Mm + 2) continue;  // never read
    const long o = IJ(b, ii, jj);
    sU[q] = U[o];
    sV[q] = V[o];
    sFU[q] = FU[o];
    sFV[q] = FV[o];
  }
  __syncthreads();
  if (!act) return;
  const AccL a{sU, sV, sFU, sFV, ib, jb};
  uv_horiz_rhs(d, a, i, j, k, ub, up != 0);
}

// The same without CURVGRID with every global load issued at block entry
// (the window and the lane's own ru, rv, Hz, fomn): one memory wait per
// block.  Bit-identical.
template <int TY>
__global__ void __launch_bounds__(kBX * TY) k_uv_horiz1(Dev d, Range R, int nrhs, UVBounds ub, int up) {
  const uint3 bI = h_tile(d.p.tile_grp);
  constexpr int NW = kUVW * (TY + 4);
  __shared__ double sU[NW], sV[NW], sFU[NW], sFV[NW];
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * TY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2;
  const double* U = F.u + (long)(nrhs - 1) * b.n3 + kk;
  const double* V = F.v + (long)(nrhs - 1) * b.n3 + kk;
  const double* FU = F.FlxU + kk;
  const double* FV = F.FlxV + kk;
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  constexpr int NR = (NW + kBX * TY - 1) / (kBX * TY);
  double wU[NR], wV[NR], wFU[NR], wFV[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q = tid + r * kBX * TY;
    const int ii = ib + q % kUVW, jj = jb + q / kUVW;
    const bool ok = q < NW && ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2;
    const long o = ok ? IJ(b, ii, jj) : 0;
    wU[r] = ok ? U[o] : 0.0;
    wV[r] = ok ? V[o] : 0.0;
    wFU[r] = ok ? FU[o] : 0.0;
    wFV[r] = ok ? FV[o] : 0.0;
  }
  const long ij = act ? IJ(b, i, j) : IJ(b, R.i0, R.j0), o = ij + kk;
  UVPre p;
  p.ru = F.ru[o]; p.rv = F.rv[o];
  p.hz0 = p.hzx = p.hzy = p.f0 = p.fx = p.fy = 0.0;
  if (d.p.uv_cor) {
    p.hz0 = F.Hz[o]; p.hzx = F.Hz[o - 1]; p.hzy = F.Hz[o - b.nx2];
    p.f0 = F.fomn[ij]; p.fx = F.fomn[ij - 1]; p.fy = F.fomn[ij - b.nx2];
  }
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q = tid + r * kBX * TY;
    if (q < NW) { sU[q] = wU[r]; sV[q] = wV[r]; sFU[q] = wFU[r]; sFV[q] = wFV[r]; }
  }
  __syncthreads();
  if (!act) return;
  const AccL a{sU, sV, sFU, sFV, ib, jb};
  uv_horiz_rhs_pre(d, a, i, j, o, p, ub, up != 0);
}


void launch_uv_horiz(const Dev& d, hipStream_t s, int nrhs, int up) {
  const Bounds& b = d.b;
  if (!d.p.uv_cor && !d.p.uv_adv) return;   // compute_horiz_rhs_uv_terms.h adds nothing
  Range R{b.istr, b.iend, b.jstr, b.jend};
  const UVBounds ub = uv_bounds(b);
  if (!d.p.hoist || d.p.curvgrid)
    hipLaunchKernelGGL(k_uv_horiz, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, nrhs, ub, up);
  else if (d.p.h_ty == 8)
    hipLaunchKernelGGL(k_uv_horiz1<8>, grid3_ty(R, b.N, 8), dim3(kBX, 8), 0, s, d, R, nrhs, ub, up);
  else
    hipLaunchKernelGGL(k_uv_horiz1<4>, grid3_ty(R, b.N, 4), dim3(kBX, 4), 0, s, d, R, nrhs, ub, up);
}

// ---- bottom drag r_D (compute_rd_bott_drag.h), log-layer with Zob ----
__global__ void __launch_bounds__(256) k_rd(Dev d, Range R, int nstp) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j);
  if (d.p.Zob > 0.0) {
    const double* U = F.u + (long)(nstp - 1) * b.n3;
    const double* V = F.v + (long)(nstp - 1) * b.n3;
    const double u0 = U[ij], u1 = U[ij + 1], v0 = V[ij], v1 = V[ij + b.nx2];
    const double cff = sqrt(0.333333333333 * (u0 * u0 + u1 * u1 + u0 * u1 + v0 * v0 + v1 * v1 + v0 * v1));
    const double q = d.p.vonKar / log(1.0 + 0.5 * F.Hz[ij] / d.p.Zob);
    F.r_D[ij] = cff * (q * q);
  } else {
    double rd = d.p.rdrg;
    F.r_D[ij] = dmin(rd, 0.8 * F.Hz[ij] / d.p.dt);
  }
}

// ---- momentum, per column: vertical spline advection into ru/rv, then
// implicit viscosity with implicit no-slip bottom (IMPLCT_NO_SLIP_BTTM_BC).
// LDS: A = spline FC -> flux -> DC(k); B = spline CF -> CF(k-1). ----
#ifndef ROMS_PREUV_PF
#define ROMS_PREUV_PF 8
#endif
constexpr int kPreUvPF = ROMS_PREUV_PF;   // levels of loads in flight in pre_uv_col's forward sweep
template <class C>
__device__ __forceinline__ void pre_uv_col(const Dev& d, int i, int j, int dir, const PreCoef& c, int nstp, int nnew,
                                           int nrhs, const C& A, const C& B) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, indx = 3 - nstp;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const long s = dir == 0 ? 1 : b.nx2;
#ifdef ROMS_PREUV_SPLINE_PLAIN
  uv_vert_flux_lds<false>(d, ij, nrhs, dir, A, B);
#else
  uv_vert_flux_lds<true>(d, ij, nrhs, dir, A, B);
#endif
  double* Uall = dir == 0 ? F.u : F.v;
  const double* __restrict__ rr = (dir == 0 ? F.ru : F.rv) + ij;
  const double* __restrict__ Ustp = Uall + (long)(nstp - 1) * b.n3 + ij;
  double* __restrict__ Uidx = Uall + (long)(indx - 1) * b.n3 + ij;
  double* __restrict__ Unew = Uall + (long)(nnew - 1) * b.n3 + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Akv = F.Akv + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = c.dtau * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  // DC(k) before elimination; also stores u(indx) = Hz*u(nstp).  The updated
  // ru(k) is dead after pre_step3d -- the corrector's prsgrd assigns ru before
  // any read (prsgrd.F:293) -- so it is not stored (as in k_pre_uv_seg)
  auto DCinit = [&](int k, double hbk, double hbkm) {
    const long o = (long)(k - 1) * n2;
    const double r = uv_rr_update(rr[o], A, k);
    const double us = Ustp[o];
    const double v = 0.5 * (hbk + hbkm) * (c.cf_stp * us + c.cf_bak * Uidx[o]) + DC0 * r;
    Uidx[o] = 0.5 * (Hz[o] + Hz[o - s]) * us;
    return v;
  };
  const double* __restrict__ Hf = F.c2 + ij;
  const double* __restrict__ Hb = F.c3 + ij;
  const long ms = dir == 0 ? -1 : -(long)b.nx2;   // offset of the (im,jm) column
  auto lev = [&](int k) { return (long)(k - 1) * n2; };
  const double hbN = Hb[lev(N)], hfN = Hf[lev(N)], hbNm = Hb[lev(N) + ms], hfNm = Hf[lev(N) + ms];
  double hbK = Hb[lev(N - 1)], hfK = Hf[lev(N - 1)], hbKm = Hb[lev(N - 1) + ms], hfKm = Hf[lev(N - 1) + ms];
  double FCk = 2.0 * c.dtau * (Akv[(long)(N - 1) * n2] + Akv[(long)(N - 1) * n2 - s]) / (hfN + hfNm + hfK + hfKm);
  double WCk = DC0 * 0.5 * (Wi[(long)(N - 1) * n2] + Wi[(long)(N - 1) * n2 - s]);
  double cff = 1.0 / (0.5 * (hfN + hfNm) + FCk - fmin0(WCk));
  double CFk = cff * (FCk + fmax0(WCk));             // CF(N-1)
  double DCk1 = cff * (DCinit(N, hbN, hbNm) + c.dtau * sstr);  // DC(N)
  A[N] = DCk1;
  B[N - 1] = CFk;
  // Forward elimination, levels N-1..2.  Iteration k reads level k-1 of
  // Hb/Hf/Akv/Wi and level k of ru/u/Hz, and stores u(indx)(k).
  // The compiler cannot prove the u stores of level k miss the loads of
  // the levels below (same arrays, offsets n2 apart), so it issues no load
  // ahead of a store; a ring of kPF iterations' raw loads, refilled before
  // each iteration's stores, keeps kPF levels of loads in flight.  At
  // <= 1 wave per SIMD (two LDS column slots per wave) the ring's VGPRs cost
  // no occupancy.  Same arithmetic in the same order as the reference loop.
  struct Lv { double hb, hf, hbm, hfm, ak, aks, wi, wis, r, us, ui, hz, hzs; };
  auto load = [&](int k) {   // the raw loads of iteration k (clamped to a valid level)
    k = k < 2 ? 2 : k;
    const long o = lev(k), l = lev(k - 1);
    return Lv{Hb[l], Hf[l], Hb[l + ms], Hf[l + ms], Akv[o], Akv[o - s], Wi[o], Wi[o - s],   // w-level k-1
              rr[o], Ustp[o], Uidx[o], Hz[o], Hz[o - s]};
  };
  auto iter = [&](int k, const Lv& v) {
    const double FCl = 2.0 * c.dtau * (v.ak + v.aks) / (hfK + hfKm + v.hf + v.hfm);
    const double WCl = DC0 * 0.5 * (v.wi + v.wis);
    cff = 1.0 / (0.5 * (hfK + hfKm) + FCl - fmin0(WCl) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
    const double CFl = cff * (FCl + fmax0(WCl));
    const long o = lev(k);
    const double r = uv_rr_update(v.r, A, k);
    const double dci = 0.5 * (hbK + hbKm) * (c.cf_stp * v.us + c.cf_bak * v.ui) + DC0 * r;
    Uidx[o] = 0.5 * (v.hz + v.hzs) * v.us;
    const double DCk = cff * (dci + DCk1 * (FCk - fmin0(WCk)));
    B[k - 1] = CFl;
    A[k] = DCk;
    DCk1 = DCk; FCk = FCl; WCk = WCl; CFk = CFl;
    hbK = v.hb; hfK = v.hf; hbKm = v.hbm; hfKm = v.hfm;
  };
  constexpr int PF = kPreUvPF;
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
  const double rd = F.r_D[ij], rdm = F.r_D[ij - s];
  double un = (DCinit(1, hbK, hbKm) + DCk1 * (FCk - fmin0(WCk))) /
              (0.5 * (hfK + hfKm) + 0.5 * c.dtau * (rd + rdm) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
  Unew[0] = un;
#pragma unroll 8
  for (int k = 2; k <= N; k++) {
    un = A[k] + B[k - 1] * un;
    Unew[(long)(k - 1) * n2] = un;
  }
}

template <class C>
__global__ void __launch_bounds__(64) k_pre_uv(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<C>(2, d.b.N);
  const Bounds& b = d.b;
  const long ij = IJ(b, i, j);
  const C A = ColMake<C>::at(d, 0, (int)bI.z, ij), B = ColMake<C>::at(d, 1, (int)bI.z, ij);
  if (bI.z == 0) {
    if (i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend) pre_uv_col(d, i, j, 0, c, nstp, nnew, nrhs, A, B);
  } else {
    if (i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend) pre_uv_col(d, i, j, 1, c, nstp, nnew, nrhs, A, B);
  }
}

// ---- segment-partitioned variants (k_colseg.h) for deep grids: block =
// kSegCW columns x S segments.  The spline reconstruction and the implicit
// diffusion / viscosity are each one partitioned tridiagonal system whose
// rows are those of k_pre_tracer_v / pre_uv_col (pre_step3d4S.F:198-489). ----
__global__ void __launch_bounds__(kSegBlock, 2) k_pre_tracer_seg(Dev d, Range R, PreCoef c, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const SegSpan sg = seg_span(N);
  const int iu = tile_i0(R.i0) + (int)bI.x * kSegCW + sg.col;
  const bool act = iu >= R.i0 && iu <= R.i1;
  const int i = act ? iu : (iu < R.i0 ? R.i0 : R.i1), j = R.j0 + (int)bI.y;
  const int itrc = 1 + (int)bI.z;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const int c0 = sg.c0, n = sg.n;
  auto cell = [&](int k) { return (long)(min(max(k, 1), N) - 1) * n2; };   // rho level k (clamped)
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Hf = F.c2 + ij;   // Hz_fwd (k_pre_tracer_h)
  const long tb = (long)(itrc - 1) * 3 * b.n3;
  const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + tb + ij;
  double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + tb + ij;
  double hz[KR + 1], tt[KR], fl[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {   // all rows, clamped levels: straight-line loads
    hz[q] = Hz[cell(c0 - 1 + q)];
    if (q < KR) tt[q] = Tr[cell(c0 - 1 + q)];
  }
  tracer_spline_seg<KR>(sg, N, n2, X, hz, tt, F.We + ij, fl);
  // implicit diffusion on Hz_fwd, cells k = c0+p (its loads kept out of the spline phase)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < KR + 1; q++) hz[q] = Hf[cell(c0 - 1 + q)];
  const int iAkt = itrc < b.nTS ? itrc : b.nTS;
  const double* __restrict__ Akt = F.Akt + (long)(iAkt - 1) * b.n3w + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double DC0 = c.dtau * F.pm[ij] * F.pn[ij];
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q (0 at the bottom and the surface)
    const int r = c0 - 1 + q;
    const long w = (long)min(max(r, 1), N - 1) * n2;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * c.dtau * Akt[w], hz[qa] + hz[q]);
    const double wv = DC0 * Wi[w];
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.eliminate(n, [&](int p, double& a, double& bb, double& cc, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    a = -(fcl + fmax0(wcl));
    bb = hz[p + 1] + fcu + fmax0(wcu) + fcl - fmin0(wcl);
    cc = -(fcu - fmin0(wcu));
    dd = Tn[cell(c0 + p)] - c.dtau * F.pm[ij] * F.pn[ij] * (fl[p + 1 < KR ? p + 1 : KR - 1] - fl[p]);
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  if (act) {
#pragma unroll
    for (int p = 0; p < KR; p++)
      if (p < n) Tn[cell(c0 + p)] = T.D[p];
  }
}

// ---- k_pre_tracer_seg with buffer loads/stores (Params::seg_buf, see
// k_step3d_t_segb): wave-uniform level offsets in SGPRs, the lane's column in
// one VGPR.  PF: the diffusion phase's t(nnew) rows and Hz_fwd loaded at
// entry with the spline inputs.  Same expressions and order: bitwise equal
// to k_pre_tracer_seg. ----
template <bool PF, bool UNI = true>
__global__ void __launch_bounds__(kSegBlock, ROMS_PRE_T_SEG_WAVES) k_pre_tracer_segb(Dev d, Range R, PreCoef c, int nnew,
                                                                                   int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  SegSpan sg = seg_span(N);
  constexpr bool kU = UNI && kSegCW == kCX;   // scalar level offsets need one segment per wavefront
  if constexpr (kU) seg_uniform(sg);
  // UNI: level offsets in the SGPR soffset; else added to the VGPR offset
  auto LD = [&](const BufF64& B, unsigned v, unsigned l) { return kU ? B.ld(v, l) : B.ld(v + l, 0u); };
  auto ST = [&](const BufF64& B, double x, unsigned v, unsigned l) {
    if constexpr (kU) B.st(x, v, l);
    else B.st(x, v + l, 0u);   // v = kBufOff stays beyond the extent
  };
  const int iu = tile_i0(R.i0) + (int)bI.x * kSegCW + sg.col;
  const bool act = iu >= R.i0 && iu <= R.i1;
  const int i = act ? iu : (iu < R.i0 ? R.i0 : R.i1), j = R.j0 + (int)bI.y;
  const int itrc = 1 + (int)bI.z;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const int c0 = sg.c0, n = sg.n;
  const unsigned vo = (unsigned)ij * 8u;
  auto lev = [&](int k) { return (unsigned)(min(max(k, 1), N) - 1) * (unsigned)n2 * 8u; };
  auto wlev = [&](int r) { return (unsigned)min(max(r, 1), N - 1) * (unsigned)n2 * 8u; };
  const BufF64 Hz(F.Hz), Hf(F.c2), We(F.We), Wi(F.Wi);
  const long tb = (long)(itrc - 1) * 3 * b.n3;
  const BufF64 Tr(F.t + (long)(nrhs - 1) * b.n3 + tb), Tn(F.t + (long)(nnew - 1) * b.n3 + tb);
  double hz[KR + 1], tt[KR], fl[KR], hf[KR + 1], tn[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {
    hz[q] = LD(Hz, vo, lev(c0 - 1 + q));
    if (q < KR) tt[q] = LD(Tr, vo, lev(c0 - 1 + q));
  }
  if constexpr (PF) {
#pragma unroll
    for (int q = 0; q < KR + 1; q++) {
      hf[q] = LD(Hf, vo, lev(c0 - 1 + q));
      if (q < KR) tn[q] = LD(Tn, vo, lev(c0 + q));
    }
  }
  spline_fc_seg<KR>(sg, N, X, hz, tt, fl);
  {
    double we[KR];
#pragma unroll
    for (int q = 0; q < KR; q++) we[q] = LD(We, vo, wlev(c0 - 1 + q));
#pragma unroll
    for (int q = 0; q < KR; q++) pin(we[q]);
#pragma unroll
    for (int q = 0; q < KR; q++) {
      const int r = c0 - 1 + q;
      fl[q] = (r == 0 || r == N) ? 0.0 : fl[q] * we[q];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < KR + 1; q++) hz[q] = PF ? hf[q] : LD(Hf, vo, lev(c0 - 1 + q));
  const int iAkt = itrc < b.nTS ? itrc : b.nTS;
  const BufF64 Akt(F.Akt + (long)(iAkt - 1) * b.n3w);
  const BufF64 Pm(F.pm), Pn(F.pn);   // 2-D metrics through the lane's offset too (no 64-bit ij kept live)
  const double pm = LD(Pm, vo, 0), pn = LD(Pn, vo, 0);
  const double DC0 = c.dtau * pm * pn;
  auto fcw = [&](int q, double& fc, double& wc) {
    const int r = c0 - 1 + q;
    const unsigned w = wlev(r);
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * c.dtau * LD(Akt, vo, w), hz[qa] + hz[q]);
    const double wv = DC0 * LD(Wi, vo, w);
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.eliminate(n, [&](int p, double& a, double& bb, double& cc, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    a = -(fcl + fmax0(wcl));
    bb = hz[p + 1] + fcu + fmax0(wcu) + fcl - fmin0(wcl);
    cc = -(fcu - fmin0(wcu));
    dd = (PF ? tn[p] : LD(Tn, vo, lev(c0 + p))) - c.dtau * pm * pn * (fl[p + 1 < KR ? p + 1 : KR - 1] - fl[p]);
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  const unsigned vs = act ? vo : kBufOff;
#pragma unroll
  for (int p = 0; p < KR; p++)
    if (p < n) ST(Tn, T.D[p], vs, lev(c0 + p));
}

// kLds (UV_ADV, nrhs == nstp -- always so in the predictor): the spline
// phase, which loads Hz, Hz of the (i-1)/(j-1) neighbour and u(nrhs) = u(nstp)
// of every row anyway, also loads u(indx) and leaves in dynamic LDS the row's
// cf_stp*u(nstp) + cf_bak*u(indx) and the new u(indx) = Hz*u(nstp); the
// viscosity phase and the store phase then read no u(nstp), u(indx) or Hz
// (at C3 these reloads missed L2: 4 of the v column's 18 array passes).
// Dynamic LDS: 2 x (KR-1) doubles per thread, [row][thread].
template <bool kLds>
__global__ void __launch_bounds__(kSegBlock * kSegJMax, 2) k_pre_uv_seg(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, indx = 3 - nstp;
  const SegSpan sg = seg_span(N);
  SegCol col;
  seg_uv_col(d, R, bI, sg, col);
  if (col.idle) return;   // uniform over the block
  const int dir = col.dir;
  const bool act = col.act;
  const long n2 = b.n2, ij = IJ(b, col.i, col.j), s = dir == 0 ? 1 : b.nx2;
  const int c0 = sg.c0, n = sg.n;
  auto cell = [&](int k) { return (long)(min(max(k, 1), N) - 1) * n2; };   // rho level k (clamped)
  double* Uall = dir == 0 ? F.u : F.v;
  const int nthr = (int)(blockDim.x * blockDim.y * blockDim.z);
  const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  double* const Sb = roms_smem + tid;                        // row q-1: cf_stp*u(nstp) + cf_bak*u(indx)
  double* const Su = roms_smem + (long)(KR - 1) * nthr + tid;  // row q-1: Hz*u(nstp), the new u(indx)
  double fl[KR];
  if constexpr (kLds) {
    const double* __restrict__ Uix = Uall + (long)(indx - 1) * b.n3 + ij;
    uv_spline_seg<KR>(d, sg, X, ij, nrhs, dir, fl, [&](int q, long L, double h0, double h1, double u) {
      if (q >= 1 && q < KR) {   // cells c0..c0+KR-2 (q is a constant of the unrolled load loop)
        Sb[(q - 1) * nthr] = c.cf_stp * u + c.cf_bak * Uix[L];
        Su[(q - 1) * nthr] = 0.5 * (h0 + h1) * u;
      }
    });
  } else {
    uv_spline_seg<KR>(d, sg, X, ij, nrhs, dir, fl);
  }
  __builtin_amdgcn_sched_barrier(0);   // the viscosity phase's loads stay out of the spline phase
  const double* __restrict__ rr = (dir == 0 ? F.ru : F.rv) + ij;
  const double* __restrict__ Ustp = Uall + (long)(nstp - 1) * b.n3 + ij;
  double* __restrict__ Uidx = Uall + (long)(indx - 1) * b.n3 + ij;
  double* __restrict__ Unew = Uall + (long)(nnew - 1) * b.n3 + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Akv = F.Akv + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double* __restrict__ Hf = F.c2 + ij;   // Hz_fwd, Hz_bak (k_pre_tracer_h)
  const double* __restrict__ Hb = F.c3 + ij;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = c.dtau * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  // row p's right-hand side: ru(k) with the vertical advection (uv_rr_update;
  // the updated ru itself is dead -- the corrector's prsgrd overwrites it,
  // prsgrd.F:293 -- so it is not stored); u(indx) = Hz*u(nstp) is stored
  // after the solve, so the rows carry no stores (no may-alias ordering)
  auto rhs = [&](int p) {
    const int k = c0 + p;
    const long o = cell(k);
    const double r = k == 1 ? rr[o] - fl[1] : rr[o] - fl[p + 1 < KR ? p + 1 : KR - 1] + fl[p];
    double ub;
    if constexpr (kLds) ub = Sb[(p < KR - 1 ? p : KR - 2) * nthr];
    else ub = c.cf_stp * Ustp[o] + c.cf_bak * Uidx[o];
    const double v = 0.5 * (Hb[o] + Hb[o - s]) * ub + DC0 * r;
    return k == N ? v + c.dtau * sstr : v;
  };
  double hf[KR + 1], hfm[KR + 1];   // Hz_fwd(c0-1+q) of the column and of its (i-1) / (j-1) neighbour
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {
    const long L = cell(c0 - 1 + q);
    hf[q] = Hf[L];
    hfm[q] = Hf[L - s];
  }
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q (0 at the bottom and the surface)
    const int r = c0 - 1 + q;
    const long w = (long)min(max(r, 1), N - 1) * n2;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * c.dtau * (Akv[w] + Akv[w - s]), hf[qa] + hfm[qa] + hf[q] + hfm[q]);
    const double wv = DC0 * 0.5 * (Wi[w] + Wi[w - s]);
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  const double rd = F.r_D[ij], rdm = F.r_D[ij - s];
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
    const double b1 = 0.5 * (hf[p + 1] + hfm[p + 1]) + 0.5 * c.dtau * (rd + rdm) + fcu + fmax0(wcu);
    const double bk = 0.5 * (hf[p + 1] + hfm[p + 1]) + fcl - fmin0(wcl) + fcu + fmax0(wcu);
    bb = k == 1 ? b1 : bk;
    dd = rhs(p);
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  if (act) {
    // u(indx) = Hz*u(nstp): from LDS (kLds), else formed here from reloads
    // rather than kept in registers across the solve
    double uix[KR];
#pragma unroll
    for (int p = 0; p < KR; p++) {
      const long o = cell(c0 + p);
      if constexpr (kLds) uix[p] = Su[(p < KR - 1 ? p : KR - 2) * nthr];
      else uix[p] = 0.5 * (Hz[o] + Hz[o - s]) * Ustp[o];
    }
#pragma unroll
    for (int p = 0; p < KR; p++)
      if (p < n) {
        Unew[cell(c0 + p)] = T.D[p];
        Uidx[cell(c0 + p)] = uix[p];
      }
  }
}

// ---- k_pre_uv_seg<true> with buffer loads/stores (Params::seg_buf bit
// 128): wave-uniform level offsets in SGPRs (seg_uniform), the lane's column
// and its neighbour in VGPR offsets.  Same expressions and order: bitwise
// equal to k_pre_uv_seg<true>.  PF: the viscosity rows' Hz_fwd pairs
// loaded at entry with the spline inputs. ----
template <bool PF, bool UNI = true>
__global__ void __launch_bounds__(kSegBlock * kSegJMax, 2) k_pre_uv_segb(Dev d, Range R, PreCoef c, int nstp, int nnew,
                                                                         int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, indx = 3 - nstp;
  SegSpan sg = seg_span(N);
  constexpr bool kU = UNI && kSegCW == kCX;   // scalar level offsets need one segment per wavefront
  if constexpr (kU) seg_uniform(sg);
  // UNI: level offsets in the SGPR soffset; else added to the VGPR offset
  auto LD = [&](const BufF64& B, unsigned v, unsigned l) { return kU ? B.ld(v, l) : B.ld(v + l, 0u); };
  auto ST = [&](const BufF64& B, double x, unsigned v, unsigned l) {
    if constexpr (kU) B.st(x, v, l);
    else B.st(x, v + l, 0u);   // v = kBufOff stays beyond the extent
  };
  SegCol col;
  seg_uv_col(d, R, bI, sg, col);
  if (col.idle) return;   // uniform over the block
  const int dir = col.dir;
  const bool act = col.act;
  const long n2 = b.n2, ij = IJ(b, col.i, col.j), s = dir == 0 ? 1 : b.nx2;
  const int c0 = sg.c0, n = sg.n;
  const unsigned lv = (unsigned)n2 * 8u, vo = (unsigned)ij * 8u, vm = vo - (unsigned)s * 8u;
  auto lev = [&](int k) { return (unsigned)(min(max(k, 1), N) - 1) * lv; };   // rho level k (clamped)
  double* Uall = dir == 0 ? F.u : F.v;
  const int nthr = (int)(blockDim.x * blockDim.y * blockDim.z);
  const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  double* const Sb = roms_smem + tid;                        // row q-1: cf_stp*u(nstp) + cf_bak*u(indx)
  double* const Su = roms_smem + (long)(KR - 1) * nthr + tid;  // row q-1: Hz*u(nstp), the new u(indx)
  const BufF64 Uix(Uall + (long)(indx - 1) * b.n3), Unew(Uall + (long)(nnew - 1) * b.n3), Hf(F.c2);
  double hf[KR + 1], hfm[KR + 1];   // Hz_fwd(c0-1+q) of the column and of its (i-1) / (j-1) neighbour
  auto load_hf = [&] {
#pragma unroll
    for (int q = 0; q < KR + 1; q++) {
      const unsigned L = lev(c0 - 1 + q);
      hf[q] = LD(Hf, vo, L);
      hfm[q] = LD(Hf, vm, L);
    }
  };
  if constexpr (PF) load_hf();
  double fl[KR];
  uv_spline_segb<KR, kU>(d, sg, X, ij, nrhs, dir, fl, [&](int q, unsigned L, double h0, double h1, double u) {
    if (q >= 1 && q < KR) {   // cells c0..c0+KR-2 (q is a constant of the unrolled load loop)
      Sb[(q - 1) * nthr] = c.cf_stp * u + c.cf_bak * LD(Uix, vo, L);
      Su[(q - 1) * nthr] = 0.5 * (h0 + h1) * u;
    }
  });
  __builtin_amdgcn_sched_barrier(0);   // the viscosity phase's loads stay out of the spline phase
  const BufF64 rr(dir == 0 ? F.ru : F.rv), Akv(F.Akv), Wi(F.Wi), Hb(F.c3);
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  const double DC0 = c.dtau * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  auto rhs = [&](int p) {
    const int k = c0 + p;
    const unsigned o = lev(k);
    const double rro = LD(rr, vo, o);
    const double r = k == 1 ? rro - fl[1] : rro - fl[p + 1 < KR ? p + 1 : KR - 1] + fl[p];
    const double ub = Sb[(p < KR - 1 ? p : KR - 2) * nthr];
    const double v = 0.5 * (LD(Hb, vo, o) + LD(Hb, vm, o)) * ub + DC0 * r;
    return k == N ? v + c.dtau * sstr : v;
  };
  if constexpr (!PF) load_hf();
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q (0 at the bottom and the surface)
    const int r = c0 - 1 + q;
    const unsigned w = (unsigned)min(max(r, 1), N - 1) * lv;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * c.dtau * (LD(Akv, vo, w) + LD(Akv, vm, w)), hf[qa] + hfm[qa] + hf[q] + hfm[q]);
    const double wv = DC0 * 0.5 * (LD(Wi, vo, w) + LD(Wi, vm, w));
    fc = in ? f : 0.0;
    wc = in ? wv : 0.0;
  };
  const double rd = F.r_D[ij], rdm = F.r_D[ij - s];
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
    const double b1 = 0.5 * (hf[p + 1] + hfm[p + 1]) + 0.5 * c.dtau * (rd + rdm) + fcu + fmax0(wcu);
    const double bk = 0.5 * (hf[p + 1] + hfm[p + 1]) + fcl - fmin0(wcl) + fcu + fmax0(wcu);
    bb = k == 1 ? b1 : bk;
    dd = rhs(p);
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  const unsigned vs = act ? vo : kBufOff;
#pragma unroll
  for (int p = 0; p < KR; p++)
    if (p < n) {
      const unsigned o = lev(c0 + p);
      ST(Unew, T.D[p], vs, o);
      ST(Uix, Su[(p < KR - 1 ? p : KR - 2) * nthr], vs, o);
    }
}

static size_t pre_uv_seg_lds_bytes(unsigned nthr) {
  return (size_t)2 * kSegRows * nthr * sizeof(double);
}
void setup_pre_uv_seg() {
  (void)hipFuncSetAttribute((const void*)k_pre_uv_seg<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pre_uv_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_pre_uv_segb<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pre_uv_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_pre_uv_segb<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pre_uv_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_pre_uv_segb<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pre_uv_seg_lds_bytes(kSegBlock * kSegJMax));
  (void)hipFuncSetAttribute((const void*)k_pre_uv_segb<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pre_uv_seg_lds_bytes(kSegBlock * kSegJMax));
}

void setup_column_kernels_t(size_t bytes);
void setup_column_kernels_uv1(size_t bytes);
bool setup_column_kernels(int N) {
  const size_t bytes = col_lds_bytes(2, N);
  if (bytes > 160 * 1024) return false;
  if (bytes > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)k_pre_tracer_v<ColLds>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    (void)hipFuncSetAttribute((const void*)k_pre_uv<ColLds>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    setup_column_kernels_t(bytes);
    setup_column_kernels_uv1(bytes);
  }
  return true;
}

double pre_step3d_dtau(const Dev& d, const Tlev& t) {
  const double AM3_crv = 1.0 / 6.0;
  return t.iic == t.forw_start ? 0.5 * d.p.dt : d.p.dt * (1.0 - AM3_crv);
}

void launch_pre_step3d(const Dev& d, hipStream_t s, const Tlev& t, bool uv_done, bool hb_done, const Side* side) {
  const Bounds& b = d.b;
  PreCoef c;
  const double AM3_crv = 1.0 / 6.0;
  if (t.iic == t.forw_start) { c.dtau = 0.5 * d.p.dt; c.cf_stp = 1.0; c.cf_bak = 0.0; }
  else { c.dtau = d.p.dt * (1.0 - AM3_crv); c.cf_stp = 0.5 + AM3_crv; c.cf_bak = 0.5 - AM3_crv; }
  c.dtau = pre_step3d_dtau(d, t);   // (the same value; omega's Hz_bak/fwd use it too)
  // hb_done only with the hoisted tracer kernel (k_pre_tracer_h forms everything)
  hb_done = hb_done && d.p.hoist && b.NT <= 2;
  Range RI{b.istr, b.iend, b.jstr, b.jend};
  Range RH{b.istr - 1, b.iend, b.jstr - 1, b.jend};
  // horizontal part on rows rh (the ring i = istr-1, j = jstr-1 included):
  // the rows strips cover (k_tracer_strip.hip), the rest on tiles
  auto horiz_tiles = [&](const Range& rh) {
    if (d.p.hoist && d.p.h_jc > 0 && (b.NT == 1 || b.NT == 2)) {
      const dim3 g = grid3_jc(rh, b.N, d.p.h_jc), bs(kBX, kBY);
      const int jc = d.p.h_jc;
      if (b.NT == 2 && hb_done)
        hipLaunchKernelGGL((k_pre_tracer_hj<2, true>), g, bs, 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs, jc);
      else if (b.NT == 2)
        hipLaunchKernelGGL((k_pre_tracer_hj<2, false>), g, bs, 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs, jc);
      else if (hb_done)
        hipLaunchKernelGGL((k_pre_tracer_hj<1, true>), g, bs, 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs, jc);
      else
        hipLaunchKernelGGL((k_pre_tracer_hj<1, false>), g, bs, 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs, jc);
    } else if (d.p.hoist && b.NT == 2 && d.p.h_ty == 8) {
      if (hb_done)
        hipLaunchKernelGGL((k_pre_tracer_h1<2, 8, true>), grid3_ty(rh, b.N, 8), dim3(kBX, 8), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
      else
        hipLaunchKernelGGL((k_pre_tracer_h1<2, 8, false>), grid3_ty(rh, b.N, 8), dim3(kBX, 8), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
    } else if (d.p.hoist && b.NT == 2) {
      if (hb_done)
        hipLaunchKernelGGL((k_pre_tracer_h1<2, 4, true>), grid3_ty(rh, b.N, 4), dim3(kBX, 4), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
      else
        hipLaunchKernelGGL((k_pre_tracer_h1<2, 4, false>), grid3_ty(rh, b.N, 4), dim3(kBX, 4), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
    } else if (d.p.hoist && b.NT == 1) {
      if (hb_done)
        hipLaunchKernelGGL((k_pre_tracer_h1<1, 4, true>), grid3_ty(rh, b.N, 4), dim3(kBX, 4), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
      else
        hipLaunchKernelGGL((k_pre_tracer_h1<1, 4, false>), grid3_ty(rh, b.N, 4), dim3(kBX, 4), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
    } else {
      hipLaunchKernelGGL(k_pre_tracer_h, grid3_of(rh, b.N), dim3(kBX, kBY), 0, s, d, rh, c, t.nstp, t.nnew, t.nrhs);
    }
  };
  auto horiz = [&](const Range& rh) {
    int jA = 0, jB = -1;
    if (d.p.hoist && d.p.h_jc == 0 &&
        launch_tracer_strip(d, s, rh, 1, false, hb_done, t.nnew, t.nrhs, c.dtau, c.cf_stp, c.cf_bak, t.nstp, jA, jB)) {
      if (jA > rh.j0) horiz_tiles(Range{rh.i0, rh.i1, rh.j0, jA - 1});
      if (jB < rh.j1) horiz_tiles(Range{rh.i0, rh.i1, jB + 1, rh.j1});
    } else {
      horiz_tiles(rh);
    }
  };
  // column solves on rows ri
  auto cols = [&](const Range& ri, hipStream_t st) {
    dim3 gt = gridc_of(ri);
    gt.z = b.NT;
    if (d.p.colseg && (d.p.seg_buf & 1) && (d.p.seg_buf & 16))
      hipLaunchKernelGGL(k_pre_tracer_segb<true>, seg_grid_of(ri, b.NT), dim3(kCX, seg_waves(b.N)), 0, st, d, ri, c,
                         t.nnew, t.nrhs);
    else if (d.p.colseg && (d.p.seg_buf & 1) && (d.p.seg_buf & 1024))
      hipLaunchKernelGGL((k_pre_tracer_segb<false, false>), seg_grid_of(ri, b.NT), dim3(kCX, seg_waves(b.N)), 0, st, d, ri,
                         c, t.nnew, t.nrhs);
    else if (d.p.colseg && (d.p.seg_buf & 1))
      hipLaunchKernelGGL(k_pre_tracer_segb<false>, seg_grid_of(ri, b.NT), dim3(kCX, seg_waves(b.N)), 0, st, d, ri, c,
                         t.nnew, t.nrhs);
    else if (d.p.colseg)
      hipLaunchKernelGGL(k_pre_tracer_seg, seg_grid_of(ri, b.NT), dim3(kCX, seg_waves(b.N)), 0, st, d, ri, c, t.nnew,
                         t.nrhs);
    else if ((d.p.colreg & 2) && b.N == 50 && !d.f.colscr)
      hipLaunchKernelGGL(k_pre_tracer_v_reg<50>, gt, dim3(kCX), col_lds_bytes(1, 50), st, d, ri, c, t.nnew, t.nrhs);
    else if (d.f.colscr)
      hipLaunchKernelGGL(k_pre_tracer_v<ColGlb>, gt, dim3(kCX), 0, st, d, ri, c, t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL(k_pre_tracer_v<ColLds>, gt, dim3(kCX), col_lds_bytes(2, b.N), st, d, ri, c, t.nnew, t.nrhs);
  };
  // Params::t_chunk: horizontal part and column solves alternate over strips
  // of t_chunk rows, so each strip's t(nnew) -- the horizontal result the
  // solver reads back -- is still in the Infinity Cache when it is read
  if (d.p.t_chunk > 0 && !side && d.p.colseg) {
    for (int ja = b.jstr; ja <= b.jend; ja += d.p.t_chunk) {
      const int jb = min(ja + d.p.t_chunk - 1, b.jend);
      horiz(Range{b.istr - 1, b.iend, ja == b.jstr ? b.jstr - 1 : ja, jb});
      cols(Range{b.istr, b.iend, ja, jb}, s);
    }
  } else {
    horiz(RH);
    // The tracer column solves (t(nnew), reading Hz_fwd) and the momentum ones
    // (u, v(nnew), u, v(indx), reading Hz_fwd/bak, ru, rv) share no output:
    // with a side stream they run side by side once the horizontal tracer
    // kernel has formed the ring of Hz_fwd/bak both read
    hipStream_t st = s;
    if (side) {
      (void)hipEventRecord(side->efork, s);
      (void)hipStreamWaitEvent(side->s2, side->efork, 0);
      st = side->s2;
    }
    cols(RI, st);
  }
  hipStream_t st = side ? side->s2 : s;
  for (int itrc = 1; itrc <= b.NT && side; itrc++) launch_t3dbc(d, st, t, itrc);
  if (side) launch_exchange_tracers(d, st, t.nnew);
  if (!uv_done) launch_uv_horiz(d, s, t.nrhs, 0);
  Range Rd{b.istrU - 1, b.iend, b.jstrV - 1, b.jend};
  hipLaunchKernelGGL(k_rd, grid_of(Rd), dim3(kBX, kBY), 0, s, d, Rd, t.nstp);
  dim3 gu = gridc_of(RI);
  gu.z = 2;
  if (d.p.colseg) {
    const dim3 gs = seg_uv_grid(d, RI, d.p.seg_jrows), bs(kCX, seg_waves(b.N), d.p.seg_jrows);
    ktimer_mark(s, kTimedPreUvSeg, 0);
    if (d.p.preuv_lds && d.p.uv_adv && t.nrhs == t.nstp && (d.p.seg_buf & 128) && (d.p.seg_buf & 256) &&
        !(d.p.seg_buf & 512))
      hipLaunchKernelGGL(k_pre_uv_segb<true>, gs, bs, pre_uv_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, RI, c, t.nstp,
                         t.nnew, t.nrhs);
    else if (d.p.preuv_lds && d.p.uv_adv && t.nrhs == t.nstp && (d.p.seg_buf & 128) && (d.p.seg_buf & 512) &&
             (d.p.seg_buf & 256))
      hipLaunchKernelGGL((k_pre_uv_segb<true, false>), gs, bs, pre_uv_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, RI, c,
                         t.nstp, t.nnew, t.nrhs);
    else if (d.p.preuv_lds && d.p.uv_adv && t.nrhs == t.nstp && (d.p.seg_buf & 128) && (d.p.seg_buf & 512))
      hipLaunchKernelGGL((k_pre_uv_segb<false, false>), gs, bs, pre_uv_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, RI, c,
                         t.nstp, t.nnew, t.nrhs);
    else if (d.p.preuv_lds && d.p.uv_adv && t.nrhs == t.nstp && (d.p.seg_buf & 128))
      hipLaunchKernelGGL(k_pre_uv_segb<false>, gs, bs, pre_uv_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, RI, c, t.nstp, t.nnew,
                         t.nrhs);
    else if (d.p.preuv_lds && d.p.uv_adv && t.nrhs == t.nstp)
      hipLaunchKernelGGL(k_pre_uv_seg<true>, gs, bs, pre_uv_seg_lds_bytes(bs.x * bs.y * bs.z), s, d, RI, c, t.nstp,
                         t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL(k_pre_uv_seg<false>, gs, bs, 0, s, d, RI, c, t.nstp, t.nnew, t.nrhs);
    ktimer_mark(s, kTimedPreUvSeg, 1, 1);
  }
  else if (d.f.colscr)
    hipLaunchKernelGGL(k_pre_uv<ColGlb>, gu, dim3(kCX), 0, s, d, RI, c, t.nstp, t.nnew, t.nrhs);
  else
    hipLaunchKernelGGL(k_pre_uv<ColLds>, gu, dim3(kCX), col_lds_bytes(2, b.N), s, d, RI, c, t.nstp, t.nnew, t.nrhs);
  launch_river_uv(d, s, t.nnew, 1);   // pre_step3d4S.F:493-522
  launch_u3dbc(d, s, t);
  launch_v3dbc(d, s, t);
  if (side) {
    (void)hipEventRecord(side->ejoin, st);
    (void)hipStreamWaitEvent(s, side->ejoin, 0);
    return;
  }
  for (int itrc = 1; itrc <= b.NT; itrc++) launch_t3dbc(d, s, t, itrc);
  launch_exchange_tracers(d, s, t.nnew);
}

}  // namespace roms
