// k_step3d_t.hip -- tracer corrector step3d_t_iso_tile (step3d_t_ISO.F:45-1178,
// non-isoneutral branch: UPSTREAM_TS + SPLINE_TS) and the Laplacian tracer
// diffusion t3dmix_tile (t3dmix_S.F).  One lane per water column; all levels
// and the tridiagonal solve stay in the lane.
#include "k_colseg.h"

namespace roms {

// Horizontal advection, one thread per (i,j,k) cell, all tracers.
// up: UPSTREAM_TS; ADV_ISONEUTRAL builds without it (step3d_t_ISO.F:4-6)
__global__ void __launch_bounds__(256) k_step3d_t_h(Dev d, Range R, int nnew, int nrhs, int up) {
  const uint3 bI = xcd_tile();
  __shared__ TracerWin W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2;
  tracer_win_fill(b, F, W, ib, jb, kk, nullptr);
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, i, j), o = ij + kk;
  const AccTL a{W.T, W.UM, W.VM, W.FU, W.FV, ib, jb};
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    const long tb = (long)(itrc - 1) * 3 * b.n3;
    const double* Tr = F.t + (long)(nrhs - 1) * b.n3 + tb;
    __syncthreads();
    tracer_win_fill(b, F, W, ib, jb, kk, Tr);
    __syncthreads();
    if (!act) continue;
    double* Tn = F.t + (long)(nnew - 1) * b.n3 + tb;
    double FX0 = tracer_fx(b, a, i, j, up), FX1 = tracer_fx(b, a, i + 1, j, up);
    double FE0 = tracer_fe(b, a, i, j, up), FE1 = tracer_fe(b, a, i, j + 1, up);
    if (d.p.nriv > 0) {   // river inflow faces (compute_horiz_tracer_fluxes.h:217-246)
      river_tracer_flux(d, 0, i, j, k, itrc, FX0); river_tracer_flux(d, 0, i + 1, j, k, itrc, FX1);
      river_tracer_flux(d, 1, i, j, k, itrc, FE0); river_tracer_flux(d, 1, i, j + 1, k, itrc, FE1);
    }
    Tn[o] = Tn[o] - d.p.dt * F.pm[ij] * F.pn[ij] * (FX1 - FX0 + FE1 - FE0);
  }
}

// The same for NTT <= 2 tracers with every global load issued at entry (see
// k_pre_tracer_h1): one memory wait per block.  Bit-identical.
template <int NTT, int TY>
struct TracerWinS {
  static constexpr int kN = kUVW * (TY + 4);
  double UM[kN], VM[kN], FU[kN], FV[kN], T[NTT][kN];
};
template <int NTT, int TY>
__global__ void __launch_bounds__(kBX * TY) k_step3d_t_h1(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = h_tile(d.p.tile_grp);
  __shared__ TracerWinS<NTT, TY> W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * TY;
  const int ib = i0 - 2, jb = j0 - 2;
  const long kk = (long)(k - 1) * b.n2;
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
  const long ij = act ? IJ(b, i, j) : IJ(b, R.i0, R.j0), o = ij + kk;
  const double pm = F.pm[ij], pn = F.pn[ij];
  double tn[NTT];
#pragma unroll
  for (int t = 0; t < NTT; t++) tn[t] = F.t[(long)(nnew - 1) * b.n3 + (long)t * 3 * b.n3 + o];
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
#pragma unroll
  for (int t = 0; t < NTT; t++) {
    const int itrc = t + 1;
    const AccTL a{W.T[t], W.UM, W.VM, W.FU, W.FV, ib, jb};
    double FX0 = tracer_fx(b, a, i, j, true), FX1 = tracer_fx(b, a, i + 1, j, true);
    double FE0 = tracer_fe(b, a, i, j, true), FE1 = tracer_fe(b, a, i, j + 1, true);
    if (d.p.nriv > 0) {   // river inflow faces (compute_horiz_tracer_fluxes.h:217-246)
      river_tracer_flux(d, 0, i, j, k, itrc, FX0); river_tracer_flux(d, 0, i + 1, j, k, itrc, FX1);
      river_tracer_flux(d, 1, i, j, k, itrc, FE0); river_tracer_flux(d, 1, i, j + 1, k, itrc, FE1);
    }
    F.t[(long)(nnew - 1) * b.n3 + (long)t * 3 * b.n3 + o] = tn[t] - d.p.dt * pm * pn * (FX1 - FX0 + FE1 - FE0);
  }
}

// Vertical part per column: spline advection on t(nrhs), surface fluxes
// (+ KPP non-local and solar terms), implicit diffusion.  LDS slots: A holds
// FC (spline) then DC(k) at A[k-1]; B holds the spline CF then Thomas CF.
// ISO: ADV_ISONEUTRAL's STABILIZE diffusivity Akz joins Akt (step3d_t_ISO.F:1049-1065)
template <class C, bool ISO = false>
__global__ void __launch_bounds__(64) k_step3d_t_v(Dev d, Range R, int nnew, int nrhs) {
  ROMS_IJC_OR_RETURN(R)
  col_lds_poison<C>(2, d.b.N);
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const double dt = P.dt;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const double rm = F.rmask[ij];
  const double* __restrict__ Hz = F.Hz + ij;
  const C A = ColMake<C>::at(d, 0, (int)bI.z, ij), B = ColMake<C>::at(d, 1, (int)bI.z, ij);
  {
    const int itrc = 1 + (int)bI.z;
    const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3 + ij;
    double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3 + ij;
    const double stf = F.stflx[ij + (long)(itrc - 1) * n2];
    // spline interface values FC(0:N) (compute_vert_tracer_fluxes.h)
    tracer_spline_lds(N, n2, Hz, Tr, F.We + ij, A, B);
    A[N] = 0.0;
    A[0] = 0.0;
    // advective update + surface/KPP terms fused into the Thomas elimination
    const int iAkt = itrc < b.nTS ? itrc : b.nTS;
    const double* __restrict__ Akt0 = F.Akt + (long)(iAkt - 1) * b.n3w + ij;
    const double* __restrict__ Akz = ISO ? F.Akz + ij : nullptr;
    struct AktAkz {   // Akt(k) [+ Akz(k)]
      const double *a, *z;
      __device__ double operator[](long w) const { return ISO ? a[w] + z[w] : a[w]; }
    } const Akt{Akt0, Akz};
    const double* __restrict__ Wi = F.Wi + ij;
    const double DC0 = dt * F.pm[ij] * F.pn[ij];
    const bool kppT = P.lmd && itrc == 1, kppS = P.lmd_nonlocal && itrc == 2 && P.salinity;
  auto gh = [&](long o) { return P.lmd_nonlocal ? F.ghat[ij + o] : 0.0; };
    const double sr = F.srflx[ij];
    // pipe_frc.F sources (step3d_t_ISO.F:927-934)
    const int pidx = P.npip > 0 ? F.pipe_idx[ij] : 0;
    const double pflx = pidx > 0 ? F.pipe_flx[ij] : 0.0;
    const double ptrc = pidx > 0 ? F.pipe_trc[(pidx - 1) + (itrc - 1) * P.npip] : 0.0;
    auto tval_of = [&](int k, double tnk) {
      const long o = (long)(k - 1) * n2;
      double t = tnk - dt * F.pm[ij] * F.pn[ij] * (A[k] - A[k - 1]);
      if (pidx > 0) t = t + dt * F.pm[ij] * F.pn[ij] * pflx * F.pipe_prf[(pidx - 1) + (k - 1) * P.npip] * ptrc;
      if (k == N) {
        // heat of rain: 2 m air temperature under BULK_FRC, else the water's (step3d_t_ISO.F:939-951)
        if (itrc == 1) t = t + dt * F.swflx[ij] * (P.bulk_frc ? F.tair[ij] : t / Hz[o]);
        t = t + dt * stf;
      }
      if (kppT) {
        // without LMD_NONLOCAL the ghat term is absent: gh() = 0 leaves sr*swr_frac exact
        if (k <= N - 1) t = t + dt * (sr * F.swr_frac[ij + (long)k * n2] - gh((long)k * n2) * (stf - sr));
        if (k >= 2) t = t - dt * (sr * F.swr_frac[ij + o] - gh(o) * (stf - sr));
      } else if (kppS) {
        if (k <= N - 1) t = t + (-dt * F.ghat[ij + (long)k * n2] * stf);
        if (k >= 2) t = t - (-dt * F.ghat[ij + o] * stf);
      }
      return t;
    };
    auto tval = [&](int k) { return tval_of(k, Tn[(long)(k - 1) * n2]); };
    double FCk = 2.0 * dt * Akt[n2] / (Hz[0] + Hz[n2]);
    double WCk = DC0 * Wi[n2];
    double cff = 1.0 / (Hz[0] + FCk + fmax0(WCk));
    double CFk = cff * (FCk - fmin0(WCk));
    double DCk = cff * tval(1);
    B[1] = CFk;
    A[0] = DCk;
    {
      double hzk = Hz[n2];  // Hz of rho level k (starts at k=2)
      auto thomas = [&](int k, double akt, double hz1, double wi, double tn) {
        const double hz0 = hzk;
        const double FCn = 2.0 * dt * akt / (hz0 + hz1);
        const double WCn = wi * DC0;
        cff = 1.0 / (hz0 + FCn + fmax0(WCn) + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
        const double CFn = cff * (FCn - fmin0(WCn));
        const double DCn = cff * (tval_of(k, tn) + DCk * (FCk + fmax0(WCk)));
        B[k] = CFn;
        A[k - 1] = DCn;
        FCk = FCn; WCk = WCn; CFk = CFn; DCk = DCn;
        hzk = hz1;
      };
      double ra[kPF], rhz[kPF], rwi[kPF], rtn[kPF];   // Akt(k), Hz(k+1), Wi(k), Tn(k) of level k
#pragma unroll
      for (int q = 0; q < kPF; q++) {
        const int k = min(2 + q, N - 1);
        ra[q] = Akt[(long)k * n2]; rhz[q] = Hz[(long)k * n2]; rwi[q] = Wi[(long)k * n2];
        rtn[q] = Tn[(long)(k - 1) * n2];
      }
      int k2 = 2;
      for (; k2 + kPF - 1 <= N - 1; k2 += kPF) {
#pragma unroll
        for (int q = 0; q < kPF; q++) {
          const double akt = ra[q], hz1 = rhz[q], wi = rwi[q], tn = rtn[q];
          const int kn = min(k2 + q + kPF, N - 1);
          ra[q] = Akt[(long)kn * n2]; rhz[q] = Hz[(long)kn * n2]; rwi[q] = Wi[(long)kn * n2];
          rtn[q] = Tn[(long)(kn - 1) * n2];
          thomas(k2 + q, akt, hz1, wi, tn);
        }
      }
      for (int k = k2; k <= N - 1; k++)
        thomas(k, Akt[(long)k * n2], Hz[(long)k * n2], Wi[(long)k * n2], Tn[(long)(k - 1) * n2]);
    }
    const long oN = (long)(N - 1) * n2;
    double tt = (tval(N) + DCk * (FCk + fmax0(WCk))) / (Hz[oN] + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk))) * rm;
    Tn[oN] = tt;
#pragma unroll 8
    for (int k = N - 1; k >= 1; k--) {
      tt = (A[k - 1] + B[k] * tt) * rm;
      Tn[(long)(k - 1) * n2] = tt;
    }
  }
}

// ---- segment-partitioned variant of k_step3d_t_v (k_colseg.h): block =
// 64 columns x S segment wavefronts, one tracer per grid z.  The spline
// interface values FC(0:N) and the implicit diffusion are each solved as one
// partitioned tridiagonal system; the surface, KPP and pipe terms of the
// diffusion r.h.s. are those of k_step3d_t_v (step3d_t_ISO.F:913-1100). ----
__global__ void __launch_bounds__(kSegBlock, 2) k_step3d_t_seg(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const double dt = P.dt;
  const SegSpan sg = seg_span(N);
  const int iu = tile_i0(R.i0) + (int)bI.x * kSegCW + sg.col;
  const bool act = iu >= R.i0 && iu <= R.i1;
  const int i = act ? iu : (iu < R.i0 ? R.i0 : R.i1), j = R.j0 + (int)bI.y;
  const int itrc = 1 + (int)bI.z;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const int c0 = sg.c0, n = sg.n;
  const bool last = sg.s == sg.S - 1;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3 + ij;
  double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3 + ij;
  const double* __restrict__ We = F.We + ij;
  auto cell = [&](int k) { return (long)(min(max(k, 1), N) - 1) * n2; };   // rho level k (clamped)
  // hz[q] = Hz(c0-1+q), q = 0..KR; tt[q] = t(nrhs)(c0-1+q), q = 0..KR-1 (clamped to 1..N)
  double hz[KR + 1], tt[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {
    hz[q] = Hz[cell(c0 - 1 + q)];
    if (q < KR) tt[q] = Tr[cell(c0 - 1 + q)];
  }
  // spline interface values FC(c0-1+q) and the advective fluxes FC*We (into tt)
  {
    double fc[KR];
    spline_fc_seg<KR>(sg, N, X, hz, tt, fc);
    double we[KR];   // every row's We issued as one batch (pin, k_colseg.h)
#pragma unroll
    for (int q = 0; q < KR; q++) we[q] = We[(long)min(max(c0 - 1 + q, 1), N - 1) * n2];
#pragma unroll
    for (int q = 0; q < KR; q++) pin(we[q]);
#pragma unroll
    for (int q = 0; q < KR; q++) {
      const int r = c0 - 1 + q;
      tt[q] = (r == 0 || r == N) ? 0.0 : fc[q] * we[q];
    }
  }
  // implicit diffusion rows, cells k = c0+p, p = 0..n-1.  The scheduling
  // barrier keeps this phase's loads out of the spline phase (hoisted there
  // they pushed the kernel to 281 VGPRs, one wave per SIMD)
  __builtin_amdgcn_sched_barrier(0);
  const int iAkt = itrc < b.nTS ? itrc : b.nTS;
  const double* __restrict__ Akt = F.Akt + (long)(iAkt - 1) * b.n3w + ij;
  const double* __restrict__ Wi = F.Wi + ij;
  const double DC0 = dt * F.pm[ij] * F.pn[ij];
  const bool kppT = P.lmd && itrc == 1, kppS = P.lmd_nonlocal && itrc == 2 && P.salinity;
  const double sr = F.srflx[ij];
  const double stf = F.stflx[ij + (long)(itrc - 1) * n2];
  // right-hand sides (step3d_t_ISO.F:922-1040): flux divergence, pipes, rain
  // heat, surface flux, KPP solar / non-local terms, in the reference's order
  double rhs[KR];
#pragma unroll
  for (int p = 0; p < KR; p++) rhs[p] = Tn[cell(c0 + p)] - dt * F.pm[ij] * F.pn[ij] * (tt[p + 1 < KR ? p + 1 : KR - 1] - tt[p]);
  if (P.npip > 0) {   // pipe_frc.F sources (step3d_t_ISO.F:927-934)
    const int pidx = F.pipe_idx[ij];
    if (pidx > 0) {
      const double pflx = F.pipe_flx[ij], ptrc = F.pipe_trc[(pidx - 1) + (itrc - 1) * P.npip];
#pragma unroll
      for (int p = 0; p < KR; p++) {
        const int k = min(c0 + p, N);
        rhs[p] = rhs[p] + dt * F.pm[ij] * F.pn[ij] * pflx * F.pipe_prf[(pidx - 1) + (k - 1) * P.npip] * ptrc;
      }
    }
  }
  {
    // the surface cell k = N (row n-1 of the last segment): heat of rain --
    // the 2 m air temperature under BULK_FRC, else the water's own -- and the
    // surface flux (step3d_t_ISO.F:939-959); picked out and put back by selects
    const bool top = last;
    double t = 0.0;
#pragma unroll
    for (int p = 0; p < KR; p++) t = p == n - 1 ? rhs[p] : t;
    const double swf = F.swflx[ij], hzN = Hz[cell(N)];
    if (itrc == 1) t = t + dt * swf * (P.bulk_frc ? F.tair[ij] : t / hzN);
    t = t + dt * stf;
#pragma unroll
    for (int p = 0; p < KR; p++) rhs[p] = (top && p == n - 1) ? t : rhs[p];
  }
  if (kppT || kppS) {
    auto gh = [&](long o) { return P.lmd_nonlocal ? F.ghat[ij + o] : 0.0; };
#pragma unroll
    for (int p = 0; p < KR; p++) {
      const int k = min(c0 + p, N);
      const long ou = (long)min(k, N - 1) * n2, ol = (long)max(k - 1, 1) * n2;   // w-levels k and k-1
      double t = rhs[p];
      if (kppT) {
        const double up = dt * (sr * F.swr_frac[ij + ou] - gh(ou) * (stf - sr));
        const double lo = dt * (sr * F.swr_frac[ij + ol] - gh(ol) * (stf - sr));
        t = k <= N - 1 ? t + up : t;
        t = k >= 2 ? t - lo : t;
      } else {
        const double up = -dt * F.ghat[ij + ou] * stf, lo = -dt * F.ghat[ij + ol] * stf;
        t = k <= N - 1 ? t + up : t;
        t = k >= 2 ? t - lo : t;
      }
      rhs[p] = t;
    }
  }
  // FC, WC at interface r (0 at the bottom and the surface)
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q
    const int r = c0 - 1 + q;
    const long w = (long)min(max(r, 1), N - 1) * n2;
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * dt * Akt[w], hz[q] + hz[qa]);
    const double c = DC0 * Wi[w];
    fc = in ? f : 0.0;
    wc = in ? c : 0.0;
  };
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.eliminate(n, [&](int p, double& a, double& bb, double& c, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    a = -(fcl + fmax0(wcl));
    bb = hz[p + 1] + fcu + fmax0(wcu) + fcl - fmin0(wcl);
    c = -(fcu - fmin0(wcu));
    dd = rhs[p];
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  if (act) {
    const double rm = F.rmask[ij];
#pragma unroll
    for (int p = 0; p < KR; p++)
      if (p < n) Tn[cell(c0 + p)] = T.D[p] * rm;
  }
}

// ---- k_step3d_t_seg with buffer loads/stores (Params::seg_buf): a wave is
// one segment, so its first cell c0 and row count n are wave-uniform
// (readfirstlane); every level offset is then one SGPR shared by all fields
// (soffset), the lane's column one VGPR (voffset), and no load carries a
// 64-bit per-row address.  Same expressions in the same order: bitwise equal
// to k_step3d_t_seg. ----
#ifndef ROMS_SEG_T_GROUP
#define ROMS_SEG_T_GROUP kSegLoadGroup
#endif
// PF: t(nnew) of the segment's rows (the diffusion r.h.s.) loaded at entry
// with the spline phase's inputs, so they land during its solve.  RL: Hz
// reloaded for the diffusion phase instead of kept live across the spline
// solve (30 VGPRs at its register peak).
template <bool PF, bool RL = false, bool UNI = true>
__global__ void __launch_bounds__(kSegBlock, ROMS_T_SEG_WAVES) k_step3d_t_segb(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = seg_tile(d.p.seg_order, d.p.seg_xg);
  __shared__ SegXchg X;
  constexpr int KR = kSegRows + 1;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const double dt = P.dt;
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
  const bool last = sg.s == sg.S - 1;
  const unsigned vo = (unsigned)ij * 8u;
  // byte offset of rho level k (clamped to 1..N) / w level r (clamped to lo..hi)
  auto lev = [&](int k) { return (unsigned)(min(max(k, 1), N) - 1) * (unsigned)n2 * 8u; };
  auto wlev = [&](int r, int lo, int hi) { return (unsigned)min(max(r, lo), hi) * (unsigned)n2 * 8u; };
  const BufF64 Hz(F.Hz), We(F.We), Wi(F.Wi);
  const BufF64 Tr(F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3);
  const BufF64 Tn(F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3);
  double hz[KR + 1], tt[KR], tn[KR];
#pragma unroll
  for (int q = 0; q < KR + 1; q++) {
    hz[q] = LD(Hz, vo, lev(c0 - 1 + q));
    if (q < KR) tt[q] = LD(Tr, vo, lev(c0 - 1 + q));
  }
  if constexpr (PF) {
#pragma unroll
    for (int p = 0; p < KR; p++) tn[p] = LD(Tn, vo, lev(c0 + p));
  }
  {
    double fc[KR];
    spline_fc_seg<KR>(sg, N, X, hz, tt, fc);
    double we[KR];
#pragma unroll
    for (int q = 0; q < KR; q++) we[q] = LD(We, vo, wlev(c0 - 1 + q, 1, N - 1));
#pragma unroll
    for (int q = 0; q < KR; q++) pin(we[q]);
#pragma unroll
    for (int q = 0; q < KR; q++) {
      const int r = c0 - 1 + q;
      tt[q] = (r == 0 || r == N) ? 0.0 : fc[q] * we[q];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (RL) {
#pragma unroll
    for (int q = 0; q < KR + 1; q++) hz[q] = LD(Hz, vo, lev(c0 - 1 + q));
  }
  const int iAkt = itrc < b.nTS ? itrc : b.nTS;
  const BufF64 Akt(F.Akt + (long)(iAkt - 1) * b.n3w);
  const BufF64 Pm(F.pm), Pn(F.pn);
  const double pm = Pm.ld(vo, 0), pn = Pn.ld(vo, 0);
  const double DC0 = dt * pm * pn;
  const bool kppT = P.lmd && itrc == 1, kppS = P.lmd_nonlocal && itrc == 2 && P.salinity;
  const double sr = BufF64(F.srflx).ld(vo, 0);
  const double stf = BufF64(F.stflx).ld(vo, (unsigned)(itrc - 1) * (unsigned)n2 * 8u);
  // right-hand sides (step3d_t_ISO.F:922-1040): flux divergence, pipes, rain
  // heat, surface flux, KPP solar / non-local terms, in the reference's order;
  // every row's loads issued before the elimination
  double rhs[KR];
#pragma unroll
  for (int p = 0; p < KR; p++)
    rhs[p] = (PF ? tn[p] : LD(Tn, vo, lev(c0 + p))) - dt * pm * pn * (tt[p + 1 < KR ? p + 1 : KR - 1] - tt[p]);
  if (P.npip > 0) {   // pipe_frc.F sources (step3d_t_ISO.F:927-934)
    const int pidx = F.pipe_idx[ij];
    if (pidx > 0) {
      const double pflx = F.pipe_flx[ij], ptrc = F.pipe_trc[(pidx - 1) + (itrc - 1) * P.npip];
#pragma unroll
      for (int p = 0; p < KR; p++) {
        const int k = min(c0 + p, N);
        rhs[p] = rhs[p] + dt * pm * pn * pflx * F.pipe_prf[(pidx - 1) + (k - 1) * P.npip] * ptrc;
      }
    }
  }
  if (last) {   // the surface cell k = N, row n-1 of the last segment (wave-uniform)
    double t = 0.0;
#pragma unroll
    for (int p = 0; p < KR; p++) t = p == n - 1 ? rhs[p] : t;
    if (itrc == 1) {
      const double swf = BufF64(F.swflx).ld(vo, 0);
      t = t + dt * swf * (P.bulk_frc ? BufF64(F.tair).ld(vo, 0) : t / LD(Hz, vo, lev(N)));
    }
    t = t + dt * stf;
#pragma unroll
    for (int p = 0; p < KR; p++) rhs[p] = p == n - 1 ? t : rhs[p];
  }
  if (kppT || kppS) {
    // the KPP term of w level m is added to the cell below it (k = m, m <=
    // N-1) and subtracted from the cell above (k = m+1, m >= 1): one load
    // per level, each row's upper term its next row's lower one.  Every
    // level's swr_frac / ghat is loaded first, outside any data-dependent
    // branch, so the loads issue together (a load per term inside the
    // kppT / nl selects waited on a round trip per row)
    const BufF64 Sw(F.swr_frac), Gh(F.ghat);
    const bool nl = P.lmd_nonlocal;
    double swv[KR + 1], ghv[KR + 1];
    if (kppT) {
#pragma unroll
      for (int q = 0; q < KR + 1; q++) {
        const unsigned o = wlev(c0 - 1 + q, 1, N - 1);
        swv[q] = LD(Sw, vo, o);
        ghv[q] = LD(Gh, vo, o);
      }
    } else {
#pragma unroll
      for (int q = 0; q < KR + 1; q++) {
        swv[q] = 0.0;
        ghv[q] = LD(Gh, vo, wlev(c0 - 1 + q, 1, N - 1));
      }
    }
    auto term = [&](int q) {   // w level c0-1+q
      return kppT ? dt * (sr * swv[q] - (nl ? ghv[q] : 0.0) * (stf - sr)) : -dt * ghv[q] * stf;
    };
    double lo = term(0);
#pragma unroll
    for (int p = 0; p < KR; p++) {
      const int k = min(c0 + p, N);
      const double up = term(p + 1);
      double t = rhs[p];
      t = k <= N - 1 ? t + up : t;
      t = k >= 2 ? t - lo : t;
      rhs[p] = t;
      lo = up;
    }
  }
  auto fcw = [&](int q, double& fc, double& wc) {   // interface c0-1+q
    const int r = c0 - 1 + q;
    const unsigned w = wlev(r, 1, N - 1);
    const bool in = r > 0 && r < N;
    const int qa = q + 1 < KR + 1 ? q + 1 : KR;
    const double f = SEG_DIV(2.0 * dt * LD(Akt, vo, w), hz[q] + hz[qa]);
    const double c = DC0 * LD(Wi, vo, w);
    fc = in ? f : 0.0;
    wc = in ? c : 0.0;
  };
  double fcl, wcl;
  fcw(0, fcl, wcl);
  __syncthreads();  // X reused by the second coupling
  SegTri<KR> T;
  T.template eliminate<ROMS_SEG_T_GROUP>(n, [&](int p, double& a, double& bb, double& c, double& dd) {
    double fcu, wcu;
    fcw(p + 1, fcu, wcu);
    a = -(fcl + fmax0(wcl));
    bb = hz[p + 1] + fcu + fmax0(wcu) + fcl - fmin0(wcl);
    c = -(fcu - fmin0(wcu));
    dd = rhs[p];
    fcl = fcu; wcl = wcu;
  });
  double xL, xR;
  T.couple(sg, n, X, xL, xR);
  T.solve(n, xL, xR);
  const double rm = BufF64(F.rmask).ld(vo, 0);
  const unsigned vs = act ? vo : kBufOff;
  // straight-line stores (rows past n take kBufOff and are dropped): with a
  // branch per row the compiler waited for every previous store before the
  // next one (vmcnt(0) at each branch join, 14 store round trips per wave)
#pragma unroll
  for (int p = 0; p < KR; p++) ST(Tn, T.D[p] * rm, p < n ? vs : kBufOff, lev(c0 + p));
}

void setup_column_kernels_t(size_t bytes) {
  (void)hipFuncSetAttribute((const void*)k_step3d_t_v<ColLds>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes);
  (void)hipFuncSetAttribute((const void*)k_step3d_t_v<ColLds, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes);
}

void launch_step3d_t(const Dev& d, hipStream_t s, const Tlev& t, bool exchange) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  if (d.p.iso) {
    // ADV_ISONEUTRAL: centred horizontal fluxes, the rotated biharmonic
    // operator per tracer, then the column part with Akt + Akz; in order,
    // no rim-first overlap
    hipLaunchKernelGGL(k_step3d_t_h, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, t.nnew, t.nrhs, 0);
    for (int itrc = 1; itrc <= b.NT; itrc++) launch_iso_tracer(d, s, t, itrc);
    dim3 gt = gridc_of(R);
    gt.z = b.NT;
    if (d.f.colscr)
      hipLaunchKernelGGL((k_step3d_t_v<ColGlb, true>), gt, dim3(kCX), 0, s, d, R, t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL((k_step3d_t_v<ColLds, true>), gt, dim3(kCX), col_lds_bytes(2, b.N), s, d, R, t.nnew, t.nrhs);
    for (int itrc = 1; itrc <= b.NT; itrc++) launch_t3dbc(d, s, t, itrc);
    launch_exchange_tracers(d, s, t.nnew);
    return;
  }
  // horizontal fluxes, then the column solves, on a sub-range of the interior
  auto h_tiles = [&](const Range& r) {
    if (d.p.hoist && b.NT == 2 && d.p.h_ty == 8)
      hipLaunchKernelGGL((k_step3d_t_h1<2, 8>), grid3_ty(r, b.N, 8), dim3(kBX, 8), 0, s, d, r, t.nnew, t.nrhs);
    else if (d.p.hoist && b.NT == 2)
      hipLaunchKernelGGL((k_step3d_t_h1<2, 4>), grid3_ty(r, b.N, 4), dim3(kBX, 4), 0, s, d, r, t.nnew, t.nrhs);
    else if (d.p.hoist && b.NT == 1)
      hipLaunchKernelGGL((k_step3d_t_h1<1, 4>), grid3_ty(r, b.N, 4), dim3(kBX, 4), 0, s, d, r, t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL(k_step3d_t_h, grid3_of(r, b.N), dim3(kBX, kBY), 0, s, d, r, t.nnew, t.nrhs, 1);
  };
  auto run = [&](const Range& r) {
    // horizontal advection: the rows strips cover (k_tracer_strip.hip), the rest on tiles
    int jA = 0, jB = -1;
    if (d.p.hoist && launch_tracer_strip(d, s, r, 0, true, false, t.nnew, t.nrhs, 0.0, 0.0, 0.0, 0, jA, jB)) {
      if (jA > r.j0) h_tiles(Range{r.i0, r.i1, r.j0, jA - 1});
      if (jB < r.j1) h_tiles(Range{r.i0, r.i1, jB + 1, r.j1});
    } else {
      h_tiles(r);
    }
    dim3 gt = gridc_of(r);
    gt.z = b.NT;
    if (d.p.colseg) {
      ktimer_mark(s, kTimedStep3dTSeg, 0);
      if ((d.p.seg_buf & 2) && (d.p.seg_buf & 8))
        hipLaunchKernelGGL((k_step3d_t_segb<false, true>), seg_grid_of(r, b.NT), dim3(kCX, seg_waves(b.N)), 0, s, d, r,
                           t.nnew, t.nrhs);
      else if ((d.p.seg_buf & 2) && (d.p.seg_buf & 4) && (d.p.seg_buf & 1024))
        hipLaunchKernelGGL((k_step3d_t_segb<true, false, false>), seg_grid_of(r, b.NT), dim3(kCX, seg_waves(b.N)), 0, s, d,
                           r, t.nnew, t.nrhs);
      else if ((d.p.seg_buf & 2) && (d.p.seg_buf & 4))
        hipLaunchKernelGGL(k_step3d_t_segb<true>, seg_grid_of(r, b.NT), dim3(kCX, seg_waves(b.N)), 0, s, d, r, t.nnew, t.nrhs);
      else if (d.p.seg_buf & 2)
        hipLaunchKernelGGL(k_step3d_t_segb<false>, seg_grid_of(r, b.NT), dim3(kCX, seg_waves(b.N)), 0, s, d, r, t.nnew, t.nrhs);
      else
        hipLaunchKernelGGL(k_step3d_t_seg, seg_grid_of(r, b.NT), dim3(kCX, seg_waves(b.N)), 0, s, d, r, t.nnew, t.nrhs);
      ktimer_mark(s, kTimedStep3dTSeg, 1, 1);
    }
    else if (d.f.colscr)
      hipLaunchKernelGGL(k_step3d_t_v<ColGlb>, gt, dim3(kCX), 0, s, d, r, t.nnew, t.nrhs);
    else
      hipLaunchKernelGGL(k_step3d_t_v<ColLds>, gt, dim3(kCX), col_lds_bytes(2, b.N), s, d, r, t.nnew, t.nrhs);
  };
  auto edges = [&] {
    for (int itrc = 1; itrc <= b.NT; itrc++) launch_t3dbc(d, s, t, itrc);
  };
  // Params::t_chunk: the horizontal part and the column solve alternate over
  // strips of t_chunk rows (see launch_pre_step3d)
  auto run_all = [&] {
    if (d.p.t_chunk > 0 && d.p.colseg) {
      for (int ja = R.j0; ja <= R.j1; ja += d.p.t_chunk) run(Range{R.i0, R.i1, ja, min(ja + d.p.t_chunk - 1, R.j1)});
    } else {
      run(R);
    }
  };
  ExchList L;
  if (!exchange) {   // t3dmix follows and exchanges t(nnew) itself
    run_all();
    edges();
  } else if (tracer_exch_list(d, t.nnew, L)) {
    launch_rim_first(d, s, R, L, run, edges);
  } else {
    run_all();
    edges();
    launch_exchange_tracers(d, s, t.nnew);
  }
}

// ---- t3dmix: Laplacian diffusion along S, t(nnew) += dt*pm*pn*div(F)/Hz.
// One lane per column walking all levels, every tracer in one launch: the
// column's 2-D metric factors are read once (t3dmix_S.F:60-259). ----
__global__ void __launch_bounds__(256) k_t3dmix(Dev d, Range R, int nnew, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), sj = b.nx2, n2 = b.n2;
  const double* __restrict__ Hz = F.Hz;
  const double pmn = d.p.dt * F.pm[ij] * F.pn[ij];
  if (b.NT == 2) {
    // both tracers in one walk over k (each level's loads of T and S in
    // flight together); per tracer the same expressions as below
    double ax0[2], ax1[2], ay0[2], ay1[2];
    const double* __restrict__ Tr[2];
    double* __restrict__ Tn[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const double* d2 = F.diff2 + (long)q * n2;
      Tr[q] = F.t + (long)(nrhs - 1) * b.n3 + (long)q * 3 * b.n3;
      Tn[q] = F.t + (long)(nnew - 1) * b.n3 + (long)q * 3 * b.n3;
      ax0[q] = 0.25 * (d2[ij] + d2[ij - 1]) * F.pmon_u[ij];
      ax1[q] = 0.25 * (d2[ij + 1] + d2[ij]) * F.pmon_u[ij + 1];
      ay0[q] = 0.25 * (d2[ij] + d2[ij - sj]) * F.pnom_v[ij];
      ay1[q] = 0.25 * (d2[ij + sj] + d2[ij]) * F.pnom_v[ij + sj];
    }
    const double um0 = F.umask[ij], um1 = F.umask[ij + 1], vm0 = F.vmask[ij], vm1 = F.vmask[ij + sj];
#pragma unroll 2
    for (int k = 1; k <= b.N; k++) {
      const long o = ij + (long)(k - 1) * n2;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const double FX1 = ax1[q] * (Hz[o + 1] + Hz[o]) * (Tr[q][o + 1] - Tr[q][o]) * um1;
        const double FX0 = ax0[q] * (Hz[o] + Hz[o - 1]) * (Tr[q][o] - Tr[q][o - 1]) * um0;
        const double FE1 = ay1[q] * (Hz[o + sj] + Hz[o]) * (Tr[q][o + sj] - Tr[q][o]) * vm1;
        const double FE0 = ay0[q] * (Hz[o] + Hz[o - sj]) * (Tr[q][o] - Tr[q][o - sj]) * vm0;
        Tn[q][o] = Tn[q][o] + pmn * (FX1 - FX0 + FE1 - FE0) / Hz[o];
      }
    }
    return;
  }
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    const double* d2 = F.diff2 + (long)(itrc - 1) * n2;
    const double* __restrict__ Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    double* __restrict__ Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    // 0.25*(diff2+diff2)*pmon_u per face (the first factors of the reference product)
    const double ax0 = 0.25 * (d2[ij] + d2[ij - 1]) * F.pmon_u[ij], ax1 = 0.25 * (d2[ij + 1] + d2[ij]) * F.pmon_u[ij + 1];
    const double ay0 = 0.25 * (d2[ij] + d2[ij - sj]) * F.pnom_v[ij], ay1 = 0.25 * (d2[ij + sj] + d2[ij]) * F.pnom_v[ij + sj];
    const double um0 = F.umask[ij], um1 = F.umask[ij + 1], vm0 = F.vmask[ij], vm1 = F.vmask[ij + sj];
#pragma unroll 2
    for (int k = 1; k <= b.N; k++) {
      const long o = ij + (long)(k - 1) * n2;
      const double FX1 = ax1 * (Hz[o + 1] + Hz[o]) * (Tr[o + 1] - Tr[o]) * um1;
      const double FX0 = ax0 * (Hz[o] + Hz[o - 1]) * (Tr[o] - Tr[o - 1]) * um0;
      const double FE1 = ay1 * (Hz[o + sj] + Hz[o]) * (Tr[o + sj] - Tr[o]) * vm1;
      const double FE0 = ay0 * (Hz[o] + Hz[o - sj]) * (Tr[o] - Tr[o - sj]) * vm0;
      Tn[o] = Tn[o] + pmn * (FX1 - FX0 + FE1 - FE0) / Hz[o];
    }
  }
}

// Two tracers with each level's Hz, T(nrhs), S(nrhs) windows (i0-1..i0+64 x
// j0-1..j0+4) staged in LDS once per block and the next level's in flight in
// registers (about 5 loads per lane per level for the stencils instead of
// 15); the per-tracer expressions of k_t3dmix, bit-identical.  Lanes past
// the range walk the levels too (barriers) and store nothing.
constexpr int kTMW = kBX + 2, kTMN = kTMW * (kBY + 2), kTMQ = (3 * kTMN + kBX * kBY - 1) / (kBX * kBY);
__global__ void __launch_bounds__(256) k_t3dmix_stg(Dev d, Range R, int nnew, int nrhs) {
  const uint3 bI = xcd_tile();
  __shared__ double sW[3 * kTMN];   // Hz, T, S
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  if (!act) { i = i < R.i0 ? R.i0 : (i < R.i1 ? i : R.i1); j = j < R.j1 ? j : R.j1; }
  const long ij = IJ(b, i, j), sj = b.nx2, n2 = b.n2;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  const double pmn = d.p.dt * F.pm[ij] * F.pn[ij];
  double ax0[2], ax1[2], ay0[2], ay1[2];
  double* __restrict__ Tn[2];
  const double* Tr[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const double* d2 = F.diff2 + (long)q * n2;
    Tr[q] = F.t + (long)(nrhs - 1) * b.n3 + (long)q * 3 * b.n3;
    Tn[q] = F.t + (long)(nnew - 1) * b.n3 + (long)q * 3 * b.n3;
    ax0[q] = 0.25 * (d2[ij] + d2[ij - 1]) * F.pmon_u[ij];
    ax1[q] = 0.25 * (d2[ij + 1] + d2[ij]) * F.pmon_u[ij + 1];
    ay0[q] = 0.25 * (d2[ij] + d2[ij - sj]) * F.pnom_v[ij];
    ay1[q] = 0.25 * (d2[ij + sj] + d2[ij]) * F.pnom_v[ij + sj];
  }
  const double um0 = F.umask[ij], um1 = F.umask[ij + 1], vm0 = F.vmask[ij], vm1 = F.vmask[ij + sj];
  // window entries of this thread: field (0 Hz, 1 T, 2 S, -1 none) and 2-D offset
  long wo[kTMQ];
  int wf[kTMQ];
#pragma unroll
  for (int m = 0; m < kTMQ; m++) {
    const int q = tid + m * kBX * kBY;
    const int f = q < 3 * kTMN ? q / kTMN : -1, qq = q - (f < 0 ? 0 : f) * kTMN;
    const int ii = i0 - 1 + qq % kTMW, jj = j0 - 1 + qq / kTMW;
    const bool ok = f >= 0 && ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2;
    wf[m] = ok ? f : -1;
    wo[m] = ok ? IJ(b, ii, jj) : 0;
  }
  auto ldw = [&](int k, double (&x)[kTMQ]) {
    const long kk = (long)(k - 1) * n2;
#pragma unroll
    for (int m = 0; m < kTMQ; m++)
      x[m] = wf[m] == 0 ? F.Hz[wo[m] + kk] : wf[m] == 1 ? Tr[0][wo[m] + kk] : wf[m] == 2 ? Tr[1][wo[m] + kk] : 0.0;
  };
  const int c = (threadIdx.x + 1) + (threadIdx.y + 1) * kTMW;   // the lane's cell in the window
  double w[kTMQ];
  ldw(1, w);
  for (int k = 1; k <= b.N; k++) {
    const long o = ij + (long)(k - 1) * n2;
    const double tn0 = Tn[0][o], tn1 = Tn[1][o];
    if (k > 1) __syncthreads();   // the previous level's window consumed
#pragma unroll
    for (int m = 0; m < kTMQ; m++) {
      const int q = tid + m * kBX * kBY;
      if (q < 3 * kTMN) sW[q] = w[m];
    }
    if (k < b.N) ldw(k + 1, w);
    __syncthreads();
    const double* H = sW;
    const double hz = H[c];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const double* T = sW + (1 + q) * kTMN;
      const double FX1 = ax1[q] * (H[c + 1] + hz) * (T[c + 1] - T[c]) * um1;
      const double FX0 = ax0[q] * (hz + H[c - 1]) * (T[c] - T[c - 1]) * um0;
      const double FE1 = ay1[q] * (H[c + kTMW] + hz) * (T[c + kTMW] - T[c]) * vm1;
      const double FE0 = ay0[q] * (hz + H[c - kTMW]) * (T[c] - T[c - kTMW]) * vm0;
      if (act) Tn[q][o] = (q == 0 ? tn0 : tn1) + pmn * (FX1 - FX0 + FE1 - FE0) / hz;
    }
  }
}

void launch_t3dmix(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  const bool stg = d.p.t3dmix_stg && b.NT == 2;
  auto run = [&](const Range& r) {
    if (stg) hipLaunchKernelGGL(k_t3dmix_stg, grid_of(r), dim3(kBX, kBY), 0, s, d, r, t.nnew, t.nrhs);
    else hipLaunchKernelGGL(k_t3dmix, grid_of(r), dim3(kBX, kBY), 0, s, d, r, t.nnew, t.nrhs);
  };
  ExchList L;
  if (tracer_exch_list(d, t.nnew, L)) {
    launch_rim_first(d, s, R, L, run, [] {});
  } else {
    run(R);
    launch_exchange_tracers(d, s, t.nnew);
  }
}

}  // namespace roms
