// k_vertical.hip -- column kernels: set_depth, set_HUV, set_HUV1, omega, rho_eos.
//
// One lane owns one (i,j) water column and walks k in registers; lanes of a
// wavefront are 64 consecutive i, so every level access is one coalesced
// 512-byte row.  Arithmetic order follows the reference statements so FP64
// results match the CPU reference bit for bit (built with -ffp-contract=off).
#include "roms_dev.h"
#include "k_chain.h"
#include "k_colseg.h"

namespace roms {

// ---------------------------------------------------------------------------
// set_depth_tile (set_depth.F:16-186): z_w, z_r, Hz from zeta(knew); at iic=0
// also hinv and the initial fast-time fluxes DU_avg1/DV_avg1.
// ---------------------------------------------------------------------------
// last: the end of the fast loop -- zeta(knew) = Zt_avg1 first (the fast-time
// average replaces the last fast step's zeta, step2d_FB.F:566), stored here
// on the same range instead of by a launch of its own
__global__ void __launch_bounds__(256) k_set_depth(Dev d, Range R, int iic, int knew, int last) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j);
  if (iic == 0) {
    F.hinv[ij] = 1.0 / (F.h[ij] + d.p.hc);
    if (i >= b.istr)
      F.DU_avg1[ij] = 0.5 * (F.h[IJ(b, i - 1, j)] + F.h[ij] + F.zeta[IJL(b, i, j, 1)] + F.zeta[IJL(b, i - 1, j, 1)]) *
                      F.dn_u[ij] * (F.ubar[IJL(b, i, j, 1)]);
    if (j >= b.jstr)
      F.DV_avg1[ij] = 0.5 * (F.h[ij] + F.h[IJ(b, i, j - 1)] + F.zeta[IJL(b, i, j, 1)] + F.zeta[IJL(b, i, j - 1, 1)]) *
                      F.dm_v[ij] * (F.vbar[IJL(b, i, j, 1)]);
  }
  const int N = b.N;
  const double hc = d.p.hc, ds = 1.0 / (double)N;
  const double hh = F.h[ij];
  const double hi = iic == 0 ? 1.0 / (hh + hc) : F.hinv[ij];
  double z;
  if (last) {
    z = F.Zt_avg1[ij];
    F.zeta[IJL(b, i, j, knew)] = z;
  } else {
    z = F.zeta[IJL(b, i, j, knew)];
  }
  double zw_prev = -hh;
  F.z_w[ij] = zw_prev;
  for (int k = 1; k <= N; k++) {
    const double cff_w = hc * ds * (double)(k - N);
    const double cff_r = hc * ds * ((double)(k - N) - 0.5);
    const double zw = z + (z + hh) * (cff_w + F.Cs_w[k] * hh) * hi;
    const double zr = z + (z + hh) * (cff_r + F.Cs_r[k] * hh) * hi;
    F.z_w[ij + (long)k * b.n2] = zw;
    F.z_r[ij + (long)(k - 1) * b.n2] = zr;
    F.Hz[ij + (long)(k - 1) * b.n2] = zw - zw_prev;
    zw_prev = zw;
  }
}

void launch_set_depth(const Dev& d, hipStream_t s, const Tlev& t, bool exchange, bool last) {
  const Bounds& b = d.b;
  Range R{b.istrR, b.iendR, b.jstrR, b.jendR};
  hipLaunchKernelGGL(k_set_depth, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.iic, t.knew, (int)last);
  if (t.iic == 0) launch_exchange(d, s, d.f.hinv, 1);
  if (exchange) launch_exchange_list(d, s, ExchList{{d.f.z_w, d.f.z_r, d.f.Hz}, {b.N + 1, b.N, b.N}, 3});
}

// ---------------------------------------------------------------------------
// set_HUV_tile (set_depth.F:190-234)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_set_huv(Dev d, Range R, int nrhs, int huv) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const bool du = i >= b.istr && i <= b.iendR && j >= b.jstrR && j <= b.jendR;
  const bool dv = i >= b.istrR && i <= b.iendR && j >= b.jstr && j <= b.jendR;
  const long ij = IJ(b, i, j), n2 = b.n2;
  // one lane per column, all levels: dn_u/dm_v read once per column
  const double dnu = du ? F.dn_u[ij] : 0.0, dmv = dv ? F.dm_v[ij] : 0.0;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ U = F.u + (long)(nrhs - 1) * b.n3 + ij;
  const double* __restrict__ V = F.v + (long)(nrhs - 1) * b.n3 + ij;
  double* __restrict__ FU = F.FlxU + ij;
  double* __restrict__ FV = F.FlxV + ij;
  double* __restrict__ HU = F.Hz_u + ij;
  double* __restrict__ HV = F.Hz_v + ij;
#pragma unroll 4
  for (int k = 1; k <= b.N; k++) {
    const long o = (long)(k - 1) * n2;
    const double hz = Hz[o];
    if (du) {
      const double hzm = Hz[o - 1];
      FU[o] = 0.5 * (hz + hzm) * dnu * (U[o]);
      if (huv) HU[o] = 0.5 * (hz + hzm);
    }
    if (dv) {
      const double hzm = Hz[o - b.nx2];
      FV[o] = 0.5 * (hz + hzm) * dmv * (V[o]);
      if (huv) HV[o] = 0.5 * (hz + hzm);
    }
  }
}

void launch_set_huv(const Dev& d, hipStream_t s, const Tlev& t, bool store_huv) {
  const Bounds& b = d.b;
  Range R{b.istrR < b.istr ? b.istrR : b.istr, b.iendR, b.jstrR < b.jstr ? b.jstrR : b.jstr, b.jendR};
  launch_rim_first(
      d, s, R, ExchList{{d.f.FlxU, d.f.FlxV}, {b.N, b.N}, 2},
      [&](const Range& r) {
        hipLaunchKernelGGL(k_set_huv, grid_of(r), dim3(kBX, kBY), 0, s, d, r, t.nrhs, (int)store_huv);
      },
      [] {});
}

// ---------------------------------------------------------------------------
// set_HUV1_tile (set_depth.F:239-422): remove the barotropic mismatch of
// u,v(nnew) against NOW/MID/BAK-extrapolated DU_avg's, recompute FlxU,FlxV.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_set_huv1(Dev d, Range R, int nnew, int first) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double NOW = 3.63, MID = 4.47, BAK = 2.05;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  for (int dir = 0; dir < 2; dir++) {
    if (dir == 0 && !(i >= b.istr && i <= b.iendR && j >= b.jstrR && j <= b.jendR)) continue;
    if (dir == 1 && !(i >= b.istrR && i <= b.iendR && j >= b.jstr && j <= b.jendR)) continue;
    const long s = dir == 0 ? 1 : b.nx2;
    const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
    double* __restrict__ u = (dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3 + ij;
    double* __restrict__ Flx = (dir == 0 ? F.FlxU : F.FlxV) + ij;
    const double* __restrict__ Hz = F.Hz + ij;
    long o = (long)(N - 1) * n2;
    double dcN = 0.5 * (Hz[o] + Hz[o - s]) * dn;
    double DC0 = dcN, FC0 = dcN * u[o];
#pragma unroll 8
    for (int k = N - 1; k >= 1; k--) {
      o = (long)(k - 1) * n2;
      const double dck = 0.5 * (Hz[o] + Hz[o - s]) * dn;
      DC0 = DC0 + dck;
      FC0 = FC0 + dck * u[o];
    }
    const double a1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
    if (first) FC0 = (FC0 - a1) / DC0;
    else {
      const double a2 = dir == 0 ? F.DU_avg2[ij] : F.DV_avg2[ij];
      const double ab = dir == 0 ? F.DU_avg_bak[ij] : F.DV_avg_bak[ij];
      FC0 = (FC0 - NOW * a1 + MID * a2 - BAK * ab) / DC0;
    }
    const double um = dir == 0 ? F.umask[ij] : F.vmask[ij];
#pragma unroll 8
    for (int k = 1; k <= N; k++) {
      o = (long)(k - 1) * n2;
      const double dck = 0.5 * (Hz[o] + Hz[o - s]) * dn;
      const double un = (u[o] - FC0) * um;
      u[o] = un;
      Flx[o] = dck * (un);
    }
  }
}

// Chained form (k_chain.h): the column's u and Hz_u*dn stay in the lane's
// registers between the sum and the correction pass; the two sums run down
// the segments in the reference's k = N..1 order (bit-identical).  The level
// loops are raw-buffer accesses as in k_uv2_fused: the lane's column and
// segment in one VGPR offset, the level in an SGPR; a level the lane does not
// own and every store of an inactive lane take kBufOff (load 0, store
// dropped), so the loops are straight-line code.  FULL: N == 4*KL (C3).
// KL > 13: the lane's Hz_u*dn levels sit in LDS (as k_uv2_fused's Hz_u), so
// the block fits 4 waves per SIMD in registers
template <int KL, bool FULL = false>
__global__ void __launch_bounds__(256, KL > 13 ? 3 : 4) k_set_huv1_chain(Dev d, Range R, int nnew, int first) {
  constexpr bool kDcLds = KL > 13;
  __shared__ double sDc[kDcLds ? KL * 256 : 1];
  const uint3 bI = xcd_tile();
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double NOW = 3.63, MID = 4.47, BAK = 2.05;
  const int N = b.N;
  const ChainLane cl = chain_lane<KL>(R, bI, N);
  const int nk = FULL ? KL : cl.nk;
  const long n2 = b.n2;
  // grid z = 2: one direction per block (both directions' loads in flight
  // at once across blocks); grid z = 1: both, one after the other
  const int d0 = gridDim.z == 2 ? (int)bI.z : 0, d1 = gridDim.z == 2 ? d0 + 1 : 2;
#pragma unroll 1
  for (int dir = d0; dir < d1; dir++) {
    const int ilo = dir == 0 ? b.istr : b.istrR, jlo = dir == 0 ? b.jstrR : b.jstr;
    const int ic = min(max(cl.i, ilo), b.iendR), jc = min(max(cl.j, jlo), b.jendR);
    const bool act = ic == cl.i && jc == cl.j && cl.in;
    const long ij = IJ(b, ic, jc), s = dir == 0 ? 1 : b.nx2;
    const double dn = dir == 0 ? F.dn_u[ij] : F.dm_v[ij];
    const BufF64 bU((dir == 0 ? F.u : F.v) + (long)(nnew - 1) * b.n3, b.n3), bHz(F.Hz, b.n3),
        bFl(dir == 0 ? F.FlxU : F.FlxV, b.n3);
    const unsigned vo = (unsigned)((ij + (long)(cl.lo - 1) * n2) * 8), vom = vo - (unsigned)(s * 8);
    auto so = [&](int q) { return (unsigned)((long)q * n2 * 8); };
    auto vq = [&](int q) { return q < nk ? vo : kBufOff; };
    auto vqm = [&](int q) { return q < nk ? vom : kBufOff; };
    auto vsq = [&](int q) { return act && q < nk ? vo : kBufOff; };
    double uu[KL], dcr[kDcLds ? 1 : KL];
    struct DcRef {   // dc[q]: Hz_u*dn of the lane's level lo+q, in LDS (kDcLds) or registers
      double* l;
      double* r;
      __device__ __forceinline__ double& operator[](int q) const { return kDcLds ? l[q * 256] : r[q]; }
    } const dc{sDc + threadIdx.x, dcr};
#pragma unroll
    for (int q = 0; q < KL; q++) {
      uu[q] = bU.ld(vq(q), so(q));
      dc[q] = 0.5 * (bHz.ld(vq(q), so(q)) + bHz.ld(vqm(q), so(q))) * dn;
      if (q % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    }
    double DC0, FC0;
    chain_down(cl, DC0, FC0, [&](double& a, double& c) {
#pragma unroll
      for (int q = KL - 1; q >= 0; q--) {
        a = q < nk ? a + dc[q] : a;
        c = q < nk ? c + dc[q] * uu[q] : c;
      }
    });
    const double a1 = dir == 0 ? F.DU_avg1[ij] : F.DV_avg1[ij];
    if (first) FC0 = (FC0 - a1) / DC0;
    else {
      const double a2 = dir == 0 ? F.DU_avg2[ij] : F.DV_avg2[ij];
      const double ab = dir == 0 ? F.DU_avg_bak[ij] : F.DV_avg_bak[ij];
      FC0 = (FC0 - NOW * a1 + MID * a2 - BAK * ab) / DC0;
    }
    const double um = dir == 0 ? F.umask[ij] : F.vmask[ij];
#pragma unroll
    for (int q = 0; q < KL; q++) {
      const double un = (uu[q] - FC0) * um;
      bU.st(un, vsq(q), so(q));
      bFl.st(dc[q] * (un), vsq(q), so(q));
    }
  }
}

void launch_set_huv1(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R{b.istrR < b.istr ? b.istrR : b.istr, b.iendR, b.jstrR < b.jstr ? b.jstrR : b.jstr, b.jendR};
  const int kl = chain_kl(b.N), first = (int)(t.iic == t.forw_start);
  dim3 gc = chain_grid_of(R);
  gc.z = d.p.chain_dirz ? 2 : 1;
  if (d.p.chain && kl == 5) hipLaunchKernelGGL(k_set_huv1_chain<5>, gc, dim3(256), 0, s, d, R, t.nnew, first);
  else if (d.p.chain && kl == 13) hipLaunchKernelGGL(k_set_huv1_chain<13>, gc, dim3(256), 0, s, d, R, t.nnew, first);
  else if (d.p.chain && kl == 25 && b.N == 100)
    hipLaunchKernelGGL((k_set_huv1_chain<25, true>), gc, dim3(256), 0, s, d, R, t.nnew, first);
  else if (d.p.chain && kl == 25) hipLaunchKernelGGL(k_set_huv1_chain<25>, gc, dim3(256), 0, s, d, R, t.nnew, first);
  else hipLaunchKernelGGL(k_set_huv1, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nnew, first);
  launch_exchange_list(d, s, ExchList{{d.f.FlxU, d.f.FlxV, d.f.u + (long)(t.nnew - 1) * b.n3,
                                        d.f.v + (long)(t.nnew - 1) * b.n3}, {b.N, b.N, b.N, b.N}, 4});
}

// ---------------------------------------------------------------------------
// omega_tile (omega.F:17-236): bottom-up continuity, grid-motion removal,
// Courant-limited explicit/implicit split of the vertical flux (We/Wi).
// ---------------------------------------------------------------------------
#ifndef ROMS_OMEGA_PF
#define ROMS_OMEGA_PF 4
#endif
__global__ void __launch_bounds__(256) k_omega(Dev d, Range R, double dtau) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double cu_min = 0.6, cu_max = 1.0, cmnx_ratio = cu_min / cu_max, cutoff = 2.0 - cmnx_ratio,
               r4cmx = 0.25 / (1.0 - cmnx_ratio);
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  const double* __restrict__ FU = F.FlxU + ij;
  const double* __restrict__ FV = F.FlxV + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ zw = F.z_w + ij;
  double* __restrict__ Wi = F.Wi + ij;
  double* __restrict__ We = F.We + ij;
  auto cx = [&](long o) { return fmax0(FU[o + 1]) - fmin0(FU[o]) + fmax0(FV[o + sj]) - fmin0(FV[o]); };
  // Two bottom-up passes over the column.  Pass 1 only forms the column
  // total of the divergence (omega.F:95-110) for the grid-motion term; pass 2
  // re-accumulates the same partial sums in the same order (bit-identical
  // Wi(k)) and applies the Courant split level by level (omega.F:120-165),
  // so Wi is never stored and re-read.  The split at level k needs
  // CX(k), CX(k+1), Hz(k), Hz(k+1): one level of look-ahead.
  const int pidx = d.p.npip > 0 ? F.pipe_idx[ij] : 0;
  const double pflx = pidx > 0 ? F.pipe_flx[ij] : 0.0;
  const double* __restrict__ prf = pidx > 0 ? F.pipe_prf + (pidx - 1) : nullptr;
  auto div = [&](int k, double wi) {  // wi - div(k) (+ pipe source), omega.F:102-108
    const long o = (long)(k - 1) * n2;
    wi = wi - FU[o + 1] + FU[o] - FV[o + sj] + FV[o];
    if (pidx > 0) wi = wi + pflx * prf[(long)(k - 1) * d.p.npip];
    return wi;
  };
  double wi = 0.0;
#pragma unroll 8
  for (int k = 1; k <= N; k++) wi = div(k, wi);
  wi = wi + F.swflx[ij] * F.dm_r[ij] * F.dn_r[ij];
  const double zw0 = zw[0];
  const double wrk = wi / (zw[(long)N * n2] - zw0);
  Wi[0] = 0.0;
  We[0] = 0.0;
  Wi[(long)N * n2] = 0.0;
  We[(long)N * n2] = 0.0;
  const double CX0 = dtau * F.pm[ij] * F.pn[ij];
#if ROMS_OMEGA_PF > 0
  // Pass 2 through a ring of ROMS_OMEGA_PF levels' raw loads, refilled
  // ahead of each level's We/Wi stores (which would otherwise hold back every
  // later load: the compiler cannot prove the arrays apart); the flux values
  // of level k serve both its divergence and its Courant number, as in the
  // reference, so each is loaded once.  Same expressions and order.
  struct Lv { double fu1, fu0, fv1, fv0, hz, zw; };   // rho level m; zw: w-level m-1
  auto ld = [&](int m) {
    m = m > N ? N : m;
    const long o = (long)(m - 1) * n2;
    return Lv{FU[o + 1], FU[o], FV[o + sj], FV[o], Hz[o], zw[o]};
  };
  Lv cur = ld(1);
  double cx_k = fmax0(cur.fu1) - fmin0(cur.fu0) + fmax0(cur.fv1) - fmin0(cur.fv0), hz_k = cur.hz;
  wi = 0.0;
  auto lev = [&](int k, const Lv& up) {
    const long o1 = (long)k * n2;  // level k+1 (rho layout) == w-level k
    wi = wi - cur.fu1 + cur.fu0 - cur.fv1 + cur.fv0;
    if (pidx > 0) wi = wi + pflx * prf[(long)(k - 1) * d.p.npip];
    double w = wi - wrk * (up.zw - zw0);
    const double cx_up = fmax0(up.fu1) - fmin0(up.fu0) + fmax0(up.fv1) - fmin0(up.fv0);
    const double hz_up = up.hz;
    const double c2d = dmax(cx_k, cx_up);
    const double dh = dmin(hz_k, hz_up);
    const double cw_max = cu_max * dh - c2d * CX0;
    double we;
    if (cw_max > 0.0) {
      const double cw_max2 = cw_max * cw_max;
      const double cw_min = cw_max * cmnx_ratio;
      const double cw = fabs(w) * CX0;
      double cff;
      if (cw < cw_min) cff = cw_max2;
      else if (cw < cutoff * cw_max) cff = cw_max2 + r4cmx * ((cw - cw_min) * (cw - cw_min));
      else cff = cw_max * cw;
      we = cw_max2 * w / cff;
      w = w - we;
    } else {
      we = 0.0;
    }
    We[o1] = we;
    Wi[o1] = w;
    cx_k = cx_up;
    hz_k = hz_up;
    cur = up;
  };
  constexpr int PF = ROMS_OMEGA_PF;
  Lv ring[PF];
#pragma unroll
  for (int q = 0; q < PF; q++) ring[q] = ld(2 + q);
  int k0 = 1;
  for (; k0 + PF - 1 <= N - 1; k0 += PF) {
#pragma unroll
    for (int q = 0; q < PF; q++) {
      const Lv up = ring[q];
      ring[q] = ld(k0 + q + 1 + PF);
      lev(k0 + q, up);
    }
  }
#pragma unroll
  for (int q = 0; q < PF; q++)
    if (k0 + q <= N - 1) lev(k0 + q, ring[q]);
}
#else
  double cx_k = cx(0), hz_k = Hz[0];
  wi = 0.0;
#pragma unroll 8
  for (int k = 1; k <= N - 1; k++) {
    const long o1 = (long)k * n2;  // level k+1 (rho layout) == w-level k
    wi = div(k, wi);
    double w = wi - wrk * (zw[o1] - zw0);
    const double cx_up = cx(o1);
    const double hz_up = Hz[o1];
    const double c2d = dmax(cx_k, cx_up);
    const double dh = dmin(hz_k, hz_up);
    const double cw_max = cu_max * dh - c2d * CX0;
    double we;
    if (cw_max > 0.0) {
      const double cw_max2 = cw_max * cw_max;
      const double cw_min = cw_max * cmnx_ratio;
      const double cw = fabs(w) * CX0;
      double cff;
      if (cw < cw_min) cff = cw_max2;
      else if (cw < cutoff * cw_max) cff = cw_max2 + r4cmx * ((cw - cw_min) * (cw - cw_min));
      else cff = cw_max * cw;
      we = cw_max2 * w / cff;
      w = w - we;
    } else {
      we = 0.0;
    }
    We[o1] = we;
    Wi[o1] = w;
    cx_k = cx_up;
    hz_k = hz_up;
  }
}
#endif

// Segment form of k_omega for deep grids (one read of every input).  k_omega's
// lane walks its column twice -- pass 1 for the column total of the
// divergence, pass 2 to re-form the same partial sums for the Courant split --
// and so reads FlxU/FlxV twice (at C3 the second read misses L2: 9.3 array
// passes of traffic for 6 of data).  Here a block of S wavefronts covers 64
// columns of one row j and wave s holds the raw inputs of its segment of
// levels (k_colseg.h seg_span) in registers, loaded once:
//   1. the partial sums wi(k) run up the column as one chain through the
//      waves in k order (wave s starts from wave s-1's last sum, handed over
//      in LDS between barriers): the same operations in the same order as
//      omega.F:102-108, so every wi(k) and the total are bit-identical;
//   2. with the total's wrk every level's Courant split (omega.F:120-165) is
//      independent: Courant number and Hz of the level above come from the
//      wave above through LDS at the segment top.
// Lanes outside the range solve a clamped duplicate column and store nothing.
//
// kHB (the predictor's omega, ROMS_GPU_OMEGA_HB): the same block also forms
// pre_step3d's Hz_bak / Hz_fwd = Hz +- 0.5 dtau pm pn (div(FlxU, FlxV) +
// We + Wi at the top - at the bottom) of its cells (pre_step3d4S.F:136-148,
// k_pre_tracer_h1's expression and order) into c3 / c2: the fluxes, Hz and
// the new We/Wi are all in its registers, and nothing between omega and
// pre_step3d writes them.  The flux differences of the level are kept in
// dynamic LDS across the chain ([kOmR][threads], through an opaque offset).
constexpr int kOmR = kSegRows;   // levels per wave (N <= kSegRows * kSegMaxS)
// CW columns per block (ROMS_GPU_OMEGA_CW, default 16: four segments per
// wavefront, several blocks per CU whose load and chain phases overlap;
// 1.41 -> 1.24 ms per C3 call against 64, r5_w_omega_cw_par_ab.txt; level
// offsets then go in the VGPR offset -- with SGPR offsets 32 columns had
// measured 1.76 ms, r5_p_seg_cw32_ab.txt).  PAR (ROMS_GPU_OMEGA_PAR, opt-in):
// each segment sums its own levels from zero while the others do, one
// barrier, then adds the lower segments' totals in k order -- the chain of S
// barrier steps becomes one (sums reassociated: not bitwise to PAR false;
// no faster at 16 columns).
constexpr int kOmCW = kCX, kOmBlock = kSegMaxS * kOmCW;
template <bool kHB, int CW = kOmCW, bool PAR = false>
__global__ void __launch_bounds__(kSegMaxS * CW, 2) k_omega_seg(Dev d, Range R, double dtau, double hcff) {
  // ROMS_GPU_OMEGA_ORD: the segment solvers' grouped block order (seg_tile)
  const uint3 bI = d.p.omega_ord ? seg_tile(d.p.omega_ord, d.p.seg_xg) : xcd_tile();
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double cu_min = 0.6, cu_max = 1.0, cmnx_ratio = cu_min / cu_max, cutoff = 2.0 - cmnx_ratio,
               r4cmx = 0.25 / (1.0 - cmnx_ratio);
  SegSpan sg = seg_span<CW>(N);
  constexpr bool kU = CW == kCX;   // one segment per wavefront: level offsets in SGPRs
  if constexpr (kU) seg_uniform<CW>(sg);
  const int s = sg.s, S = sg.S, c0 = sg.c0, n = sg.n, l = sg.col;
  const int iu = tile_i0(R.i0) + (int)bI.x * CW + l, ju = R.j0 + (int)bI.y;
  const bool act = iu >= R.i0 && iu <= R.i1 && ju <= R.j1;
  const int i = iu < R.i0 ? R.i0 : (iu < R.i1 ? iu : R.i1), j = ju < R.j1 ? ju : R.j1;
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  // buffer loads: the lane's column (and its i+1 / j+1 neighbour) in a VGPR,
  // the level in an SGPR (kU) or added to the VGPR offset
  const unsigned vo = (unsigned)ij * 8u, lv = (unsigned)n2 * 8u;
  const BufF64 FU(F.FlxU), FV(F.FlxV), Hz(F.Hz), zw(F.z_w);
  auto LD = [&](const BufF64& B, unsigned v, unsigned o) { return kU ? B.ld(v, o) : B.ld(v + o, 0u); };
  auto ST = [&](const BufF64& B, double x, unsigned v, unsigned o) {
    if constexpr (kU) B.st(x, v, o);
    else B.st(x, v + o, 0u);   // v = kBufOff stays beyond the extent
  };
  __shared__ double Lw[kSegMaxS][CW], Lcx[kSegMaxS][CW], Lhz[kSegMaxS][CW];
  __shared__ double Lte[kHB ? kSegMaxS : 1][CW], Lti[kHB ? kSegMaxS : 1][CW];   // kHB: segment tops' We, Wi
  double fu1[kOmR], fu0[kOmR], fv1[kOmR], fv0[kOmR], cx[kOmR], hz[kOmR], zk[kOmR];
#pragma unroll
  for (int q = 0; q < kOmR; q++) {   // rho level k = c0+q (clamped), w-level k
    const int k = min(c0 + q, N);
    const unsigned o = (unsigned)(k - 1) * lv;
    fu1[q] = LD(FU, vo + 8u, o); fu0[q] = LD(FU, vo, o); fv1[q] = LD(FV, vo + (unsigned)sj * 8u, o); fv0[q] = LD(FV, vo, o);
    hz[q] = LD(Hz, vo, o);
    zk[q] = LD(zw, vo, (unsigned)k * lv);
  }
  const double zw0 = zw.ld(vo, 0), zwN = zw.ld(vo, (unsigned)N * lv);
  const double wsrf = F.swflx[ij] * F.dm_r[ij] * F.dn_r[ij];
  const double CX0 = dtau * F.pm[ij] * F.pn[ij];
  const int pidx = d.p.npip > 0 ? F.pipe_idx[ij] : 0;
  const double pflx = pidx > 0 ? F.pipe_flx[ij] : 0.0;
  const double* __restrict__ prf = pidx > 0 ? F.pipe_prf + (pidx - 1) : nullptr;
#pragma unroll
  for (int q = 0; q < kOmR; q++) cx[q] = fmax0(fu1[q]) - fmin0(fu0[q]) + fmax0(fv1[q]) - fmin0(fv0[q]);
  const int nthr = (int)(blockDim.x * blockDim.y);
  int tl = (int)(threadIdx.x + blockDim.x * threadIdx.y);
  __asm__ volatile("" : "+v"(tl));
  if constexpr (kHB) {
#pragma unroll
    for (int q = 0; q < kOmR; q++) roms_smem[q * nthr + tl] = fu1[q] - fu0[q] + fv1[q] - fv0[q];
  }
  Lcx[s][l] = cx[0];
  Lhz[s][l] = hz[0];
  // 1. the partial sums, wave by wave in k order
  double wk[kOmR];
  if constexpr (PAR) {
    double wi = 0.0;
#pragma unroll
    for (int q = 0; q < kOmR; q++) {
      double v = wi - fu1[q] + fu0[q] - fv1[q] + fv0[q];
      if (pidx > 0) v = v + pflx * prf[(long)(min(c0 + q, N) - 1) * d.p.npip];
      wi = q < n ? v : wi;
      wk[q] = wi;
    }
    Lw[s][l] = wi;
    __syncthreads();
    double base = 0.0;
    for (int t = 0; t < s; t++) base = base + Lw[t][l];
#pragma unroll
    for (int q = 0; q < kOmR; q++) wk[q] = base + wk[q];
  } else
  for (int t = 0; t < S; t++) {
    if (s == t) {
      double wi = t == 0 ? 0.0 : Lw[t - 1][l];
#pragma unroll
      for (int q = 0; q < kOmR; q++) {
        double v = wi - fu1[q] + fu0[q] - fv1[q] + fv0[q];
        if (pidx > 0) v = v + pflx * prf[(long)(min(c0 + q, N) - 1) * d.p.npip];
        wi = q < n ? v : wi;
        wk[q] = wi;
      }
      Lw[t][l] = wi;
    }
    __syncthreads();
  }
  // 2. the Courant split of w-levels k = c0..c0+n-1 (k <= N-1)
  double wtot = Lw[S - 1][l];
  if constexpr (PAR) {
    wtot = 0.0;
    for (int t = 0; t < S; t++) wtot = wtot + Lw[t][l];
  }
  const double wrk = (wtot + wsrf) / (zwN - zw0);
  const double cx_top = s + 1 < S ? Lcx[s + 1][l] : 0.0, hz_top = s + 1 < S ? Lhz[s + 1][l] : 0.0;
  if (!kHB && !act) return;
  const BufF64 Wi(F.Wi), We(F.We);
  const unsigned vs = act ? vo : kBufOff;   // lanes outside the range store nothing
  // kHB: Hz_bak/fwd of cell k needs We, Wi at w-levels k and k-1
  const double hbf = kHB ? hcff * F.pm[ij] * F.pn[ij] : 0.0;
  const BufF64 Hf(F.c2), Hb(F.c3);
  double we_p = 0.0, wi_p = 0.0, we_f = 0.0, wi_f = 0.0;   // previous level's, the segment's first level's
  int tr = tl;
  __asm__ volatile("" : "+v"(tr));   // a second opaque offset: the stored differences are not forwarded
  auto hb_store = [&](int q, double we1, double wi1, double we0, double wi0) {
    const double div = roms_smem[q * nthr + tr];
    const double FlxDiv = hbf * (div + we1 + wi1 - we0 - wi0);
    const unsigned o = (unsigned)(c0 + q - 1) * lv;
    ST(Hf, hz[q] - FlxDiv, vs, o);
    ST(Hb, hz[q] + FlxDiv, vs, o);
  };
  if (s == 0) {
    ST(Wi, 0.0, vs, 0);
    ST(We, 0.0, vs, 0);
    ST(Wi, 0.0, vs, (unsigned)N * lv);
    ST(We, 0.0, vs, (unsigned)N * lv);
  }
#pragma unroll
  for (int q = 0; q < kOmR; q++) {
    const int k = c0 + q;
    double w = wk[q] - wrk * (zk[q] - zw0);
    const double cx_up = q + 1 < n ? cx[q + 1 < kOmR ? q + 1 : kOmR - 1] : cx_top;
    const double hz_up = q + 1 < n ? hz[q + 1 < kOmR ? q + 1 : kOmR - 1] : hz_top;
    const double c2d = dmax(cx[q], cx_up);
    const double dh = dmin(hz[q], hz_up);
    const double cw_max = cu_max * dh - c2d * CX0;
    double we;
    if (cw_max > 0.0) {
      const double cw_max2 = cw_max * cw_max;
      const double cw_min = cw_max * cmnx_ratio;
      const double cw = fabs(w) * CX0;
      double cff;
      if (cw < cw_min) cff = cw_max2;
      else if (cw < cutoff * cw_max) cff = cw_max2 + r4cmx * ((cw - cw_min) * (cw - cw_min));
      else cff = cw_max * cw;
      we = cw_max2 * w / cff;
      w = w - we;
    } else {
      we = 0.0;
    }
    if (q < n && k <= N - 1) {   // wave-uniform when kU
      ST(We, we, vs, (unsigned)k * lv);
      ST(Wi, w, vs, (unsigned)k * lv);
    }
    if constexpr (kHB) {
      const double we1 = k <= N - 1 ? we : 0.0, wi1 = k <= N - 1 ? w : 0.0;   // We(N) = Wi(N) = 0
      if (q == 0) { we_f = we1; wi_f = wi1; }
      if (q >= 1 && q < n) hb_store(q, we1, wi1, we_p, wi_p);
      if (q == n - 1) { Lte[s][l] = we1; Lti[s][l] = wi1; }   // this segment's top w-level, for the wave above
      we_p = we1; wi_p = wi1;
    }
  }
  if constexpr (kHB) {
    __syncthreads();
    const double we0 = s > 0 ? Lte[s - 1][l] : 0.0, wi0 = s > 0 ? Lti[s - 1][l] : 0.0;   // We(0) = Wi(0) = 0
    hb_store(0, we_f, wi_f, we0, wi0);
  }
}

// Closed-edge copies of We/Wi into the boundary ghost row (omega.F:171-232).
__global__ void k_omega_edges(Dev d) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = (int)blockIdx.y;  // k = 0..N
  const int nj = b.jend - b.jstr + 1, ni = b.iend - b.istr + 1;
  int di = 0, dj = 0, si = 0, sj = 0;
  if (p < nj) {
    if (!b.west_edge) return;
    dj = sj = b.jstr + p; di = b.istr - 1; si = b.istr;
  } else if (p < 2 * nj) {
    if (!b.east_edge) return;
    dj = sj = b.jstr + p - nj; di = b.iend + 1; si = b.iend;
  } else if (p < 2 * nj + ni) {
    if (!b.south_edge) return;
    di = si = b.istr + p - 2 * nj; dj = b.jstr - 1; sj = b.jstr;
  } else if (p < 2 * nj + 2 * ni) {
    if (!b.north_edge) return;
    di = si = b.istr + p - 2 * nj - ni; dj = b.jend + 1; sj = b.jend;
  } else {
    const int c = p - 2 * nj - 2 * ni;
    if (c == 0 && b.west_edge && b.south_edge) { di = b.istr - 1; dj = b.jstr - 1; si = b.istr; sj = b.jstr; }
    else if (c == 1 && b.west_edge && b.north_edge) { di = b.istr - 1; dj = b.jend + 1; si = b.istr; sj = b.jend; }
    else if (c == 2 && b.east_edge && b.south_edge) { di = b.iend + 1; dj = b.jstr - 1; si = b.iend; sj = b.jstr; }
    else if (c == 3 && b.east_edge && b.north_edge) { di = b.iend + 1; dj = b.jend + 1; si = b.iend; sj = b.jend; }
    else return;
  }
  const long dst = IJ(b, di, dj) + (long)k * b.n2, src = IJ(b, si, sj) + (long)k * b.n2;
  F.We[dst] = F.We[src];
  F.Wi[dst] = F.Wi[src];
}

static size_t omega_hb_lds_bytes(unsigned nthr) { return (size_t)kOmR * nthr * sizeof(double); }
void setup_omega_seg() {
  (void)hipFuncSetAttribute((const void*)k_omega_seg<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)omega_hb_lds_bytes(kOmBlock));
  (void)hipFuncSetAttribute((const void*)k_omega_seg<true, kOmCW, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)omega_hb_lds_bytes(kOmBlock));
}

// k_omega_seg<kHB, CW, PAR> by ROMS_GPU_OMEGA_CW / ROMS_GPU_OMEGA_PAR
template <bool kHB, int CW>
static void omega_seg_cw(const Dev& d, hipStream_t s, const Range& r, double dtau, double hcff) {
  const Bounds& b = d.b;
  const dim3 gs((r.i1 - tile_i0(r.i0) + CW) / CW, r.j1 - r.j0 + 1), bs(kCX, seg_waves<CW>(b.N));
  const size_t lds = kHB ? omega_hb_lds_bytes(bs.x * bs.y) : 0;
  if (d.p.omega_par) hipLaunchKernelGGL((k_omega_seg<kHB, CW, true>), gs, bs, lds, s, d, r, dtau, hcff);
  else hipLaunchKernelGGL((k_omega_seg<kHB, CW, false>), gs, bs, lds, s, d, r, dtau, hcff);
}
template <bool kHB>
static void omega_seg(const Dev& d, hipStream_t s, const Range& r, double dtau, double hcff) {
  if (d.p.omega_cw == 16) omega_seg_cw<kHB, 16>(d, s, r, dtau, hcff);
  else if (d.p.omega_cw == 32) omega_seg_cw<kHB, 32>(d, s, r, dtau, hcff);
  else omega_seg_cw<kHB, kOmCW>(d, s, r, dtau, hcff);
}

// hcff > 0 (the predictor's call): also form pre_step3d's Hz_bak / Hz_fwd of
// the interior cells into c3 / c2 with 0.5*dtau = hcff (k_omega_seg<true>);
// returns whether it did (one segment launch over the whole interior)
bool launch_omega(const Dev& d, hipStream_t s, const Tlev& t, double hcff) {
  const Bounds& b = d.b;
  double dtau;
  if (t.nrhs == 3) dtau = d.p.dt;
  else if (t.iic == t.forw_start) dtau = 0.5 * d.p.dt;
  else dtau = 0.6 * d.p.dt;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  const bool seg_ok = d.p.omega_seg && b.N <= kSegRows * kSegMaxS;
  const bool hb = hcff > 0.0 && seg_ok && R.i1 - R.i0 + 1 >= 32 && !rim_overlap_on(d, R);
  launch_rim_first(
      d, s, R, ExchList{{d.f.We, d.f.Wi}, {b.N + 1, b.N + 1}, 2},
      [&](const Range& r) {
        // the segment form for full-width ranges (rim strips keep k_omega)
        if (hb)
          omega_seg<true>(d, s, r, dtau, hcff);
        else if (seg_ok && r.i1 - r.i0 + 1 >= 32)
          omega_seg<false>(d, s, r, dtau, 0.0);
        else
          hipLaunchKernelGGL(k_omega, grid_of(r), dim3(kBX, kBY), 0, s, d, r, dtau);
      },
      [&] {
        if (b.west_edge || b.east_edge || b.south_edge || b.north_edge) {
          const int n = 2 * (b.jend - b.jstr + 1) + 2 * (b.iend - b.istr + 1) + 4;
          hipLaunchKernelGGL(k_omega_edges, dim3((n + 255) / 256, b.N + 1), dim3(256), 0, s, d);
        }
      });
  return hb;
}

// ---------------------------------------------------------------------------
// rho_eos_tile (rho_eos.F:24-409) over the extended range incl. halos.
// Linear EOS -> rho; NONLIN_EOS -> JM95 split form rho1,qp1 (DUKO_2001).
// bvf for LMD; VAR_RHO_2D column integrals rhoA, rhoS.
// ---------------------------------------------------------------------------
// prsgrd's hydrostatic pressure P (k_prsgrd_P, prsgrd.F:200-330) carried
// along rho_eos's own top-down sweep (kP, ROMS_GPU_P_IN_RHO): the sweep has
// z_r and the fresh rho1/qp1 (rho) of every level in registers, so P costs no
// reads of its own.  P of level m needs level m-1, so it runs one level
// behind: level(k) feeds the values of level k and completes P(k+1); last()
// completes P(1).  Expressions and order of k_prsgrd_P (bit-identical).
struct PColumn {
  double g, grho, HalfGRho, qp2, zwN, ptide;
  bool split, tides;
  BufF64 Pb{nullptr};   // P, stored through the column's buffer offset (kBufOff: a column outside doP)
  unsigned vP, lv;
  int N;
  double zC, rC, qC;                     // level m (pending)
  double eZk, eRk, dZ1, dR1, P1, z1, v1;
  __device__ __forceinline__ double rhov(double r1, double q1, double z) const {
    if (split) {
      const double dpth = -z;
      return r1 + q1 * dpth * (1.0 - qp2 * dpth);
    }
    return r1;
  }
  __device__ __forceinline__ double eRof(double ru, double rl, double qu, double ql, double zu, double zl) const {
    if (split) {
      const double dpth = -0.5 * (zu + zl);
      return ru - rl + (qu - ql) * dpth * (1.0 - qp2 * dpth);
    }
    return ru - rl;
  }
  // P-iteration of level m with level m-1 = (zM, rM, qM) (m >= 2) or none (m = 1)
  __device__ __forceinline__ void iter(int m, double zM, double rM, double qM) {
    const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
    if (m == N) {
      eZk = zC - zM;
      eRk = eRof(rC, rM, qC, qM, zC, zM);   // e(N) = e(N-1)
      dZ1 = 0.0; dR1 = 0.0; P1 = 0.0; z1 = 0.0; v1 = 0.0;
    }
    double eZm, eRm;
    if (m >= 2) { eZm = zC - zM; eRm = eRof(rC, rM, qC, qM, zC, zM); }
    else { eZm = eZk; eRm = eRk; }     // e(0) = e(1)
    const double dZk = [&] { const double c = 2.0 * eZk * eZm; return c / (eZk + eZm); }();
    double dRk;
    {
      const double c = 2.0 * eRk * eRm;
      dRk = c > 0.0 ? c / (eRk + eRm) : 0.0;
    }
    const double v0 = rhov(rC, qC, zC);
    if (split) {
      const double dpth = -zC;
      dRk = dRk - qC * dZk * (1.0 - 2.0 * qp2 * dpth);
    }
    double Pk;
    if (m == N) {
      const double rNm = rhov(rM, qM, zM);
      Pk = g * zwN + grho * (v0 + 0.5 * (v0 - rNm) * (zwN - zC) / (zC - zM)) * (zwN - zC);
      if (tides) Pk = Pk - g * ptide;
    } else {
      Pk = P1 + HalfGRho * ((v1 + v0) * (z1 - zC) -
                            OneFifth * ((dR1 - dRk) * (z1 - zC - OneTwelfth * (dZ1 + dZk)) -
                                        (dZ1 - dZk) * (v1 - v0 - OneTwelfth * (dR1 + dRk))));
    }
    Pb.st(Pk, vP, (unsigned)(m - 1) * lv);
    P1 = Pk;
    dZ1 = dZk; dR1 = dRk;
    eZk = eZm; eRk = eRm;
    z1 = zC; v1 = v0;
  }
  // rho_eos produced level k (k = N..1)
  __device__ __forceinline__ void level(int k, double z, double r, double q) {
    if (k < N) iter(k + 1, z, r, q);
    zC = z; rC = r; qC = q;
  }
  __device__ __forceinline__ void last() { iter(1, 0.0, 0.0, 0.0); }
};
__device__ __forceinline__ PColumn p_column(const Dev& d, int i, int j, long ij, bool split) {
  const Bounds& b = d.b;
  PColumn c;
  c.g = d.p.g; c.grho = d.p.g / d.p.rho0; c.HalfGRho = 0.5 * c.grho; c.qp2 = d.p.qp2;
  c.split = split; c.tides = d.p.tides != 0; c.N = b.N; c.lv = (unsigned)b.n2 * 8u;
  // k_prsgrd_P's range (0..Lm x 0..Mm) and its P columns
  const bool doP = i >= 0 && i <= b.Lm && j >= 0 && j <= b.Mm && i >= b.istrU - 1 && i <= b.iend;
  c.Pb = BufF64(d.f.P);
  c.vP = doP ? (unsigned)ij * 8u : kBufOff;
  c.zwN = d.f.z_w[ij + (long)b.N * b.n2];
  c.ptide = c.tides ? d.f.ptide[ij] : 0.0;
  return c;
}

template <bool kP>
__global__ void __launch_bounds__(256) k_rho_eos_linear(Dev d, Range R, int tidx) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double rm = F.rmask[ij];
  const double cff0 = P.salinity ? (P.Tcoef * P.T0 - P.Scoef * P.S0) : (P.Tcoef * P.T0);
  const double* __restrict__ T = F.t + (long)(tidx - 1) * b.n3 + ij;
  const double* __restrict__ Sa = T + 3 * b.n3;
  const double* __restrict__ Hz = F.Hz + ij;
  double* __restrict__ rho = F.rho + ij;
  const bool salt = P.salinity;
  auto rhok = [&](long o) {
    double r = cff0 - P.Tcoef * T[o];
    if (salt) r = r + P.Scoef * Sa[o];
    return r * rm;
  };
  // rho(k) and the VAR_RHO_2D integrals from the top down in one pass
  PColumn pc;
  if constexpr (kP) pc = p_column(d, i, j, ij, false);
  const double* __restrict__ zrp = F.z_r + ij;
  long o = (long)(N - 1) * n2;
  double rk = rhok(o);
  rho[o] = rk;
  if constexpr (kP) pc.level(N, zrp[o], rk, 0.0);
  double cff = Hz[o] * rk;
  double rhoS = 0.5 * cff * Hz[o];
  double rhoA = cff;
#pragma unroll 8
  for (int k = N - 1; k >= 1; k--) {
    o = (long)(k - 1) * n2;
    rk = rhok(o);
    rho[o] = rk;
    if constexpr (kP) pc.level(k, zrp[o], rk, 0.0);
    const double hz = Hz[o];
    cff = hz * rk;
    rhoS = rhoS + hz * (rhoA + 0.5 * cff);
    rhoA = rhoA + cff;
  }
  if constexpr (kP) pc.last();
  if (P.lmd) {
    const double c = P.g / P.rho0;
    const double* __restrict__ zr = F.z_r + ij;
    double* __restrict__ bvf = F.bvf + ij;
    for (int k = 1; k <= N - 1; k++) {
      const long q = (long)(k - 1) * n2;
      bvf[(long)k * n2] = c * (rho[q] - rho[q + n2]) / (zr[q + n2] - zr[q]);
    }
    bvf[(long)N * n2] = bvf[(long)(N - 1) * n2];
    bvf[0] = bvf[n2];
  }
  const double cff1 = 1.0 / P.rho0;
  cff = 1.0 / (F.z_w[ij + (long)N * n2] - F.z_w[ij]);
  F.rhoA[ij] = cff * cff1 * rhoA;
  F.rhoS[ij] = 2.0 * cff * cff * cff1 * rhoS;
}

#ifndef ROMS_RHO_UNROLL
// 1: 2 SGPR spills and 4 waves/SIMD instead of 13 spills at 3 (unroll 4);
// rho_eos 1.446 vs 1.441 ms per C3 call, within noise (profiles/r6_e_tracer_strip_ab.txt)
#define ROMS_RHO_UNROLL 1
#endif
#ifndef ROMS_RHO_PF
#define ROMS_RHO_PF 4
#endif
#ifndef ROMS_RHO_MINW   // minimum waves per SIMD of k_rho_eos_split (VGPR cap; A/B builds)
#define ROMS_RHO_MINW 1
#endif
template <bool kP>
__global__ void __launch_bounds__(256, ROMS_RHO_MINW) k_rho_eos_split(Dev d, Range R, int tidx) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const double rho0 = P.rho0, qp2 = P.qp2;
  const double r00 = 999.842594, r01 = 6.793952E-2, r02 = -9.095290E-3, r03 = 1.001685E-4, r04 = -1.120083E-6,
               r05 = 6.536332E-9, r10 = 0.824493, r11 = -4.08990E-3, r12 = 7.64380E-5, r13 = -8.24670E-7,
               r14 = 5.38750E-9, rS0 = -5.72466E-3, rS1 = 1.02270E-4, rS2 = -1.65460E-6, r20 = 4.8314E-4,
               K00 = 19092.56, K01 = 209.8925, K02 = -3.041638, K03 = -1.852732e-3, K04 = -1.361629e-5,
               K10 = 104.4077, K11 = -6.500517, K12 = 0.1553190, K13 = 2.326469e-4, KS0 = -5.587545,
               KS1 = +0.7390729, KS2 = -1.909078e-2;
  double Tt = 3.8, Ts = 34.5, sqrtTs = sqrt(Ts);
  const double K0_Duk = Tt * (K01 + Tt * (K02 + Tt * (K03 + Tt * K04))) +
                        Ts * (K10 + Tt * (K11 + Tt * (K12 + Tt * K13)) + sqrtTs * (KS0 + Tt * (KS1 + Tt * KS2)));
  const double dr00 = r00 - rho0;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double rm = F.rmask[ij];
  // one top-down sweep: rho1, qp1 (rho_eos.F:208-262), bvf(k) from levels k
  // and k+1 (:270-300) and the rhoA/rhoS column integrals (:365-395), each
  // expression in the reference's order; restrict pointers let the loads of
  // the next levels issue ahead of this level's stores
  // buffer accesses: the column in one VGPR offset, the level in an SGPR
  const unsigned vo = (unsigned)ij * 8u, lv = (unsigned)n2 * 8u;
  const BufF64 T(F.t + (long)(tidx - 1) * b.n3), Sa(F.t + (long)(tidx - 1) * b.n3 + 3 * b.n3), zr(F.z_r), Hz(F.Hz),
      rho1(F.rho1), qp1(F.qp1), bvf(F.bvf);
  const bool lmd = P.lmd;
  const double gr = P.g / rho0;
  double r1p = 0.0, q1p = 0.0, zrp = 0.0;  // level k+1
  double rhoA = 0.0, rhoS = 0.0, bvN1 = 0.0, bv1 = 0.0;
  PColumn pc;
  if constexpr (kP) pc = p_column(d, i, j, ij, true);
  // the next levels' inputs are loaded before this level's stores (a ring
  // of ROMS_RHO_PF levels), so the stores -- counted with the loads by
  // vmcnt -- do not hold back the loads below them
  constexpr int PF = ROMS_RHO_PF;
  double pT[PF], pS[PF], pZ[PF], pH[PF];
#pragma unroll
  for (int q = 0; q < PF; q++) {
    const unsigned o = (unsigned)max(N - 1 - q, 0) * lv;
    pT[q] = T.ld(vo, o); pS[q] = Sa.ld(vo, o); pZ[q] = zr.ld(vo, o); pH[q] = Hz.ld(vo, o);
  }
#pragma unroll ROMS_RHO_UNROLL
  for (int k = N; k >= 1; k--) {
    const unsigned o = (unsigned)(k - 1) * lv;
    Tt = pT[0];
    Ts = pS[0];
    const double zrk = pZ[0], hz = pH[0];
#pragma unroll
    for (int q = 0; q + 1 < PF; q++) { pT[q] = pT[q + 1]; pS[q] = pS[q + 1]; pZ[q] = pZ[q + 1]; pH[q] = pH[q + 1]; }
    {
      const unsigned on = (unsigned)max(k - 1 - PF, 0) * lv;   // level k - PF (clamped; unused past the bottom)
      pT[PF - 1] = T.ld(vo, on); pS[PF - 1] = Sa.ld(vo, on); pZ[PF - 1] = zr.ld(vo, on); pH[PF - 1] = Hz.ld(vo, on);
    }
    sqrtTs = sqrt(dmax(0.0, Ts));
    const double r1 = (dr00 + Tt * (r01 + Tt * (r02 + Tt * (r03 + Tt * (r04 + Tt * r05)))) +
                       Ts * (r10 + Tt * (r11 + Tt * (r12 + Tt * (r13 + Tt * r14))) + sqrtTs * (rS0 + Tt * (rS1 + Tt * rS2)) +
                             Ts * r20)) *
                      rm;
    rho1.st(r1, vo, o);
    const double K0 = Tt * (K01 + Tt * (K02 + Tt * (K03 + Tt * K04))) +
                      Ts * (K10 + Tt * (K11 + Tt * (K12 + Tt * K13)) + sqrtTs * (KS0 + Tt * (KS1 + Tt * KS2)));
    const double q1 = 0.1 * (rho0 + r1) * (K0_Duk - K0) / ((K00 + K0) * (K00 + K0_Duk)) * rm;
    qp1.st(q1, vo, o);
    if constexpr (kP) pc.level(k, zrk, r1, q1);
    if (lmd && k < N) {
      const double dpth = -0.5 * (zrp + zrk);
      const double bv = -gr * (r1p - r1 + (q1p - q1) * dpth * (1.0 - qp2 * dpth)) / (zrp - zrk) * rm;
      bvf.st(bv, vo, (unsigned)k * lv);
      bvN1 = k == N - 1 ? bv : bvN1;   // the boundary copies below
      bv1 = k == 1 ? bv : bv1;
    }
    const double dpth = -zrk;
    const double cff = hz * (r1 + q1 * dpth * (1.0 - qp2 * dpth));
    if (k == N) {
      rhoS = 0.5 * cff * hz;
      rhoA = cff;
    } else {
      rhoS = rhoS + hz * (rhoA + 0.5 * cff);
      rhoA = rhoA + cff;
    }
    r1p = r1; q1p = q1; zrp = zrk;
  }
  if constexpr (kP) pc.last();
  if (lmd && N >= 2) {   // bvf(N) = bvf(N-1), bvf(0) = bvf(1) (rho_eos.F:300-305)
    bvf.st(bvN1, vo, (unsigned)N * lv);
    bvf.st(bv1, vo, 0);
  }
  const double cff1 = 1.0 / rho0;
  const double cff = 1.0 / (F.z_w[ij + (long)N * n2] - F.z_w[ij]);
  F.rhoA[ij] = cff * cff1 * rhoA;
  F.rhoS[ij] = 2.0 * cff * cff * cff1 * rhoS;
}

// P in rho_eos (PColumn): every rho_eos of the library then leaves P
// current for its rho1/qp1, so whole steps skip k_prsgrd_P.  Split EOS only:
// the linear EOS sweep is short and memory-bound, and P's per-level division
// chain at its lower occupancy made it slower than k_prsgrd_P
// (r3_zl_p_in_rho_ab.txt: C2 +0.08 ms/step, C3 -2.2 ms/step)
bool p_in_rho(const Dev& d) {
  const Bounds& b = d.b;
  return d.p.p_in_rho && d.p.nonlin_eos && d.p.prs_split && !d.p.tides && b.N >= 2 && b.istrE <= 0 &&
         b.iendE >= b.Lm && b.jstrE <= 0 && b.jendE >= b.Mm;
}
void launch_rho_eos(const Dev& d, hipStream_t s, const Tlev& t, int tidx) {
  const Bounds& b = d.b;
  Range R{b.istrE, b.iendE, b.jstrE, b.jendE};
  const bool kp = p_in_rho(d);
  if (d.p.nonlin_eos) {
    if (kp) hipLaunchKernelGGL(k_rho_eos_split<true>, grid_of(R), dim3(kBX, kBY), 0, s, d, R, tidx);
    else hipLaunchKernelGGL(k_rho_eos_split<false>, grid_of(R), dim3(kBX, kBY), 0, s, d, R, tidx);
  } else {
    if (kp) hipLaunchKernelGGL(k_rho_eos_linear<true>, grid_of(R), dim3(kBX, kBY), 0, s, d, R, tidx);
    else hipLaunchKernelGGL(k_rho_eos_linear<false>, grid_of(R), dim3(kBX, kBY), 0, s, d, R, tidx);
  }
}

}  // namespace roms
