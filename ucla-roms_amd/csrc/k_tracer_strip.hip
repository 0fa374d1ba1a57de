// k_tracer_strip.hip -- the horizontal tracer advection of pre_step3d
// (pre_step3d4S.F:150-180, compute_horiz_tracer_fluxes.h centred) and of
// step3d_t (step3d_t_ISO.F:188-213, UPSTREAM_TS) in strips that march along j,
// the layout of k_prsgrd_strip.hip: one wavefront is 64 consecutive columns
// of one level and owns the 60 in its middle; the i-neighbours' values come
// through DPP lane shifts, the j-neighbours' stay in registers from the rows
// before, so each face's elementary difference and flux is formed once (the
// k_*_h1 tiles form every FX / FE twice, with clamped LDS indices).  Rows no
// closed-edge extrapolation reaches take this path; the strips at a closed
// west/east edge shuffle the clamped column; the south/north bands stay on
// the tiles.  Same expressions in the same order: bit-identical.
#include "k_common.h"

namespace roms {

namespace {
__device__ __forceinline__ double tdpp_shr(double x) {
  const long long v = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double tdpp_shl(double x) {
  const long long v = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
}  // namespace

constexpr int kTStripOwn = 60;
#ifndef ROMS_T_STRIP_J
#define ROMS_T_STRIP_J 8
#endif

struct TStripGeom {
  int c00;        // column of lane 0 of strip 0 (first owned column - 2)
  int ifirst, ilast;   // owned columns (the pre_step3d ring column istr-1 included)
  int jA, jB;     // rows
  int xlo, xhi;   // FX's elementary differences extrapolate outside [xlo, xhi] (closed west / east edge)
};
struct TStripPre {   // pre_step3d's coefficients (PreCoef) and time levels
  double dtau, cf_stp, cf_bak;
  int nstp, indx;
};

// MODE 0: step3d_t, t(nnew) -= dt*pm*pn*div (k_step3d_t_h1); MODE 1:
// pre_step3d, t(nnew) = Hz_bak*(cf_stp*t(nstp) + cf_bak*t(indx)) -
// dtau*pm*pn*div and t(indx) = Hz*t(nstp), with Hz_bak / Hz_fwd formed here
// (HBF true: every cell of the launch, the ring column istr-1 included;
// HBF false: Hz_bak read from c3, formed by the predictor's omega, and the
// ring column's by k_hb_ring).  One wavefront
// per (strip, rows, level, tracer): the tracers of a level are neighbours in
// the block order, so their shared inputs (FlxU/FlxV, masks, metrics) are
// fetched once into L2; one tracer per wave keeps the buffer descriptors
// (4 SGPRs each) within the scalar register file.  MODE 1 requires nrhs ==
// nstp (pre_step3d's time indices): t(nstp) is the advected field itself.
template <bool UP, int MODE, bool HBF>
__global__ void __launch_bounds__(64) k_tracer_strip(Dev d, TStripGeom G, int nnew, int nrhs, TStripPre pc) {
  constexpr int J = ROMS_T_STRIP_J;
  const uint3 bI = xcd_tile();
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int lane = (int)threadIdx.x;
  const int c0 = G.c00 + (int)bI.x * kTStripOwn;
  const int i = c0 + lane;
  const int ja = G.jA + (int)bI.y * J;
  const int nrow = min(J, G.jB - ja + 1);
  const int tr = (int)bI.z % b.NT, k = 1 + (int)bI.z / b.NT;
  const int il = max(min(i, b.Lm + 2), -1);
  const unsigned rb = (unsigned)b.nx2 * 8u;
  const unsigned vo = (unsigned)IJ(b, il, ja) * 8u;
  const unsigned sk = (unsigned)((long)(k - 1) * b.n2) * 8u;
  const bool own = lane >= 2 && lane <= 61 && i >= G.ifirst && i <= G.ilast;
  const bool in = own && i >= b.istr;           // tracer cells (the ring column forms Hz_bak / Hz_fwd only)
  const bool xedge = c0 + 1 < G.xlo || c0 + 62 > G.xhi;
  const int lx = iclamp(i, G.xlo, G.xhi) - c0;
  const long tb = (long)tr * 3 * b.n3;
  const BufF64 bum(F.umask), bvm(F.vmask), bFU(F.FlxU), bFV(F.FlxV), bpm(F.pm), bpn(F.pn);
  const BufF64 bT(F.t + (long)(nrhs - 1) * b.n3 + tb);   // t(nrhs): advected (= t(nstp) in MODE 1)
  const BufF64 bTn(F.t + (long)(nnew - 1) * b.n3 + tb);  // t(nnew)
  auto L3 = [&](const BufF64& B, int r) { return B.ld(vo + (unsigned)(r - ja) * rb, sk); };
  auto L2 = [&](const BufF64& B, int r) { return B.ld(vo + (unsigned)(r - ja) * rb, 0u); };
  // FX at this lane's u-point / FE at a v-point from the three elementary
  // differences around it (tracer_fx / tracer_fe of k_common.h)
  auto flux = [&](double tm, double tmm, double e0, double e1, double e2, double Fl) {
    if (UP) {
      const double cm = e1 - e0, cc = e2 - e1;
      return 0.5 * (tm + tmm) * Fl - 0.1666666666666666 * (cm * fmax0(Fl) + cc * fmin0(Fl));
    }
    const double gm = 0.5 * (e1 + e0), g0 = 0.5 * (e2 + e1);
    return 0.5 * (tm + tmm - 0.3333333333333333 * (g0 - gm)) * Fl;
  };
  // ---- prologue: tracer rows ja-2..ja+1, the v-point differences at
  // ja-1, ja, ja+1 and FE at v-point ja ----
  const int j = ja;
  double T0, T1, E0, E1, FEp;
  {
    const double vmm = L2(bvm, j - 1), vm0 = L2(bvm, j), vm1 = L2(bvm, j + 1), fv0 = L3(bFV, j);
    const double tm2 = L3(bT, j - 2), tm1 = L3(bT, j - 1), t0 = L3(bT, j), t1 = L3(bT, j + 1);
    const double em = (tm1 - tm2) * vmm, e0 = (t0 - tm1) * vm0, e1 = (t1 - t0) * vm1;
    FEp = flux(t0, tm1, em, e0, e1, fv0);
    T0 = t0; T1 = t1; E0 = e0; E1 = e1;
  }
  constexpr bool hbf = MODE == 1 && HBF;
  const bool hbst = tr == 0;   // the first tracer's waves store Hz_bak / Hz_fwd
  double FVc = hbf ? L3(bFV, j) : 0.0;   // FlxV of row j
  // ---- the march: a ring of two rows' inputs, row jr+2's loads issued
  // before row jr's stores (at one row ahead the wave waited for each row's
  // loads right after issuing them: this kernel has too little arithmetic per
  // row to cover a memory round trip) ----
  struct RowIn {
    double T2, A, vm2, um, fu, fv1, pm, pn, hz, hb, we1, wi1, we0, wi0;
  };
  const unsigned skw = (unsigned)((long)k * b.n2) * 8u, skw0 = (unsigned)((long)(k - 1) * b.n2) * 8u;
  auto load_row = [&](RowIn& q, int jr) {
    q.T2 = L3(bT, jr + 2);
    q.vm2 = L2(bvm, jr + 2); q.um = L2(bum, jr); q.fu = L3(bFU, jr); q.fv1 = L3(bFV, jr + 1);
    q.pm = L2(bpm, jr); q.pn = L2(bpn, jr);
    q.hz = q.hb = q.we1 = q.wi1 = q.we0 = q.wi0 = 0.0;
    if (MODE == 0) {
      q.A = L3(bTn, jr);
    } else {
      q.A = L3(BufF64(F.t + (long)(pc.indx - 1) * b.n3 + tb), jr);   // t(indx)
      q.hz = L3(BufF64(F.Hz), jr);
      if (!HBF) q.hb = L3(BufF64(F.c3), jr);
      if (hbf) {
        const unsigned v = vo + (unsigned)(jr - ja) * rb;
        const BufF64 bWe(F.We), bWi(F.Wi);
        q.we1 = bWe.ld(v, skw); q.wi1 = bWi.ld(v, skw); q.we0 = bWe.ld(v, skw0); q.wi0 = bWi.ld(v, skw0);
      }
    }
  };
  RowIn ring0, ring1;
  load_row(ring0, j);
  if (nrow > 1) load_row(ring1, j + 1);
#pragma unroll
  for (int r = 0; r < J; r++) {
    if (r >= nrow) break;
    const int jr = ja + r;
    RowIn& slot = (r & 1) ? ring1 : ring0;
    const RowIn q = slot;
    if (r + 2 < nrow) load_row(slot, jr + 2);
    const double T2 = q.T2, A = q.A, vm2 = q.vm2, um0 = q.um, fu0 = q.fu, fv1 = q.fv1, pm = q.pm, pn = q.pn;
    const double hz = q.hz, hbl = q.hb, we1 = q.we1, wi1 = q.wi1, we0 = q.we0, wi0 = q.wi0;
    const unsigned vr = vo + (unsigned)r * rb;
    // pre_step3d's Hz_bak / Hz_fwd (pre_step3d4S.F:136-148, hz_bak_fwd)
    double hb = hbl;
    if (MODE == 1 && hbf) {
      const double cff = 0.5 * pc.dtau;
      const double FlxDiv = cff * pm * pn * (tdpp_shl(fu0) - fu0 + fv1 - FVc + we1 + wi1 - we0 - wi0);
      const double hbn = hz + FlxDiv, hf = hz - FlxDiv;
      const bool st = hbst && own;
      BufF64(F.c2).st(hf, st ? vr : kBufOff, sk);
      BufF64(F.c3).st(hbn, st ? vr : kBufOff, sk);
      hb = hbn;
    }
    FVc = fv1;
    // XI: the u-point difference at this lane, FX at this lane's u-point and
    // (from the right) at the next
    const double Tl = tdpp_shr(T0);
    double el = (T0 - Tl) * um0;
    if (xedge) el = __shfl(el, lx);
    const double FX0 = flux(T0, Tl, tdpp_shr(el), el, tdpp_shl(el), fu0);
    const double FX1 = tdpp_shl(FX0);
    // ETA: v-point j+2's difference, FE at v-point j+1 (j carried)
    const double e2 = (T2 - T1) * vm2;
    const double FE1 = flux(T1, T0, E0, E1, e2, fv1);
    const double FE0 = FEp;
    if (MODE == 0) {
      bTn.st(A - d.p.dt * pm * pn * (FX1 - FX0 + FE1 - FE0), in ? vr : kBufOff, sk);
    } else {
      const double tsk = T0;   // t(nstp) = t(nrhs)
      bTn.st(hb * (pc.cf_stp * tsk + pc.cf_bak * A) - pc.dtau * pm * pn * (FX1 - FX0 + FE1 - FE0), in ? vr : kBufOff, sk);
      BufF64(F.t + (long)(pc.indx - 1) * b.n3 + tb).st(hz * tsk, in ? vr : kBufOff, sk);
    }
    T0 = T1; T1 = T2; E0 = E1; E1 = e2; FEp = FE1;
  }
}

// pre_step3d's Hz_bak / Hz_fwd of one column (i, rows j0..j1, every level):
// hz_bak_fwd (k_common.h, pre_step3d4S.F:136-148)
__global__ void __launch_bounds__(64) k_hb_ring(Dev d, int i, int j0, int j1, double cff) {
  const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int nj = j1 - j0 + 1;
  if (q >= nj * d.b.N) return;
  const int j = j0 + q % nj, k = 1 + q / nj;
  double bak, fwd;
  hz_bak_fwd(d, i, j, k, cff, bak, fwd);
  const long o = IJ(d.b, i, j) + (long)(k - 1) * d.b.n2;
  d.f.c2[o] = fwd;
  d.f.c3[o] = bak;
}

// Rows jA..jB of R in strips; false if the configuration is not one this
// kernel covers.  mode 0: step3d_t over R = (istr..iend) x rows; mode 1:
// pre_step3d over R = (istr-1..iend) x rows.
bool launch_tracer_strip(const Dev& d, hipStream_t s, const Range& R, int mode, bool up, bool hb_done, int nnew,
                         int nrhs, double dtau, double cf_stp, double cf_bak, int nstp, int& jA, int& jB) {
  const Bounds& b = d.b;
  if (!d.p.t_strip || d.p.nriv > 0 || (mode == 1 && (nrhs != nstp || up))) return false;
  // FE's elementary differences extrapolate at closed south / north edges
  // (compute_horiz_tracer_fluxes.h): FE(j), FE(j+1) read v-points j-1..j+2
  const int ylo = b.south_edge ? b.jstr : -1000000, yhi = b.north_edge ? b.jend + 1 : 1000000;
  jA = std::max(std::max(R.j0, ylo + 1), b.jstr);
  jA = std::max(jA, 1);
  jB = std::min(std::min(R.j1, yhi - 2), b.Mm);
  if (jB < jA) return false;
  TStripGeom G;
  G.ifirst = R.i0;
  G.ilast = R.i1;
  G.c00 = R.i0 - 2;
  G.jA = jA; G.jB = jB;
  G.xlo = b.west_edge ? b.istr : -1000000;
  G.xhi = b.east_edge ? b.iend + 1 : 1000000;
  TStripPre pc{dtau, cf_stp, cf_bak, nstp, 3 - nstp};
  constexpr int J = ROMS_T_STRIP_J;
  const dim3 grid((unsigned)((R.i1 - R.i0 + kTStripOwn) / kTStripOwn), (unsigned)((jB - jA + J) / J),
                  (unsigned)(b.N * b.NT));
#define TSTRIP(UP, MODE, HB) \
  hipLaunchKernelGGL((k_tracer_strip<UP, MODE, HB>), grid, dim3(64), 0, s, d, G, nnew, nrhs, pc)
  if (mode == 0) {
    if (up) TSTRIP(true, 0, false); else TSTRIP(false, 0, false);
  } else if (!hb_done) {
    TSTRIP(false, 1, true);
  } else {
    // Hz_bak read from c3 in the cells the predictor's omega formed; the
    // ring column istr-1 of rows jA..jB forms its own (k_hb_ring)
    G.ifirst = std::max(R.i0, b.istr);
    G.c00 = G.ifirst - 2;
    const dim3 g2((unsigned)((R.i1 - G.ifirst + kTStripOwn) / kTStripOwn), grid.y, grid.z);
    hipLaunchKernelGGL((k_tracer_strip<false, 1, false>), g2, dim3(64), 0, s, d, G, nnew, nrhs, pc);
    if (R.i0 < b.istr) {
      const int n = (jB - jA + 1) * b.N;
      hipLaunchKernelGGL(k_hb_ring, dim3((n + 63) / 64), dim3(64), 0, s, d, b.istr - 1, jA, jB, 0.5 * dtau);
    }
  }
#undef TSTRIP
  return true;
}

}  // namespace roms
