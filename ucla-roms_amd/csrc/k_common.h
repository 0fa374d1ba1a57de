// k_common.h -- device restatements of the reference's shared flux fragments:
//   compute_horiz_tracer_fluxes.h  (4th-order centred / UPSTREAM_TS)
//   compute_vert_tracer_fluxes.h   (SPLINE_TS, natural b.c.)
//   compute_horiz_rhs_uv_terms.h   (UV_COR + UV_ADV, centred / UPSTREAM_UV)
//   compute_vert_rhs_uv_terms.h    (SPLINE_UV, MASKING)
// The reference evaluates these over extended index ranges into 2-D scratch;
// here each lane recomputes the face values it needs from the inputs, which
// keeps the arithmetic of every face identical and removes the scratch round
// trip through HBM.  The one-sided edge extrapolations of the reference become
// index clamps at closed (non-periodic) physical edges.
#pragma once
#include "roms_dev.h"
#include <type_traits>

namespace roms {

// Raw-buffer view of one device array (gfx950 buffer_load / buffer_store):
// the lane's byte offset in a VGPR (32-bit), the level's in an SGPR
// (soffset), so a column walk keeps no 64-bit address per level in vector
// registers -- the straight-line level loops of the column kernels otherwise
// hold one address pair per level live across their passes (k_uv2_fused
// spilled ~200 VGPRs that way).  Offsets must stay below 2 GiB from the base
// (one 3-D field or one time slot: 855 MB at 1024^2 x 100); roms_gpu_init
// refuses larger subdomains (buffer_span_ok, roms_dev.h).
// With the array's extent given, an access beyond it is dropped by the
// hardware (a store does nothing, a load returns 0): lanes that must not store
// pass kBufOff instead of branching around the store, which keeps a level
// loop straight-line code.
constexpr unsigned kBufOff = 0x80000000u;   // + any level offset below 2 GiB: beyond every extent used here
struct BufF64 {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit BufF64(const double* p, long n = 0)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), (short)0,
                                            n > 0 ? (int)(unsigned)(n * 8) : (int)0x7fffffff, 0x00020000)) {}
  __device__ __forceinline__ double ld(unsigned vb, unsigned sb) const {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)vb, (int)sb, 0));
  }
  __device__ __forceinline__ void st(double v, unsigned vb, unsigned sb) const {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) int, v), r, (int)vb,
                                          (int)sb, 0);
  }
};

// LDS window of a 64x4 tile with a 2-cell halo on every side (i0-2.., j0-2..)
constexpr int kUVW = kBX + 4, kUVH = kBY + 4, kUVN = kUVW * kUVH;

// A lane's column scratch (levels 0..N) in LDS: level k of lane l at
// smem[k*kCX + l], so a wavefront touches 64 consecutive doubles per level
// (conflict-free).  Sweeps that keep their forward-elimination results here
// issue no global stores until the back-substitution, so the global loads of
// the inputs carry no aliasing hazards and can be scheduled ahead of use.
struct ColLds {
  double* p;
  __device__ __forceinline__ double& operator[](int k) const { return p[k * kCX]; }
};
extern __shared__ double roms_smem[];
__device__ __forceinline__ ColLds col_lds(int slot, int N) {
  return ColLds{roms_smem + (long)slot * (N + 1) * kCX + threadIdx.x};
}
inline size_t col_lds_bytes(int nslots, int N) { return (size_t)nslots * (N + 1) * kCX * sizeof(double); }
// Debug builds (-DROMS_LDS_POISON): every lane fills its column slots with NaN
// at kernel entry, so a read of a slot the kernel never wrote shows up as NaN
// instead of whatever an earlier dispatch left in LDS.
template <class C>
__device__ __forceinline__ void col_lds_poison(int nslots, int N) {
#ifdef ROMS_LDS_POISON
  if constexpr (std::is_same<C, ColLds>::value)
    for (int q = 0; q < nslots * (N + 1); q++) roms_smem[q * kCX + threadIdx.x] = __builtin_nan("");
#endif
}

// The same column scratch in global memory (w-point layout, level k of column
// ij at p[k*n2]: a wavefront still touches 64 consecutive doubles per level).
// Deep columns use it: two LDS slots of N=100 levels are 103 KB per wave,
// which leaves one wave per CU; in HBM (caught by L2 / Infinity Cache) the
// solvers keep full occupancy.  Slot (z, s) of a kernel whose grid z indexes
// tracers or directions lives at colscr + (2z + s)*n3w.
struct ColGlb {
  double* p;
  long s;
  __device__ __forceinline__ double& operator[](int k) const { return p[(long)k * s]; }
};
template <class C>
struct ColMake;
template <>
struct ColMake<ColLds> {
  __device__ static ColLds at(const Dev& d, int slot, int z, long ij) { return col_lds(slot, d.b.N); }
};
template <>
struct ColMake<ColGlb> {
  __device__ static ColGlb at(const Dev& d, int slot, int z, long ij) {
    return ColGlb{d.f.colscr + ((long)z * 2 + slot) * d.b.n3w + ij, d.b.n2};
  }
};

// ---- pseudo-continuity of the predictor (pre_step3d4S.F:136-148) ----
__device__ __forceinline__ void hz_bak_fwd(const Dev& d, int i, int j, int k, double cff, double& bak, double& fwd) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), o = ij + (long)(k - 1) * b.n2, w = ij + (long)k * b.n2;
  const double FlxDiv = cff * F.pm[ij] * F.pn[ij] *
                        (F.FlxU[o + 1] - F.FlxU[o] + F.FlxV[o + b.nx2] - F.FlxV[o] + F.We[w] + F.Wi[w] -
                         F.We[w - b.n2] - F.Wi[w - b.n2]);
  bak = F.Hz[o] + FlxDiv;
  fwd = F.Hz[o] - FlxDiv;
}

// ---- SPLINE_TS vertical advective flux of one tracer column in LDS
// (compute_vert_tracer_fluxes.h): FC(0:N) by the spline elimination, then
// A[k] = FC(k)*We(k), A[0] = A[N] = 0.  Per-level inputs come through a
// register ring kPF levels ahead of use (whole unrolled groups, then a
// direct remainder), so the loads overlap the division chain.
constexpr int kPF = 8;
template <class C>
__device__ __forceinline__ void tracer_spline_lds(int N, long n2, const double* __restrict__ Hz,
                                                  const double* __restrict__ Tr, const double* __restrict__ We,
                                                  const C& A, const C& B) {
    double cfk = 1.0, fcm = 2.0 * Tr[0], hk = Hz[0], tk = Tr[0];
    A[0] = fcm;
    // inputs of the next kPF levels stay in flight in a register ring (slot q
    // of an unrolled group of kPF levels holds level k0+q+kPF after use);
    // whole groups first, the remaining < kPF levels load directly
    auto spl_fwd = [&](int k, double hk1, double tk1) {
      const double cff = 1.0 / (2.0 * hk + hk1 * (2.0 - cfk));
      const double cf1 = cff * hk;
      const double fck = cff * (3.0 * (hk * tk1 + hk1 * tk) - hk1 * fcm);
      B[k + 1] = cf1;
      A[k] = fck;
      cfk = cf1; fcm = fck; hk = hk1; tk = tk1;
    };
    int k0 = 1;
    {
      double rh[kPF], rt[kPF];
#pragma unroll
      for (int q = 0; q < kPF; q++) {
        const long L = (long)min(1 + q, N - 1) * n2;
        rh[q] = Hz[L]; rt[q] = Tr[L];
      }
      for (; k0 + kPF - 1 <= N - 1; k0 += kPF) {
#pragma unroll
        for (int q = 0; q < kPF; q++) {
          const double hk1 = rh[q], tk1 = rt[q];
          const long L = (long)min(k0 + q + kPF, N - 1) * n2;
          rh[q] = Hz[L]; rt[q] = Tr[L];
          spl_fwd(k0 + q, hk1, tk1);
        }
      }
    }
    for (int k = k0; k <= N - 1; k++) spl_fwd(k, Hz[(long)k * n2], Tr[(long)k * n2]);
    double fc1 = (2.0 * tk - fcm) / (1.0 - cfk);
    {
      auto spl_bwd = [&](int k, double we) {
        const double fck = A[k] - B[k + 1] * fc1;
        A[k + 1] = fc1 * we;
        A[k] = fck;
        fc1 = fck;
      };
      int k1 = N - 1;
      double rw[kPF];
#pragma unroll
      for (int q = 0; q < kPF; q++) rw[q] = We[(long)max(N - q, 1) * n2];
      for (; k1 - kPF + 1 >= 0; k1 -= kPF) {
#pragma unroll
        for (int q = 0; q < kPF; q++) {
          const double we = rw[q];
          rw[q] = We[(long)max(k1 - q + 1 - kPF, 1) * n2];
          spl_bwd(k1 - q, we);
        }
      }
      for (int k = k1; k >= 0; k--) spl_bwd(k, We[(long)(k + 1) * n2]);
    }
  A[N] = 0.0;
  A[0] = 0.0;
}

// ---- register-resident form of tracer_spline_lds for a compile-time depth
// NN (the k_uv1_reg pattern): FC lives in A[0..NN] (VGPRs), CF in one LDS
// slot B, and every level loop is fully unrolled so each A[k] is a fixed
// register and the compiler schedules the (alias-free) global loads ahead.
// Same expressions and order as tracer_spline_lds: bit-identical results. ----
template <int NN, class CB>
__device__ __forceinline__ void tracer_spline_reg(long n2, const double* __restrict__ Hz,
                                                  const double* __restrict__ Tr, const double* __restrict__ We,
                                                  double (&A)[NN + 1], const CB& B) {
  constexpr int N = NN;
  double cfk = 1.0, fcm = 2.0 * Tr[0], hk = Hz[0], tk = Tr[0];
  A[0] = fcm;
#pragma unroll
  for (int k = 1; k <= N - 1; k++) {
    const double hk1 = Hz[(long)k * n2], tk1 = Tr[(long)k * n2];
    const double cff = 1.0 / (2.0 * hk + hk1 * (2.0 - cfk));
    const double cf1 = cff * hk;
    const double fck = cff * (3.0 * (hk * tk1 + hk1 * tk) - hk1 * fcm);
    B[k + 1] = cf1;
    A[k] = fck;
    cfk = cf1; fcm = fck; hk = hk1; tk = tk1;
  }
  double fc1 = (2.0 * tk - fcm) / (1.0 - cfk);
#pragma unroll
  for (int k = N - 1; k >= 0; k--) {
    const double fck = A[k] - B[k + 1] * fc1;
    A[k + 1] = fc1 * We[(long)(k + 1) * n2];
    A[k] = fck;
    fc1 = fck;
  }
  A[N] = 0.0;
  A[0] = 0.0;
}

// ---- river_frc.F: velocity through a river face (dir 0: the u face
// between i-1 and i; dir 1: the v face between j-1 and j) of column ij:
// riv_vol(iriver)*(riv_flx - 10*iriver) / (dn * riv_depth), dn = dn_u / dm_v
// for the momentum (pre_step3d4S.F:497-501) or 1 for the tracer flux
// (compute_horiz_tracer_fluxes.h:223-226); riv_depth is the mean water depth
// of the two cells. ----
__device__ __forceinline__ double river_velocity(const Dev& d, int dir, long ij, bool with_dn) {
  const Fields& F = d.f;
  const Bounds& b = d.b;
  const long s = dir == 0 ? 1 : b.nx2, wN = (long)b.N * b.n2;
  const double flx = dir == 0 ? F.riv_uflx[ij] : F.riv_vflx[ij];
  const int iriver = (int)lround(flx / 10);
  const double riv_depth = 0.5 * (F.z_w[ij - s + wN] - F.z_w[ij - s] + F.z_w[ij + wN] - F.z_w[ij]);
  const double q = F.riv_vol[iriver - 1] * (flx - 10 * iriver);
  return with_dn ? q / ((dir == 0 ? F.dn_u[ij] : F.dm_v[ij]) * riv_depth) : q / riv_depth;
}
// compute_horiz_tracer_fluxes.h:217-246: the tracer flux through a river
// face at level k carries the river's concentration riv_trc(iriver, itrc)
__device__ __forceinline__ void river_tracer_flux(const Dev& d, int dir, int i, int j, int k, int itrc, double& Fl) {
  const Fields& F = d.f;
  const Bounds& b = d.b;
  const long ij = IJ(b, i, j);
  const double flx = dir == 0 ? F.riv_uflx[ij] : F.riv_vflx[ij];
  if (!(fabs(flx) > 1e-3)) return;
  const long s = dir == 0 ? 1 : b.nx2, o = ij + (long)(k - 1) * b.n2;
  const int iriver = (int)lround(flx / 10);
  const double vel = river_velocity(d, dir, ij, false);
  Fl = F.riv_trc[(iriver - 1) + (long)(itrc - 1) * d.p.nriv] * 0.5 * (F.Hz[o - s] + F.Hz[o]) * vel;
}

// ---- horizontal tracer fluxes at one face ----
// Written over an accessor (t, umask, vmask, FlxU, FlxV at one level); the
// kernels stage the block's window in LDS (AccTL).  FX at u-point m (row j):
// elementary differences FXel(q) for q=m-1..m+1, clamped at closed edges
// (FX(istr-1)=FX(istr), FX(iend+2)=FX(iend+1)).
struct AccTL {
  const double *T, *UM, *VM, *FU, *FV;  // LDS windows, row-major kUVW, origin (ib, jb)
  int ib, jb;
  __device__ __forceinline__ int at(int i, int j) const { return (i - ib) + (j - jb) * kUVW; }
  __device__ __forceinline__ double t(int i, int j) const { return T[at(i, j)]; }
  __device__ __forceinline__ double um(int i, int j) const { return UM[at(i, j)]; }
  __device__ __forceinline__ double vm(int i, int j) const { return VM[at(i, j)]; }
  __device__ __forceinline__ double fu(int i, int j) const { return FU[at(i, j)]; }
  __device__ __forceinline__ double fv(int i, int j) const { return FV[at(i, j)]; }
};
// The same windows as a ring of kRingH rows (j-marching kernels): row j sits
// in slot (j - jb) mod kRingH, jb the first window row of the block's chunk.
constexpr int kRingH = 8;
struct AccTR {
  const double *T, *UM, *VM, *FU, *FV;
  int ib, jb;
  __device__ __forceinline__ int at(int i, int j) const { return (i - ib) + ((j - jb) & (kRingH - 1)) * kUVW; }
  __device__ __forceinline__ double t(int i, int j) const { return T[at(i, j)]; }
  __device__ __forceinline__ double um(int i, int j) const { return UM[at(i, j)]; }
  __device__ __forceinline__ double vm(int i, int j) const { return VM[at(i, j)]; }
  __device__ __forceinline__ double fu(int i, int j) const { return FU[at(i, j)]; }
  __device__ __forceinline__ double fv(int i, int j) const { return FV[at(i, j)]; }
};
template <class A>
__device__ __forceinline__ double tracer_fx(const Bounds& b, const A& a, int m, int j, bool upstream) {
  const int lo = b.west_edge ? b.istr : -1000000, hi = b.east_edge ? b.iend + 1 : 1000000;
  double el[3];
  for (int q = 0; q < 3; q++) {
    const int p = iclamp(m - 1 + q, lo, hi);
    el[q] = (a.t(p, j) - a.t(p - 1, j)) * a.um(p, j);
  }
  const double Fl = a.fu(m, j);
  if (upstream) {
    const double cm = el[1] - el[0], c0 = el[2] - el[1];   // curv(m-1), curv(m)
    return 0.5 * (a.t(m, j) + a.t(m - 1, j)) * Fl - 0.1666666666666666 * (cm * fmax0(Fl) + c0 * fmin0(Fl));
  }
  const double gm = 0.5 * (el[1] + el[0]), g0 = 0.5 * (el[2] + el[1]);  // grad(m-1), grad(m)
  return 0.5 * (a.t(m, j) + a.t(m - 1, j) - 0.3333333333333333 * (g0 - gm)) * Fl;
}
template <class A>
__device__ __forceinline__ double tracer_fe(const Bounds& b, const A& a, int i, int m, bool upstream) {
  const int lo = b.south_edge ? b.jstr : -1000000, hi = b.north_edge ? b.jend + 1 : 1000000;
  double el[3];
  for (int q = 0; q < 3; q++) {
    const int p = iclamp(m - 1 + q, lo, hi);
    el[q] = (a.t(i, p) - a.t(i, p - 1)) * a.vm(i, p);
  }
  const double Fl = a.fv(i, m);
  if (upstream) {
    const double cm = el[1] - el[0], c0 = el[2] - el[1];
    return 0.5 * (a.t(i, m) + a.t(i, m - 1)) * Fl - 0.1666666666666666 * (cm * fmax0(Fl) + c0 * fmin0(Fl));
  }
  const double gm = 0.5 * (el[1] + el[0]), g0 = 0.5 * (el[2] + el[1]);
  return 0.5 * (a.t(i, m) + a.t(i, m - 1) - 0.3333333333333333 * (g0 - gm)) * Fl;
}

// Stage the (kUVW x kUVH) window around a block's 64x4 tile: the level-k
// fluxes and the masks (once), then per tracer the tracer field.
struct TracerWin {
  double T[kUVN], UM[kUVN], VM[kUVN], FU[kUVN], FV[kUVN];
};
__device__ __forceinline__ void tracer_win_fill(const Bounds& b, const Fields& F, TracerWin& W, int ib, int jb,
                                                long kk, const double* T) {
  for (int q = threadIdx.x + kBX * threadIdx.y; q < kUVN; q += kBX * kBY) {
    const int i = ib + q % kUVW, j = jb + q / kUVW;
    if (i < -1 || i > b.Lm + 2 || j < -1 || j > b.Mm + 2) continue;  // never read
    const long o = IJ(b, i, j);
    if (T) {
      W.T[q] = T[o + kk];
    } else {
      W.UM[q] = F.umask[o];
      W.VM[q] = F.vmask[o];
      W.FU[q] = F.FlxU[o + kk];
      W.FV[q] = F.FlxV[o + kk];
    }
  }
}

// grid of the j-marching per-level kernels: 64-wide strips x chunks of jc
// rows (marched 4 rows at a time) x levels
inline dim3 grid3_jc(const Range& r, int nk, int jc) {
  int ni = r.i1 - tile_i0(r.i0) + 1, nj = r.j1 - r.j0 + 1;
  if (ni < 1) ni = 1;
  if (nj < 1) nj = 1;
  return dim3((ni + kBX - 1) / kBX, (nj + jc - 1) / jc, nk);
}
// grid of the per-level horizontal kernels with 64 x ty tiles (Params::h_ty)
inline dim3 grid3_ty(const Range& r, int nk, int ty) {
  int ni = r.i1 - tile_i0(r.i0) + 1, nj = r.j1 - r.j0 + 1;
  if (ni < 1) ni = 1;
  if (nj < 1) nj = 1;
  return dim3((ni + kBX - 1) / kBX, (nj + ty - 1) / ty, nk);
}

// ---- horizontal momentum r.h.s. (Coriolis + advection) at (i,j,k) ----
struct UVBounds {
  int u_imin, u_imax, v_jmin, v_jmax;   // uxx / vee extrapolation ranges
  int e_jmin, e_jmax, x_imin, x_imax;   // uee / vxx extrapolation ranges
};
__host__ inline UVBounds uv_bounds(const Bounds& b) {
  UVBounds r;
  if (!b.ew_periodic) {
    r.u_imin = b.west_edge ? b.istrU : b.istrU - 1; r.u_imax = b.east_edge ? b.iend : b.iend + 1;
    r.x_imin = b.west_edge ? b.istr : b.istr - 1;   r.x_imax = b.east_edge ? b.iend : b.iend + 1;
  } else {
    r.u_imin = r.x_imin = b.istr - 1; r.u_imax = r.x_imax = b.iend + 1;
  }
  if (!b.ns_periodic) {
    r.v_jmin = b.south_edge ? b.jstrV : b.jstrV - 1; r.v_jmax = b.north_edge ? b.jend : b.jend + 1;
    r.e_jmin = b.south_edge ? b.jstr : b.jstr - 1;   r.e_jmax = b.north_edge ? b.jend : b.jend + 1;
  } else {
    r.v_jmin = r.e_jmin = b.jstr - 1; r.v_jmax = r.e_jmax = b.jend + 1;
  }
  return r;
}

// The UV advection fragments are written once over an accessor A giving
// u, v (time level nrhs) and FlxU, FlxV at level k: AccG reads HBM, AccL a
// block's LDS window (k_uv_horiz).  Identical arithmetic either way.
struct AccG {
  const double *U, *V, *FU, *FV;
  long kk;
  int nx2;
  __device__ __forceinline__ long at(int i, int j) const { return (long)(i + 1) + (long)(j + 1) * nx2 + kk; }
  __device__ __forceinline__ double u(int i, int j) const { return U[at(i, j)]; }
  __device__ __forceinline__ double v(int i, int j) const { return V[at(i, j)]; }
  __device__ __forceinline__ double fu(int i, int j) const { return FU[at(i, j)]; }
  __device__ __forceinline__ double fv(int i, int j) const { return FV[at(i, j)]; }
};
struct AccL {
  const double *U, *V, *FU, *FV;   // LDS windows, row-major kUVW
  int ib, jb;                      // global (i,j) of window element 0
  __device__ __forceinline__ int at(int i, int j) const { return (i - ib) + (j - jb) * kUVW; }
  __device__ __forceinline__ double u(int i, int j) const { return U[at(i, j)]; }
  __device__ __forceinline__ double v(int i, int j) const { return V[at(i, j)]; }
  __device__ __forceinline__ double fu(int i, int j) const { return FU[at(i, j)]; }
  __device__ __forceinline__ double fv(int i, int j) const { return FV[at(i, j)]; }
};

template <class A>
__device__ __forceinline__ double uxx_at(const A& a, int m, int j, const UVBounds& r) {
  m = iclamp(m, r.u_imin, r.u_imax);
  return a.u(m - 1, j) - 2.0 * a.u(m, j) + a.u(m + 1, j);
}
template <class A>
__device__ __forceinline__ double Huxx_at(const A& a, int m, int j, const UVBounds& r) {
  m = iclamp(m, r.u_imin, r.u_imax);
  return a.fu(m - 1, j) - 2.0 * a.fu(m, j) + a.fu(m + 1, j);
}
template <class A>
__device__ __forceinline__ double vee_at(const A& a, int i, int m, const UVBounds& r) {
  m = iclamp(m, r.v_jmin, r.v_jmax);
  return a.v(i, m - 1) - 2.0 * a.v(i, m) + a.v(i, m + 1);
}
template <class A>
__device__ __forceinline__ double Hvee_at(const A& a, int i, int m, const UVBounds& r) {
  m = iclamp(m, r.v_jmin, r.v_jmax);
  return a.fv(i, m - 1) - 2.0 * a.fv(i, m) + a.fv(i, m + 1);
}
template <class A>
__device__ __forceinline__ double uee_at(const A& a, int i, int m, const UVBounds& r) {
  m = iclamp(m, r.e_jmin, r.e_jmax);
  return a.u(i, m - 1) - 2.0 * a.u(i, m) + a.u(i, m + 1);
}
template <class A>
__device__ __forceinline__ double vxx_at(const A& a, int m, int j, const UVBounds& r) {
  m = iclamp(m, r.x_imin, r.x_imax);
  return a.v(m - 1, j) - 2.0 * a.v(m, j) + a.v(m + 1, j);
}

// UFx at rho-point (m,j): diagonal xi-flux of u-momentum
template <class A>
__device__ __forceinline__ double adv_UFx(const A& a, int m, int j, const UVBounds& r, bool up) {
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  const double ux0 = uxx_at(a, m, j, r), ux1 = uxx_at(a, m + 1, j, r);
  const double Hx0 = Huxx_at(a, m, j, r), Hx1 = Huxx_at(a, m + 1, j, r);
  if (up) {
    const double cff = a.fu(m, j) + a.fu(m + 1, j) - delta * (Hx0 + Hx1);
    return 0.25 * (cff * (a.u(m, j) + a.u(m + 1, j)) - gamma * (fmax0(cff) * ux0 + fmin0(cff) * ux1));
  }
  return 0.25 * (a.u(m, j) + a.u(m + 1, j) - delta * (ux0 + ux1)) * (a.fu(m, j) + a.fu(m + 1, j) - delta * (Hx0 + Hx1));
}
// VFe at rho-point (i,m)
template <class A>
__device__ __forceinline__ double adv_VFe(const A& a, int i, int m, const UVBounds& r, bool up) {
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  const double ve0 = vee_at(a, i, m, r), ve1 = vee_at(a, i, m + 1, r);
  const double He0 = Hvee_at(a, i, m, r), He1 = Hvee_at(a, i, m + 1, r);
  if (up) {
    const double cff = a.fv(i, m) + a.fv(i, m + 1) - delta * (He0 + He1);
    return 0.25 * (cff * (a.v(i, m) + a.v(i, m + 1)) - gamma * (fmax0(cff) * ve0 + fmin0(cff) * ve1));
  }
  return 0.25 * (a.v(i, m) + a.v(i, m + 1) - delta * (ve0 + ve1)) * (a.fv(i, m) + a.fv(i, m + 1) - delta * (He0 + He1));
}
// UFe at psi-point (i,m)
template <class A>
__device__ __forceinline__ double adv_UFe(const A& a, int i, int m, const UVBounds& r, bool up) {
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  const double Hv0 = a.fv(i - 1, m) - 2.0 * a.fv(i, m) + a.fv(i + 1, m);       // Hvxx(i,m)
  const double Hvm = a.fv(i - 2, m) - 2.0 * a.fv(i - 1, m) + a.fv(i, m);       // Hvxx(i-1,m)
  const double um1 = uee_at(a, i, m - 1, r), u0 = uee_at(a, i, m, r);
  if (up) {
    const double cff = a.fv(i, m) + a.fv(i - 1, m) - delta * (Hv0 + Hvm);
    return 0.25 * (cff * (a.u(i, m) + a.u(i, m - 1)) - gamma * (fmax0(cff) * um1 + fmin0(cff) * u0));
  }
  return 0.25 * (a.u(i, m) + a.u(i, m - 1) - delta * (u0 + um1)) * (a.fv(i, m) + a.fv(i - 1, m) - delta * (Hv0 + Hvm));
}
// VFx at psi-point (m,j)
template <class A>
__device__ __forceinline__ double adv_VFx(const A& a, int m, int j, const UVBounds& r, bool up) {
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  const double Hu0 = a.fu(m, j - 1) - 2.0 * a.fu(m, j) + a.fu(m, j + 1);       // Huee(m,j)
  const double Hum = a.fu(m, j - 2) - 2.0 * a.fu(m, j - 1) + a.fu(m, j);       // Huee(m,j-1)
  const double vm1 = vxx_at(a, m - 1, j, r), v0 = vxx_at(a, m, j, r);
  if (up) {
    const double cff = a.fu(m, j) + a.fu(m, j - 1) - delta * (Hu0 + Hum);
    return 0.25 * (cff * (a.v(m, j) + a.v(m - 1, j)) - gamma * (fmax0(cff) * vm1 + fmin0(cff) * v0));
  }
  return 0.25 * (a.v(m, j) + a.v(m - 1, j) - delta * (v0 + vm1)) * (a.fu(m, j) + a.fu(m, j - 1) - delta * (Hu0 + Hum));
}

// Full horizontal r.h.s. at (i,j,k): Coriolis first, then advection, with the
// two accumulation steps into ru/rv kept in the reference's order.
template <class A>
__device__ __forceinline__ void uv_horiz_rhs(const Dev& d, const A& a, int i, int j, int k, const UVBounds& r,
                                             bool up) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long kk = (long)(k - 1) * b.n2;
  const long o = IJ(b, i, j) + kk;
  // Coriolis factor cff = 0.5*Hz*fomn at rho point (m,n), plus the CURVGRID
  // curvature terms (compute_horiz_rhs_uv_terms.h:4-12)
  // (UV_COR: fomn; CURVGRID && UV_ADV: curvature; either alone is allowed)
  const bool ucor = d.p.uv_cor, curv = d.p.curvgrid, adv = d.p.uv_adv, corb = ucor || curv;
  auto cor = [&](int m, int n, long oo) {
    const long mn = IJ(b, m, n);
    if (curv) {
      const double ct = 0.5 * ((a.v(m, n) + a.v(m, n + 1)) * F.dndx[mn] - (a.u(m, n) + a.u(m + 1, n)) * F.dmde[mn]);
      return 0.5 * F.Hz[oo] * (ucor ? F.fomn[mn] + ct : ct);
    }
    return 0.5 * F.Hz[oo] * (F.fomn[mn]);
  };
  if (i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend) {
    double ru = F.ru[o];
    if (corb) {  // Coriolis UFx at i and i-1: UFx=cff*(v(j)+v(j+1))
      const double c0 = cor(i, j, o);
      const double c1 = cor(i - 1, j, o - 1);
      const double U0 = c0 * (a.v(i, j) + a.v(i, j + 1)), U1 = c1 * (a.v(i - 1, j) + a.v(i - 1, j + 1));
      ru = ru + 0.5 * (U0 + U1);
    }
    if (adv)
      ru = ru - adv_UFx(a, i, j, r, up) + adv_UFx(a, i - 1, j, r, up) - adv_UFe(a, i, j + 1, r, up) +
           adv_UFe(a, i, j, r, up);
    F.ru[o] = ru;
  }
  if (i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend) {
    double rv = F.rv[o];
    if (corb) {
      const double c0 = cor(i, j, o);
      const double c1 = cor(i, j - 1, o - b.nx2);
      const double V0 = c0 * (a.u(i, j) + a.u(i + 1, j)), V1 = c1 * (a.u(i, j - 1) + a.u(i + 1, j - 1));
      rv = rv - 0.5 * (V0 + V1);
    }
    if (adv)
      rv = rv - adv_VFx(a, i + 1, j, r, up) + adv_VFx(a, i, j, r, up) - adv_VFe(a, i, j, r, up) +
           adv_VFe(a, i, j - 1, r, up);
    F.rv[o] = rv;
  }
}

// uv_horiz_rhs without CURVGRID on values the caller loaded ahead (ru, rv,
// Hz at (i,j), (i-1,j), (i,j-1) and fomn at the same points): the kernel
// issues these loads together with its window loads (one memory wait per
// block).  Same arithmetic as uv_horiz_rhs.
struct UVPre {
  double ru, rv, hz0, hzx, hzy, f0, fx, fy;
};
template <class A>
__device__ __forceinline__ void uv_horiz_rhs_pre(const Dev& d, const A& a, int i, int j, long o, const UVPre& p,
                                                 const UVBounds& r, bool up) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const bool ucor = d.p.uv_cor, adv = d.p.uv_adv;
  if (i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend) {
    double ru = p.ru;
    if (ucor) {
      const double c0 = 0.5 * p.hz0 * (p.f0);
      const double c1 = 0.5 * p.hzx * (p.fx);
      const double U0 = c0 * (a.v(i, j) + a.v(i, j + 1)), U1 = c1 * (a.v(i - 1, j) + a.v(i - 1, j + 1));
      ru = ru + 0.5 * (U0 + U1);
    }
    if (adv)
      ru = ru - adv_UFx(a, i, j, r, up) + adv_UFx(a, i - 1, j, r, up) - adv_UFe(a, i, j + 1, r, up) +
           adv_UFe(a, i, j, r, up);
    F.ru[o] = ru;
  }
  if (i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend) {
    double rv = p.rv;
    if (ucor) {
      const double c0 = 0.5 * p.hz0 * (p.f0);
      const double c1 = 0.5 * p.hzy * (p.fy);
      const double V0 = c0 * (a.u(i, j) + a.u(i + 1, j)), V1 = c1 * (a.u(i, j - 1) + a.u(i + 1, j - 1));
      rv = rv - 0.5 * (V0 + V1);
    }
    if (adv)
      rv = rv - adv_VFx(a, i + 1, j, r, up) + adv_VFx(a, i, j, r, up) - adv_VFe(a, i, j, r, up) +
           adv_VFe(a, i, j - 1, r, up);
    F.rv[o] = rv;
  }
}

// ---- SPLINE_UV with LDS column scratch: leaves the vertical advective flux
// of u (dir 0) / v (dir 1) at w-levels in A[k], k=0..N, A[0]=A[N]=0
// (compute_vert_rhs_uv_terms.h); the r.h.s. update is rr(k) = rr(k) - A[k] +
// A[k-1] in that order (uv_rr_update).
template <bool kRing, class C>
__device__ __forceinline__ void uv_vert_flux_lds(const Dev& d, long ij, int nrhs, int dir, const C& A,
                                                 const C& B) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  if (!d.p.uv_adv) {  // no UV_ADV: no vertical advective flux (compute_vert_rhs_uv_terms.h:1)
    for (int k = 0; k <= N; k++) A[k] = 0.0;
    return;
  }
  const long n2 = b.n2;
  const long s = dir == 0 ? 1 : b.nx2;
  const double* __restrict__ Uv = (dir == 0 ? F.u : F.v) + (long)(nrhs - 1) * b.n3 + ij;
  const double* __restrict__ Hz = F.Hz + ij;
  const double* __restrict__ We = F.We + ij;
  const double* mask = dir == 0 ? F.umask : F.vmask;
  // DC(k) from the four Hz columns of rho level k (kept for the remainder loops)
  auto DCk = [&](int k) {
    const long o = (long)(k - 1) * n2;
    return 0.5625 * (Hz[o] + Hz[o - s]) - 0.0625 * (Hz[o + s] + Hz[o - 2 * s]);
  };
  double dck = DCk(1), cfk = 1.0, fcm = 2.0 * Uv[0], uk = Uv[0];
  auto fwd = [&](int k, double dc1, double uk1) {   // level k -> k+1
    const double cff = 1.0 / (2.0 * dck + dc1 * (2.0 - cfk));
    const double cf1 = cff * dck;
    const double fck = cff * (3.0 * (dck * uk1 + dc1 * uk) - dc1 * fcm);
    B[k + 1] = cf1;
    A[k] = fck;
    dck = dc1; cfk = cf1; fcm = fck; uk = uk1;
  };
  // rings hold raw loads (derived values would force the wait at prefetch)
  auto dc_of = [&](double h0, double hm, double hp, double hmm) { return 0.5625 * (h0 + hm) - 0.0625 * (hp + hmm); };
  int k0 = 1;
  if (kRing) {
    double r0[kPF], r1[kPF], r2[kPF], r3[kPF], ru[kPF];  // Hz(i), Hz(i-s), Hz(i+s), Hz(i-2s), u at level k+1
#pragma unroll
    for (int q = 0; q < kPF; q++) {
      const long o = (long)(min(2 + q, N) - 1) * n2;
      r0[q] = Hz[o]; r1[q] = Hz[o - s]; r2[q] = Hz[o + s]; r3[q] = Hz[o - 2 * s]; ru[q] = Uv[o];
    }
    for (; k0 + kPF - 1 <= N - 1; k0 += kPF) {
#pragma unroll
      for (int q = 0; q < kPF; q++) {
        const double dc1 = dc_of(r0[q], r1[q], r2[q], r3[q]), uk1 = ru[q];
        const long o = (long)(min(k0 + q + 1 + kPF, N) - 1) * n2;
        r0[q] = Hz[o]; r1[q] = Hz[o - s]; r2[q] = Hz[o + s]; r3[q] = Hz[o - 2 * s]; ru[q] = Uv[o];
        fwd(k0 + q, dc1, uk1);
      }
    }
  }
#pragma unroll 4
  for (int k = k0; k <= N - 1; k++) fwd(k, DCk(k + 1), Uv[(long)k * n2]);
  double fc1 = (2.0 * Uv[(long)(N - 1) * n2] - fcm) / (1.0 - cfk);  // FC(N)
  const double m1 = mask[ij + s], m0 = mask[ij - s];
  auto wbr = [&](double w0, double wm, double wp, double wmm) {
    return w0 + wm - 0.125 * ((wp - w0) * m1 - (wm - wmm) * m0);
  };
  auto wflux = [&](int k) {
    const long w = (long)k * n2;
    return wbr(We[w], We[w - s], We[w + s], We[w - 2 * s]);
  };
  auto bwd = [&](int k, double wf) {
    const double fck = A[k] - B[k + 1] * fc1;
    A[k] = fck * 0.5 * wf;
    fc1 = fck;
  };
  int k1 = N - 1;
  if (kRing) {
    double w0[kPF], w1[kPF], w2[kPF], w3[kPF];
#pragma unroll
    for (int q = 0; q < kPF; q++) {
      const long w = (long)max(N - 1 - q, 1) * n2;
      w0[q] = We[w]; w1[q] = We[w - s]; w2[q] = We[w + s]; w3[q] = We[w - 2 * s];
    }
    for (; k1 - kPF + 1 >= 1; k1 -= kPF) {
#pragma unroll
      for (int q = 0; q < kPF; q++) {
        const double wf = wbr(w0[q], w1[q], w2[q], w3[q]);
        const long w = (long)max(k1 - q - kPF, 1) * n2;
        w0[q] = We[w]; w1[q] = We[w - s]; w2[q] = We[w + s]; w3[q] = We[w - 2 * s];
        bwd(k1 - q, wf);
      }
    }
  }
#pragma unroll 4
  for (int k = k1; k >= 1; k--) bwd(k, wflux(k));
  A[0] = 0.0;
  A[N] = 0.0;
}
// ---- SPLINE_UV flux of a u (dir 0) / v (dir 1) column for a compile-time
// depth NN: FC in registers A[0..NN], CF in one LDS slot B; on exit A[k] is
// the vertical advective flux at w-level k (A[0] = A[N] = 0), exactly as
// uv_vert_flux_lds leaves it.  Used by k_uv1_reg and k_pre_uv_reg. ----
template <int NN>
__device__ __forceinline__ void uv_spline_reg(const Dev& d, long ij, int nrhs, int dir, double (&A)[NN + 1],
                                              const ColLds& B) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  constexpr int N = NN;
  const long n2 = b.n2;
  const long s = dir == 0 ? 1 : b.nx2;
  if (!d.p.uv_adv) {
#pragma unroll
    for (int k = 0; k <= N; k++) A[k] = 0.0;
  } else {
    const double* __restrict__ Uv = (dir == 0 ? F.u : F.v) + (long)(nrhs - 1) * b.n3 + ij;
    const double* __restrict__ Hz = F.Hz + ij;
    const double* __restrict__ We = F.We + ij;
    const double* mask = dir == 0 ? F.umask : F.vmask;
    auto DCk = [&](int k) {
      const long o = (long)(k - 1) * n2;
      return 0.5625 * (Hz[o] + Hz[o - s]) - 0.0625 * (Hz[o + s] + Hz[o - 2 * s]);
    };
    double dck = DCk(1), cfk = 1.0, fcm = 2.0 * Uv[0], uk = Uv[0];
#pragma unroll
    for (int k = 1; k <= N - 1; k++) {
      const double dc1 = DCk(k + 1), uk1 = Uv[(long)k * n2];
      const double cff = 1.0 / (2.0 * dck + dc1 * (2.0 - cfk));
      const double cf1 = cff * dck;
      const double fck = cff * (3.0 * (dck * uk1 + dc1 * uk) - dc1 * fcm);
      B[k + 1] = cf1;
      A[k] = fck;
      dck = dc1; cfk = cf1; fcm = fck; uk = uk1;
      ROMS_LEVEL_FENCE_AT(k);
    }
    double fc1 = (2.0 * Uv[(long)(N - 1) * n2] - fcm) / (1.0 - cfk);  // FC(N)
    const double m1 = mask[ij + s], m0 = mask[ij - s];
#pragma unroll
    for (int k = N - 1; k >= 1; k--) {
      const long w = (long)k * n2;
      const double wf = We[w] + We[w - s] - 0.125 * ((We[w + s] - We[w]) * m1 - (We[w - s] - We[w - 2 * s]) * m0);
      const double fck = A[k] - B[k + 1] * fc1;
      A[k] = fck * 0.5 * wf;
      fc1 = fck;
      ROMS_LEVEL_FENCE_AT(k);
    }
    A[0] = 0.0;
    A[N] = 0.0;
  }
}

template <class C>
__device__ __forceinline__ double uv_rr_update(double r, const C& A, int k) {
  return k == 1 ? r - A[1] : r - A[k] + A[k - 1];
}

}  // namespace roms
