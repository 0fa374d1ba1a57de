// k_iso.hip -- ADV_ISONEUTRAL: the rotated (isoneutral) biharmonic tracer
// operator with SW_TRIADS and STABILIZE (step3d_t_ISO.F:15-18 defines both
// with it) and its inputs:
//   dRdx, dRde    prsgrd.F:307-338, 423-453, corrector stage (nrhs == 3)
//   diff3u/v,     step3d_uv2.F:572-575, 616-619, 622-697, from the corrected
//   idRz          u,v(nnew), before the river faces are set
//   LapT, t(nnew) step3d_t_ISO.F:253-846, between the horizontal advection
//                 (centred, no UPSTREAM_TS: step3d_t_ISO.F:4-6) and the
//                 vertical part, whose implicit diffusion adds Akz
//                 (step3d_t_ISO.F:1049-1065)
//
// The reference walks k recursively through two vertical slices (k1/k2) of
// FSC, dTdz, dTdx, dTde so that a tile's scratch stays 2-D.  With 288 GB of
// HBM the device keeps them as full 3-D fields instead: every (i,j,k) is
// then independent and each phase is one level-parallel launch (grad ->
// Laplacian -> edges -> grad -> update), each cell evaluating the same
// expressions in the reference's order, so the result is the recursive
// form's bit for bit (checked against oracle/oracle_iso.c, which keeps the
// two-slice form).  The switch is off in every BASELINE configuration, so
// these kernels are written for clarity over speed: plain per-cell loads
// through L2, no LDS staging.
//
// The reference reads two unset scratch cells at physical edges (prsgrd's
// rx(istr-1) for dRdx(istr), rx(iend+2) for dRdx(iend+1), and the same for
// dRde); both here and in the oracle the edge extrapolation is continued.
#include "roms_dev.h"

namespace roms {

namespace {

constexpr double kIsoGamma = 0.0833333333333;   // step3d_uv2.F:76
constexpr double kAlphaMax = 2.;                // step3d_uv2.F:75

__device__ __forceinline__ bool in_rng(const Range& r, int i, int j) {
  return i >= r.i0 && i <= r.i1 && j >= r.j0 && j <= r.j1;
}
Range span(const Range& a, const Range& b) {
  return Range{a.i0 < b.i0 ? a.i0 : b.i0, a.i1 > b.i1 ? a.i1 : b.i1, a.j0 < b.j0 ? a.j0 : b.j0,
               a.j1 > b.j1 ? a.j1 : b.j1};
}

// prsgrd's elementary density difference rx at face m (between m-1 and m)
// along xi (xi = true) or eta, masked, extrapolated past physical edges
// (prsgrd.F:234-268, 347-381): the face index is clamped to [lo, hi]
__device__ __forceinline__ double iso_rx(const Dev& d, bool xi, int i, int j, long kk, int lo, int hi) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  if (xi) i = iclamp(i, lo, hi);
  else j = iclamp(j, lo, hi);
  const long o = IJ(b, i, j), om = xi ? IJ(b, i - 1, j) : IJ(b, i, j - 1);
  const double msk = xi ? F.umask[o] : F.vmask[o];
  if (d.p.nonlin_eos) {   // SPLIT_EOS: adiabatic difference
    const double dpth = -0.5 * (F.z_r[o + kk] + F.z_r[om + kk]);
    return (F.rho1[o + kk] - F.rho1[om + kk] + (F.qp1[o + kk] - F.qp1[om + kk]) * dpth * (1.0 - d.p.qp2 * dpth)) * msk;
  }
  return (F.rho[o + kk] - F.rho[om + kk]) * msk;
}

// dRdx over Rx, dRde over Re, one lane per (i,j,k)
__global__ void __launch_bounds__(256) k_iso_slopes(Dev d, Range R, Range Rx, Range Re, int xlo, int xhi, int ylo,
                                                    int yhi) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int k = 1 + (int)bI.z;
  const long kk = (long)(k - 1) * b.n2, o = IJ(b, i, j);
  const double r0g = d.p.rho0 / d.p.g;
  if (in_rng(Rx, i, j)) {
    const long om = IJ(b, i - 1, j);
    const double fs = F.f[o] + F.f[om];
    F.dRdx[o + kk] = 0.5 * (F.pm[o] + F.pm[om]) *
                      (r0g * 0.25 * (fs * fs) * (F.z_r[o + kk] - F.z_r[om + kk]) -
                       0.5 * iso_rx(d, true, i, j, kk, xlo, xhi) -
                       0.25 * (iso_rx(d, true, i - 1, j, kk, xlo, xhi) + iso_rx(d, true, i + 1, j, kk, xlo, xhi)));
  }
  if (in_rng(Re, i, j)) {
    const long om = IJ(b, i, j - 1);
    const double fs = F.f[o] + F.f[om];
    F.dRde[o + kk] = 0.5 * (F.pn[o] + F.pn[om]) *
                      (r0g * 0.25 * (fs * fs) * (F.z_r[o + kk] - F.z_r[om + kk]) -
                       0.5 * iso_rx(d, false, i, j, kk, ylo, yhi) -
                       0.25 * (iso_rx(d, false, i, j - 1, kk, ylo, yhi) + iso_rx(d, false, i, j + 1, kk, ylo, yhi)));
  }
}

// diff3u over Ru, diff3v over Rv, idRz over the interior at w-levels 1..N-1
__global__ void __launch_bounds__(256) k_iso_diff3(Dev d, Range R, Range Ru, Range Rv, int nnew) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, k = 1 + (int)bI.z;
  const long n2 = b.n2, kk = (long)(k - 1) * n2, o = IJ(b, i, j);
  if (in_rng(Ru, i, j))
    F.diff3u[o + kk] = sqrt(kIsoGamma * fabs(F.u[(long)(nnew - 1) * b.n3 + kk + o]) * F.dm_u[o]) * F.dm_u[o];
  if (in_rng(Rv, i, j))
    F.diff3v[o + kk] = sqrt(kIsoGamma * fabs(F.v[(long)(nnew - 1) * b.n3 + kk + o]) * F.dn_v[o]) * F.dn_v[o];
  if (k <= N - 1 && i >= b.istr && i <= b.iend && j >= b.jstr && j <= b.jend) {
    const long k1 = kk + n2;   // level k+1
    const double r0g = d.p.rho0 / d.p.g;
    double dRz;
    if (d.p.nonlin_eos) {
      const double dpth = -0.5 * (F.z_r[o + k1] + F.z_r[o + kk]);
      dRz = F.rho1[o + kk] - F.rho1[o + k1] + (F.qp1[o + kk] - F.qp1[o + k1]) * dpth * (1. - 2. * d.p.qp2 * dpth);
    } else {
      dRz = F.rho[o + kk] - F.rho[o + k1];
    }
    const double fc = F.f[o];
    dRz = dmax(dRz, 0.) + r0g * (fc * fc) * (F.z_r[o + k1] - F.z_r[o + kk]);
    const long oe = IJ(b, i + 1, j), on = IJ(b, i, j + 1);
    const double* X = F.dRdx;
    const double* E = F.dRde;
    const double dRx_max =
        dmax(dmax(F.dm_u[o] * dmax(fabs(X[o + kk]), fabs(X[o + k1])), F.dm_u[oe] * dmax(fabs(X[oe + kk]), fabs(X[oe + k1]))),
             dmax(F.dn_v[o] * dmax(fabs(E[o + kk]), fabs(E[o + k1])), F.dn_v[on] * dmax(fabs(E[on + kk]), fabs(E[on + k1]))));
    const double* zw = F.z_w + o;
    double cfs, cfb;
    if (d.p.lmd) {   // LMD_KPP / LMD_BKPP
      cfs = dmin(1., (zw[(long)N * n2] - zw[(long)k * n2]) / dmax(50., F.hbls[o]));
      cfb = dmin(1., (zw[(long)k * n2] - zw[0]) / dmax(50., F.hbbl[o]));
    } else {
      cfs = dmin(1., (zw[(long)N * n2] - zw[(long)k * n2]) / 50.);
      cfb = dmin(1., (zw[(long)k * n2] - zw[0]) / 50.);
    }
    const double cff = kAlphaMax * cfs * (2. - cfs) * cfb * (2. - cfb);
    F.idRz[o + (long)k * n2] = cff / dmax(dmax(cff * dRz, dRx_max), 1.E-33);
  }
}

// gradients of src (rho levels, stride n2): dTdz at w-levels 0..N over Rz
// (and the metric FSC = idRz*dz when fsc), dTdx over Rx, dTde over Re at
// levels 1..N (step3d_t_ISO.F:317-369, 575-617).  Grid z = kw = 0..N.
__global__ void __launch_bounds__(256) k_iso_grad(Dev d, Range R, Range Rz, Range Rx, Range Re, const double* src,
                                                  int fsc) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, kw = (int)bI.z;
  const long n2 = b.n2, o = IJ(b, i, j);
  auto S = [&](long oo, int k) { return src[oo + (long)(k - 1) * n2]; };
  if (in_rng(Rz, i, j)) {
    const int kz = kw == 0 ? 1 : (kw == N ? N - 1 : kw);   // k == N copies the slice below
    F.iso_dTdz[o + (long)kw * n2] = F.idRz[o + (long)kz * n2] * (S(o, kz + 1) - S(o, kz));
    if (fsc)
      F.iso_FSC[o + (long)kw * n2] =
          (kw == 0 || kw == N) ? 0. : F.idRz[o + (long)kw * n2] * (F.z_r[o + (long)kw * n2] - F.z_r[o + (long)(kw - 1) * n2]);
  }
  if (kw >= 1) {
    const int k = kw;
    const long kk = (long)(k - 1) * n2;
    if (in_rng(Rx, i, j)) {
      const long om = IJ(b, i - 1, j);
      F.iso_dTdx[o + kk] = 0.5 * (F.pm[o] + F.pm[om]) * (S(o, k) - S(om, k)) * F.umask[o];
    }
    if (in_rng(Re, i, j)) {
      const long om = IJ(b, i, j - 1);
      F.iso_dTde[o + kk] = 0.5 * (F.pn[o] + F.pn[om]) * (S(o, k) - S(om, k)) * F.vmask[o];
    }
  }
}

// the rotated flux through the u face at (i,j) of level k (step3d_t_ISO.F:374-388, 620-633)
__device__ __forceinline__ double iso_fx(const Dev& d, int i, int j, int k) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long n2 = b.n2, o = IJ(b, i, j), om = IJ(b, i - 1, j), kk = (long)(k - 1) * n2;
  const double* Z = F.iso_dTdz;
  const long wl = (long)(k - 1) * n2, wu = (long)k * n2;   // dTdz slices k1 (k-1/2), k2 (k+1/2)
  const double r = F.dRdx[o + kk];
  return F.diff3u[o + kk] * 0.5 * (F.Hz[o + kk] + F.Hz[om + kk]) * F.dn_u[o] *
         (F.iso_dTdx[o + kk] - 0.5 * (dmin(r, 0.) * (Z[om + wl] + Z[o + wu]) + dmax(r, 0.) * (Z[om + wu] + Z[o + wl])));
}
__device__ __forceinline__ double iso_fe(const Dev& d, int i, int j, int k) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long n2 = b.n2, o = IJ(b, i, j), om = IJ(b, i, j - 1), kk = (long)(k - 1) * n2;
  const double* Z = F.iso_dTdz;
  const long wl = (long)(k - 1) * n2, wu = (long)k * n2;
  const double r = F.dRde[o + kk];
  return F.diff3v[o + kk] * 0.5 * (F.Hz[o + kk] + F.Hz[om + kk]) * F.dm_v[o] *
         (F.iso_dTde[o + kk] - 0.5 * (dmin(r, 0.) * (Z[om + wl] + Z[o + wu]) + dmax(r, 0.) * (Z[om + wu] + Z[o + wl])));
}

// SW_TRIADS: sumX*wgt(idx) + sumE*wgt(ide) at (i,j) between levels k and
// k+1 (step3d_t_ISO.F:411-485, 722-805), terms added in the reference's order
__device__ __forceinline__ double iso_triads(const Dev& d, int i, int j, int k) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long n2 = b.n2, o = IJ(b, i, j), oe = IJ(b, i + 1, j), on = IJ(b, i, j + 1);
  const long k1 = (long)(k - 1) * n2, k2 = (long)k * n2;
  const double* X = F.dRdx;
  const double* E = F.dRde;
  const double *u3 = F.diff3u, *v3 = F.diff3v, *Tx = F.iso_dTdx, *Te = F.iso_dTde;
  const double tz = F.iso_dTdz[o + (long)k * n2];
  double sumX = 0., sumE = 0.;
  int idx = 0, ide = 0;
  if (X[o + k1] < 0.) { sumX = u3[o + k1] * X[o + k1] * (X[o + k1] * tz - Tx[o + k1]); idx = 1; }
  if (X[o + k2] > 0.) { sumX = sumX + u3[o + k2] * X[o + k2] * (X[o + k2] * tz - Tx[o + k2]); idx = idx + 1; }
  if (X[oe + k2] < 0.) { sumX = sumX + u3[oe + k2] * X[oe + k2] * (X[oe + k2] * tz - Tx[oe + k2]); idx = idx + 1; }
  if (X[oe + k1] > 0.) { sumX = sumX + u3[oe + k1] * X[oe + k1] * (X[oe + k1] * tz - Tx[oe + k1]); idx = idx + 1; }
  if (E[o + k1] < 0.) { sumE = v3[o + k1] * E[o + k1] * (E[o + k1] * tz - Te[o + k1]); ide = 1; }
  if (E[o + k2] > 0.) { sumE = sumE + v3[o + k2] * E[o + k2] * (E[o + k2] * tz - Te[o + k2]); ide = ide + 1; }
  if (E[on + k2] < 0.) { sumE = sumE + v3[on + k2] * E[on + k2] * (E[on + k2] * tz - Te[on + k2]); ide = ide + 1; }
  if (E[on + k1] > 0.) { sumE = sumE + v3[on + k1] * E[on + k1] * (E[on + k1] * tz - Te[on + k1]); ide = ide + 1; }
  auto wgt = [](int n) {   // step3d_t_ISO.F:121-122
    return n == 1 ? 1. : n == 2 ? 0.5 : n == 3 ? 0.3333333333333333 : n == 4 ? 0.25 : 0.;
  };
  return sumX * wgt(idx) + sumE * wgt(ide);
}

__device__ __forceinline__ double max4(double a, double b, double c, double e) { return dmax(dmax(a, b), dmax(c, e)); }

// STABILIZE with SW_TRIADS (step3d_t_ISO.F:656-695), fsc = the metric idRz*dz
__device__ __forceinline__ double iso_akz(const Dev& d, int i, int j, int k, double fsc) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long n2 = b.n2, o = IJ(b, i, j), oe = IJ(b, i + 1, j), on = IJ(b, i, j + 1);
  const long k1 = (long)(k - 1) * n2, k2 = (long)k * n2;
  const double* X = F.dRdx;
  const double* E = F.dRde;
  const double *u3 = F.diff3u, *v3 = F.diff3v;
  double a;
  a = fsc * X[o + k1];  const double s2_XLL = a * a;
  a = fsc * X[o + k2];  const double s2_XLU = a * a;
  a = fsc * X[oe + k2]; const double s2_XRU = a * a;
  a = fsc * X[oe + k1]; const double s2_XRL = a * a;
  a = fsc * E[o + k1];  const double s2_ELL = a * a;
  a = fsc * E[o + k2];  const double s2_ELU = a * a;
  a = fsc * E[on + k2]; const double s2_ERU = a * a;
  a = fsc * E[on + k1]; const double s2_ERL = a * a;
  const double cff = 2. / (F.Hz[o + k2] + F.Hz[o + k1]);
  const double cff2 = cff * cff, cffX = F.pm[o] * F.pm[o], cffE = F.pn[o] * F.pn[o];
  return 15. *
         (max4(u3[o + k1] * s2_XLL, u3[oe + k1] * s2_XRL, u3[o + k2] * s2_XLU, u3[oe + k2] * s2_XRU) +
          max4(v3[o + k1] * s2_ELL, v3[on + k1] * s2_ERL, v3[o + k2] * s2_ELU, v3[on + k2] * s2_ERU)) *
         (max4(u3[o + k1] * (cffX + cff2 * s2_XLL), u3[o + k2] * (cffX + cff2 * s2_XLU),
               u3[oe + k2] * (cffX + cff2 * s2_XRU), u3[oe + k1] * (cffX + cff2 * s2_XRL)) +
          max4(v3[o + k1] * (cffE + cff2 * s2_ELL), v3[o + k2] * (cffE + cff2 * s2_ELU),
               v3[on + k2] * (cffE + cff2 * s2_ERU), v3[on + k1] * (cffE + cff2 * s2_ERL)));
}

// the first rotated Laplacian: LapT over R, levels 1..N (step3d_t_ISO.F:373-511)
__global__ void __launch_bounds__(256) k_iso_lap(Dev d, Range R) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, k = 1 + (int)bI.z;
  const long n2 = b.n2, o = IJ(b, i, j);
  auto fsc = [&](int kw) {
    return (kw == 0 || kw == N) ? 0. : F.iso_FSC[o + (long)kw * n2] * iso_triads(d, i, j, kw);
  };
  const double fu = fsc(k), fl = fsc(k - 1);
  const double FX0 = iso_fx(d, i, j, k), FX1 = iso_fx(d, i + 1, j, k);
  const double FE0 = iso_fe(d, i, j, k), FE1 = iso_fe(d, i, j + 1, k);
  const long kk = (long)(k - 1) * n2;
  F.iso_LapT[o + kk] = (F.pm[o] * F.pn[o] * (FX1 - FX0 + FE1 - FE0) + fu - fl) / F.Hz[o + kk];
}

// LapT's lateral boundary values at physical edges (step3d_t_ISO.F:515-565):
// zero at closed walls, a copy of the first interior row at open ones.
// side 0: west/east columns over rows [j0,j1]; side 1: south/north rows over [i0,i1]
__global__ void __launch_bounds__(256) k_iso_lapbc(Dev d, int side, int lo, int hi) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int q = lo + (int)(blockIdx.x * blockDim.x + threadIdx.x), k = 1 + (int)blockIdx.y;
  if (q > hi) return;
  const long kk = (long)(k - 1) * b.n2;
  double* L = F.iso_LapT + kk;
  const int obc = d.p.obc;
  if (side == 0) {
    if (!b.ew_periodic && b.west_edge) L[IJ(b, b.istr - 1, q)] = (obc & 1) ? L[IJ(b, b.istr, q)] : 0.;
    if (!b.ew_periodic && b.east_edge) L[IJ(b, b.iend + 1, q)] = (obc & 2) ? L[IJ(b, b.iend, q)] : 0.;
  } else {
    if (!b.ns_periodic && b.south_edge) L[IJ(b, q, b.jstr - 1)] = (obc & 4) ? L[IJ(b, q, b.jstr)] : 0.;
    if (!b.ns_periodic && b.north_edge) L[IJ(b, q, b.jend + 1)] = (obc & 8) ? L[IJ(b, q, b.jend)] : 0.;
  }
}

// the second rotated Laplacian added to t(nnew) over the interior, and Akz
// at w-levels 1..N-1 (step3d_t_ISO.F:619-823); ts = t(nstp) of the tracer
__global__ void __launch_bounds__(256) k_iso_apply(Dev d, Range R, double* tn, const double* ts) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, k = 1 + (int)bI.z;
  const long n2 = b.n2, o = IJ(b, i, j);
  auto fsc = [&](int kw, bool store) {
    if (kw == 0 || kw == N) return 0.;
    const long w = (long)kw * n2;
    const double m = F.iso_FSC[o + w];
    const double akz = iso_akz(d, i, j, kw, m);
    if (store) F.Akz[o + w] = akz;
    const double cff = 2. / (F.Hz[o + w] + F.Hz[o + w - n2]);
    return -m * iso_triads(d, i, j, kw) - cff * akz * (ts[o + w] - ts[o + w - n2]);
  };
  const double fu = fsc(k, true), fl = fsc(k - 1, false);
  const double FX0 = -iso_fx(d, i, j, k), FX1 = -iso_fx(d, i + 1, j, k);
  const double FE0 = -iso_fe(d, i, j, k), FE1 = -iso_fe(d, i, j + 1, k);
  const long kk = (long)(k - 1) * n2;
  tn[o + kk] = tn[o + kk] + d.p.dt * (F.pm[o] * F.pn[o] * (FX1 - FX0 + FE1 - FE0) + fu - fl);
}

}  // namespace

bool iso_on(const Dev& d) { return d.p.iso != 0; }

void launch_iso_slopes(const Dev& d, hipStream_t s) {
  const Bounds& b = d.b;
  int imin, imax, jmin, jmax;   // prsgrd's ranges (prsgrd.F:120-152)
  if (!b.ew_periodic) {
    imin = b.west_edge ? b.istrU : b.istrU - 1;
    imax = b.east_edge ? b.iend : b.iend + 1;
  } else { imin = b.istr - 1; imax = b.iend + 1; }
  if (!b.ns_periodic) {
    jmin = b.south_edge ? b.jstrV : b.jstrV - 1;
    jmax = b.north_edge ? b.jend : b.jend + 1;
  } else { jmin = b.jstr - 1; jmax = b.jend + 1; }
  // faces past a physical edge read the extrapolated (clamped) difference;
  // elsewhere the clamp bounds are out of reach
  const int xlo = (!b.ew_periodic && b.west_edge) ? imin : -1000000, xhi = (!b.ew_periodic && b.east_edge) ? imax : 1000000;
  const int ylo = (!b.ns_periodic && b.south_edge) ? jmin : -1000000, yhi = (!b.ns_periodic && b.north_edge) ? jmax : 1000000;
  const Range Rx{b.istr, b.iendR, b.jstr, b.jend}, Re{b.istr, b.iend, b.jstr, b.jendR};
  const Range R = span(Rx, Re);
  hipLaunchKernelGGL(k_iso_slopes, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, Rx, Re, xlo, xhi, ylo, yhi);
  // step3d_uv1.F:529-532
  launch_exchange_list(d, s, ExchList{{d.f.dRdx, d.f.dRde}, {b.N, b.N}, 2});
}

void launch_iso_diff3(const Dev& d, hipStream_t s, const Tlev& t, int iu0, int iu1, int iv0, int iv1, int j0, int j1) {
  const Bounds& b = d.b;
  const Range Ru{iu0, iu1, j0, j1}, Rv{iv0, iv1, j0 > b.jstr ? j0 : b.jstr, j1};
  const Range R = span(span(Ru, Rv), Range{b.istr, b.iend, b.jstr, b.jend});
  hipLaunchKernelGGL(k_iso_diff3, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, Ru, Rv, t.nnew);
}

void launch_iso_exch_diff3(const Dev& d, hipStream_t s) {   // step3d_uv2.F:730-732
  const Bounds& b = d.b;
  launch_exchange_list(d, s, ExchList{{d.f.idRz, d.f.diff3u, d.f.diff3v}, {b.N + 1, b.N, b.N}, 3});
}

void launch_iso_tracer(const Dev& d, hipStream_t s, const Tlev& t, int itrc) {
  const Bounds& b = d.b;
  int imin, imax, jmin, jmax;   // step3d_t_ISO.F:132-161
  if (!b.ew_periodic) {
    imin = b.west_edge ? b.istr : b.istr - 1;
    imax = b.east_edge ? b.iend : b.iend + 1;
  } else { imin = b.istr - 1; imax = b.iend + 1; }
  if (!b.ns_periodic) {
    jmin = b.south_edge ? b.jstr : b.jstr - 1;
    jmax = b.north_edge ? b.jend : b.jend + 1;
  } else { jmin = b.jstr - 1; jmax = b.jend + 1; }
  const long tb = (long)(itrc - 1) * 3 * b.n3;
  const double* ts = d.f.t + (long)(t.nstp - 1) * b.n3 + tb;   // ntdf = nstp (step3d_t_ISO.F:162)
  double* tn = d.f.t + (long)(t.nnew - 1) * b.n3 + tb;
  // first Laplacian of t(nstp)
  {
    const Range Rz{imin - 1, imax + 1, jmin - 1, jmax + 1}, Rx{imin, imax + 1, jmin, jmax}, Re{imin, imax, jmin, jmax + 1};
    const Range R = span(Rz, span(Rx, Re));
    hipLaunchKernelGGL(k_iso_grad, grid3_of(R, b.N + 1), dim3(kBX, kBY), 0, s, d, R, Rz, Rx, Re, ts, 1);
    const Range RL{imin, imax, jmin, jmax};
    hipLaunchKernelGGL(k_iso_lap, grid3_of(RL, b.N), dim3(kBX, kBY), 0, s, d, RL);
    if (!b.ew_periodic && (b.west_edge || b.east_edge))
      hipLaunchKernelGGL(k_iso_lapbc, dim3((jmax - jmin + 1 + 255) / 256, b.N), dim3(256), 0, s, d, 0, jmin, jmax);
    if (!b.ns_periodic && (b.south_edge || b.north_edge))
      hipLaunchKernelGGL(k_iso_lapbc, dim3((imax - imin + 1 + 255) / 256, b.N), dim3(256), 0, s, d, 1, imin, imax);
  }
  // second Laplacian of LapT, added to t(nnew)
  {
    const Range Rz{b.istr - 1, b.iend + 1, b.jstr - 1, b.jend + 1}, Rx{b.istr, b.iend + 1, b.jstr, b.jend},
        Re{b.istr, b.iend, b.jstr, b.jend + 1};
    const Range R = span(Rz, span(Rx, Re));
    hipLaunchKernelGGL(k_iso_grad, grid3_of(R, b.N + 1), dim3(kBX, kBY), 0, s, d, R, Rz, Rx, Re,
                       (const double*)d.f.iso_LapT, 0);
    const Range RI{b.istr, b.iend, b.jstr, b.jend};
    hipLaunchKernelGGL(k_iso_apply, grid3_of(RI, b.N), dim3(kBX, kBY), 0, s, d, RI, tn, ts);
  }
}

}  // namespace roms
