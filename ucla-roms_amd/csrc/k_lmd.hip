// k_lmd.hip -- LMD/KPP vertical mixing on gfx950: lmd_vmix(tind)
// (lmd_vmix.F:5-433 + lmd_kpp.F:7-651, alfabeta.F:4-79) and the Jerlov
// short-wave fractions of lmd_swr_frac.F:13-88.
//
// Switch set: LMD_KPP + LMD_BKPP (always together: roms_gpu.h), LMD_RIMIX,
// LMD_CONVEC and LMD_NONLOCAL each switchable (Params), SMOOTH_RIG,
// SMOOTH_HBL, INT_AT_RHO_POINTS, MASKING (no LMD_DDMIX, no MERGE_OVERLAP, no
// LIMIT_UNSTABLE_ONLY, no BULK_FRC) -- Pipes_ana / Rivers_ana set all five,
// Iceland all but LMD_CONVEC.
//
// Two column passes replace the reference's four j-sweeps:
//   k_kpp_ext  over the extended range (I_EXT_RANGE x J_EXT_RANGE): one
//              descending sweep produces the raw gradient Richardson number
//              Rig(1:N-1) (lmd_vmix.F:155-168), the bulk-Richardson integral
//              FC(0:N) kept in LDS, the surface layer search kbls and hbl
//              (lmd_kpp.F:200-275), then the bottom layer bbl (:276-305);
//              alpha/beta, Bo, Bosol and ustar are stored for the second pass.
//   k_kpp_int  over the interior: the masked isotropic smoothing of hbl/bbl
//              (lmd_kpp_smooth_hbl.h) and of Rig at every level
//              (lmd_vmix.F:206-241) are evaluated per column from the 3x3
//              neighbourhood (closed-wall ghost copies become clamped
//              indices); Kv/Kt/Ks stream bottom-up through the Rig mixing,
//              the Lturb taper, the 1-2-1 vertical filter, the KPP shape
//              functions, the BKPP layer and the masked copy to Akv/Akt, with
//              no level-sized scratch at all.
// Every expression keeps the reference's operation order (FP64, no FMA
// contraction); integer powers are products, real powers pow().
#include <cmath>
#include <type_traits>

#include "k_common.h"

namespace roms {
namespace {

// lmd_kpp.F:70-95
constexpr double kRicr = 0.15, kEpssfc = 0.1, kC_Ek = 258.;
constexpr double kZeta_m = -0.2, kA_m = 1.257, kC_m = 8.360, kZeta_s = -1.0, kA_s = -28.86, kC_s = 98.96;
constexpr double kEPS = 1.E-20;
// lmd_vmix.F:58-70
constexpr double kRi0 = 0.7, kNu0m = 1.e-2, kNu0s = 1.e-2, kNuwm = 1.0e-4, kNuws = 0.1e-4, kNu0c = 0.1, kLturb = 10.;
constexpr double kPi = 3.14159265358979323;  // scalars.F:126

// LMD_DDMIX (lmd_vmix.F:95-101, 279-360): double-diffusive additions to Kt
// and Ks at a w-level from t(k), t(k+1) (T and S at tind) and z_w(k)
__device__ __forceinline__ void ddmix(double t0, double t1, double s0, double s1, double zwk, double& kt,
                                      double& ks) {
  const double A0 = +0.665157E-01, A1 = +0.170907E-01, A2 = -0.203814E-03, A3 = +0.298357E-05,
               A4 = -0.255019E-07, B0 = +0.378110E-02, B1 = -0.846960E-04, C0 = -0.678662E-05,
               D0 = +0.380374E-04, D1 = -0.933746E-06, D2 = +0.791325E-08, E0 = -0.164759E-06,
               F0 = -0.251520E-11, G0 = +0.512857E-12, H0 = -0.302285E-13, Smean = 35.0;
  const double lmd_nu = 1.5e-6, lmd_Rrho0 = 1.9, lmd_nuf = 10.0e-4, lmd_fdd = 0.7, lmd_tdd1 = 0.909,
               lmd_tdd2 = 4.6, lmd_tdd3 = 0.54, lmd_sdd1 = 0.15, lmd_sdd2 = 1.85, lmd_sdd3 = 0.85, eps = 1.E-14;
  const double Tt = 0.5 * (t0 + t1);
  const double Ts = 0.5 * (s0 + s1) - Smean;
  const double Tp = -zwk;
  const double alfaobeta = A0 + Tt * (A1 + Tt * (A2 + Tt * (A3 + Tt * A4))) + Ts * (B0 + Tt * B1 + Ts * C0) +
                           Tp * (D0 + Tt * (D1 + Tt * D2) + Ts * E0 + Tp * (Ts * F0 + Tt * Tt * G0 + Tp * H0));
  const double ddDT = t1 - t0;
  double ddDS = s1 - s0;
  ddDS = copysign(1., ddDS) * dmax(fabs(ddDS), eps);   // sign(1.,ddDS)*max(abs(ddDS),eps)
  double Rrho = alfaobeta * ddDT / ddDS;
  double nu_dds, nu_ddt;
  if (Rrho > 1. && ddDS > 0.) {   // salt fingering
    Rrho = dmin(Rrho, lmd_Rrho0);
    const double x = (Rrho - 1.) / (lmd_Rrho0 - 1.);
    nu_dds = 1. - x * x;
    nu_dds = lmd_nuf * nu_dds * nu_dds * nu_dds;
    nu_ddt = lmd_fdd * nu_dds;
  } else if (Rrho < 1. && Rrho > 0. && ddDS < 0.) {   // diffusive convection
    nu_ddt = lmd_nu * lmd_tdd1 * exp(lmd_tdd2 * exp(-lmd_tdd3 * ((1. / Rrho) - 1.)));
    if (Rrho < 0.5) nu_dds = nu_ddt * lmd_sdd1 * Rrho;
    else nu_dds = nu_ddt * (lmd_sdd2 * Rrho - lmd_sdd3);
  } else {
    nu_ddt = 0.;
    nu_dds = 0.;
  }
  kt = kt + nu_ddt;
  ks = ks + nu_dds;
}

struct KppConst {
  double Cg, Vtc;  // lmd_kpp.F:137-138 (power functions: evaluated on the host)
};

// lmd_wscale_ws_only.h
__device__ __forceinline__ double wscale_ws(double zscale, double Bfsfc, double hbl, double ustar, double rmask,
                                            double vonKar) {
  zscale = dmin(zscale, hbl * kEpssfc);
  zscale = zscale * rmask;
  const double zetahat = vonKar * zscale * Bfsfc;
  const double ustar3 = ustar * ustar * ustar;
  if (zetahat >= 0.) return vonKar * ustar * ustar3 / dmax(ustar3 + 5. * zetahat, 1.E-20);
  if (zetahat > kZeta_s * ustar3) return vonKar * sqrt((ustar3 - 16. * zetahat) / ustar);  // **r2
  return vonKar * pow(kA_s * ustar3 - kC_s * zetahat, 1. / 3.);
}
// lmd_wscale_wm_and_ws.h
__device__ __forceinline__ void wscale_wm_ws(double zscale, double Bfsfc, double hbl, double ustar, double rmask,
                                             double vonKar, double& wm, double& ws) {
  zscale = dmin(zscale, hbl * kEpssfc);
  zscale = zscale * rmask;
  const double zetahat = vonKar * zscale * Bfsfc;
  const double ustar3 = ustar * ustar * ustar;
  if (zetahat >= 0.) {
    wm = vonKar * ustar * ustar3 / dmax(ustar3 + 5. * zetahat, 1.E-20);
    ws = wm;
  } else {
    if (zetahat > kZeta_m * ustar3) wm = vonKar * pow(ustar * (ustar3 - 16. * zetahat), 0.25);
    else wm = vonKar * pow(kA_m * ustar3 - kC_m * zetahat, 1. / 3.);
    if (zetahat > kZeta_s * ustar3) ws = vonKar * sqrt((ustar3 - 16. * zetahat) / ustar);
    else ws = vonKar * pow(kA_s * ustar3 - kC_s * zetahat, 1. / 3.);
  }
}

// Closed-wall ghost copies of the smoothing stencils (lmd_vmix.F:170-204,
// lmd_kpp_smooth_hbl.h:13-50) as index clamps: a copied ghost cell reads the
// interior cell it was copied from, corners included.
struct EdgeClamp {
  int ilo, ihi, jlo, jhi;
  __device__ __forceinline__ long at(const Bounds& b, int i, int j) const {
    return IJ(b, i < ilo ? ilo : (i > ihi ? ihi : i), j < jlo ? jlo : (j > jhi ? jhi : j));
  }
};
EdgeClamp edge_clamp(const Bounds& b) {
  EdgeClamp c;
  c.ilo = (!b.ew_periodic && b.west_edge) ? b.istr : -1;
  c.ihi = (!b.ew_periodic && b.east_edge) ? b.iend : b.Lm + 2;
  c.jlo = (!b.ns_periodic && b.south_edge) ? b.jstr : -1;
  c.jhi = (!b.ns_periodic && b.north_edge) ? b.jend : b.Mm + 2;
  return c;
}

// Masks of the 3x3 smoothing stencil around (i,j): umask at (i..i+1, j-1..j+1),
// vmask at (i-1..i+1, j..j+1).
struct SmoothMasks {
  double um[3][2];  // [j-1..j+1][i..i+1]
  double vm[2][3];  // [j..j+1][i-1..i+1]
};
__device__ __forceinline__ SmoothMasks smooth_masks(const Bounds& b, const Fields& F, int i, int j) {
  SmoothMasks m;
#pragma unroll
  for (int dj = 0; dj < 3; dj++)
#pragma unroll
    for (int di = 0; di < 2; di++) m.um[dj][di] = F.umask[IJ(b, i + di, j - 1 + dj)];
#pragma unroll
  for (int dj = 0; dj < 2; dj++)
#pragma unroll
    for (int di = 0; di < 3; di++) m.vm[dj][di] = F.vmask[IJ(b, i - 1 + di, j + dj)];
  return m;
}

// Isotropic masked smoother evaluated at one point from w[dj][di] = wrk(i-1+di, j-1+dj)
// (lmd_vmix.F:206-241 == lmd_kpp_smooth_hbl.h:63-102 before the final rmask).
__device__ __forceinline__ double smooth_point(const double (&w)[3][3], const SmoothMasks& m) {
  const double cff = 1. / 12., cff1 = 3. / 16.;
  // FX(a,b) = (wrk(a,b)-wrk(a-1,b))*umask(a,b), a = i,i+1, b = j-1..j+1
  double FX[3][2];
#pragma unroll
  for (int dj = 0; dj < 3; dj++)
#pragma unroll
    for (int di = 0; di < 2; di++) FX[dj][di] = (w[dj][di + 1] - w[dj][di]) * m.um[dj][di];
  // FE1(a,b) = (wrk(a,b)-wrk(a,b-1))*vmask(a,b), a = i-1..i+1, b = j,j+1
  double FE1[2][3];
#pragma unroll
  for (int dj = 0; dj < 2; dj++)
#pragma unroll
    for (int di = 0; di < 3; di++) FE1[dj][di] = (w[dj + 1][di] - w[dj][di]) * m.vm[dj][di];
  // FE(i,b) for b = j, j+1 (raw FX), then FX(a,j) for a = i, i+1 updated with FE1
  const double FEj = FE1[0][1] + cff * (FX[1][1] + FX[0][0] - FX[1][0] - FX[0][1]);
  const double FEjp = FE1[1][1] + cff * (FX[2][1] + FX[1][0] - FX[2][0] - FX[1][1]);
  const double FXi = FX[1][0] + cff * (FE1[1][1] + FE1[0][0] - FE1[0][1] - FE1[1][0]);
  const double FXip = FX[1][1] + cff * (FE1[1][2] + FE1[0][1] - FE1[0][2] - FE1[1][1]);
  return w[1][1] + cff1 * (FXip - FXi + FEjp - FEj);
}

__device__ __forceinline__ void load3x3(const Bounds& b, const EdgeClamp& ec, const double* a, int i, int j,
                                        double (&w)[3][3]) {
#pragma unroll
  for (int dj = 0; dj < 3; dj++)
#pragma unroll
    for (int di = 0; di < 3; di++) w[dj][di] = a[ec.at(b, i - 1 + di, j - 1 + dj)];
}

// ---- lmd_swr_frac.F:31-85 (Jwt = 1) ----
__global__ void __launch_bounds__(256) k_swr_frac(Dev d, Range R) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const int N = b.N;
  const double mu1 = 0.35, mu2 = 23.0, r1 = 0.58;
  const double attn1 = -1. / mu1, attn2 = -1. / mu2;
  double swdk1 = r1, swdk2 = 1. - swdk1;
  double* __restrict__ sw = d.f.swr_frac + ij;
  const double* __restrict__ Hz = d.f.Hz + ij;
  sw[(long)N * n2] = 1.;
  for (int k = N; k >= 1; k--) {
    const double hz = Hz[(long)(k - 1) * n2];
    const double xi1 = attn1 * hz;
    if (xi1 > -20.) swdk1 = swdk1 * exp(xi1);
    else swdk1 = 0.;
    const double xi2 = attn2 * hz;
    if (xi2 > -20.) swdk2 = swdk2 * exp(xi2);
    else swdk2 = 0.;
    sw[(long)(k - 1) * n2] = swdk1 + swdk2;
  }
}

// levels per load batch of the KPP depth scans (kbls, the bottom layer)
#ifndef ROMS_KBLS_G
#define ROMS_KBLS_G 16
#endif
constexpr int kKblsG = ROMS_KBLS_G;
// levels of k_kpp_int's Rig window / z_w loads in flight ahead of the level formed
#ifndef ROMS_KPP_PFD
#define ROMS_KPP_PFD 1
#endif
constexpr int kKppPfd = ROMS_KPP_PFD;

// ---- pass 1: extended range ----
#ifndef ROMS_KPP_EXT_WAVES
#define ROMS_KPP_EXT_WAVES 3   // waves per SIMD the register budget is cut for (the next level in flight: 3)
#endif
template <class C>
__global__ void __launch_bounds__(64, ROMS_KPP_EXT_WAVES) k_kpp_ext(Dev d, Range E, int tind, int nstp, KppConst kc) {
  ROMS_IJC_OR_RETURN(E)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const long n2 = b.n2, ij = IJ(b, i, j), sj = b.nx2;
  const double g = P.g, vonKar = P.vonKar, Ri_inv = 1. / kRicr;
  // FC(0:N): the LDS column, or the global scratch column through the
  // column's buffer offset (ColGlb: no 64-bit address per level)
  const C FCc = ColMake<C>::at(d, 0, 0, ij);
  const BufF64 FCg(d.f.colscr);
  constexpr bool kGlb = std::is_same<C, ColGlb>::value;
  auto fc_set = [&](int k, double v) {
    if constexpr (kGlb) FCg.st(v, (unsigned)ij * 8u, (unsigned)k * (unsigned)n2 * 8u);
    else FCc[k] = v;
  };
  auto fc_get = [&](int k) {
    if constexpr (kGlb) return FCg.ld((unsigned)ij * 8u, (unsigned)k * (unsigned)n2 * 8u);
    else return FCc[k];
  };
  // alfabeta.F:46-78 at t(N,nstp); Bo, Bosol, ustar (lmd_kpp.F:154-181)
  double alpha, beta;
  const double Tt = F.t[ij + (long)(N - 1) * n2 + (long)(nstp - 1) * b.n3];
  if (P.nonlin_eos) {
    const double r01 = 6.793952E-2, r02 = -9.095290E-3, r03 = +1.001685E-4, r04 = -1.120083E-6,
                 r05 = +6.536332E-9, r10 = +0.824493, r11 = -4.08990E-3, r12 = +7.64380E-5,
                 r13 = -8.24670E-7, r14 = +5.38750E-9, rS0 = -5.72466E-3, rS1 = +1.02270E-4,
                 rS2 = -1.65460E-6, r20 = +4.8314E-4;
    const double cff = 1. / P.rho0;
    if (P.salinity) {
      const double Ts = F.t[ij + (long)(N - 1) * n2 + (long)(nstp - 1) * b.n3 + 3 * b.n3], sqrtTs = sqrt(dmax(0., Ts));
      alpha = -cff * (r01 + Tt * (2. * r02 + Tt * (3. * r03 + Tt * (4. * r04 + Tt * 5. * r05))) +
                      Ts * (r11 + Tt * (2. * r12 + Tt * (3. * r13 + Tt * 4. * r14)) + sqrtTs * (rS1 + Tt * 2. * rS2)));
      beta = cff * (r10 + Tt * (r11 + Tt * (r12 + Tt * (r13 + Tt * r14))) + 1.5 * (rS0 + Tt * (rS1 + Tt * rS2)) * sqrtTs +
                    2. * r20 * Ts);
    } else {
      alpha = -cff * (r01 + Tt * (2. * r02 + Tt * (3. * r03 + Tt * (4. * r04 + Tt * 5. * r05))));
      beta = 0.;
    }
  } else {
    alpha = fabs(P.Tcoef);
    beta = P.salinity ? fabs(P.Scoef) : 0.;
  }
  const double sr = F.srflx[ij];
  const double Bo = P.salinity ? g * (alpha * (F.stflx[ij] - sr) - beta * F.stflx[ij + n2]) : g * (alpha * (F.stflx[ij] - sr));
  const double Bosol = g * alpha * sr;
  double ustar;
  if (P.bulk_frc) {   // BULK_FRC: rho-point stresses (lmd_kpp.F:173-174)
    const double sr_ = F.sustr_r[ij], sv_ = F.svstr_r[ij];
    ustar = sqrt(sqrt(sr_ * sr_ + sv_ * sv_));
  } else {
    const double su0 = F.sustr[ij], su1 = F.sustr[ij + 1], sv0 = F.svstr[ij], sv1 = F.svstr[ij + sj];
    ustar = sqrt(sqrt(0.333333333333 * (su0 * su0 + su1 * su1 + su0 * su1 + sv0 * sv0 + sv1 * sv1 + sv0 * sv1)));
  }
  const double hbl0 = F.hbls[ij], bbl0 = F.hbbl[ij];
  const double rm = F.rmask[ij], ff = F.f[ij];
  F.lmd_Bo[ij] = Bo;
  F.lmd_Bosol[ij] = Bosol;
  F.lmd_ustar[ij] = ustar;

  // buffer accesses: the column (and its i+1 / j+1 neighbour) in VGPR
  // offsets, the level in an SGPR (no 64-bit address per level)
  const unsigned vo = (unsigned)ij * 8u, vx = vo + 8u, vy = vo + (unsigned)sj * 8u, lv = (unsigned)n2 * 8u;
  const BufF64 U(F.u + (long)(tind - 1) * b.n3), V(F.v + (long)(tind - 1) * b.n3), Hz(F.Hz), zr(F.z_r), zw(F.z_w),
      bvf(F.bvf), sw(F.swr_frac), rig(F.lmd_rig);
  const double zwN = zw.ld(vo, (unsigned)N * lv), zw0 = zw.ld(vo, 0);
  const double eh = kEpssfc * hbl0, eb = kEpssfc * bbl0;
  const double eh2 = eh * eh, eb2 = eb * eb;

  // Cr(k) = FC(k) + Vtsq(k) with sw(k), sw(k-1), bvf(k-1) at the w levels
  auto vtsq = [&](double zrk, double swk, double swm, double bm) {
    const double swdk_r = sqrt(swk * swm);
    const double zscale = zwN - zrk;
    const double Bfsfc = Bo + Bosol * (1. - swdk_r);
    const double ws = wscale_ws(zscale, Bfsfc, hbl0, ustar, rm, vonKar);
    return 1.8 * kc.Vtc * ws * sqrt(dmax(1.e-5, bm));
  };
  // a level's inputs: u, v (and the i+1 / j+1 neighbours), Hz, z_r at rho
  // level k, z_w at w level k, sw and bvf at w level k-1 (its w level k
  // values are the level above's); the next level's are loaded before this
  // level's stores, so a level costs one memory round trip, not three
  struct Lv { double u0, u1, v0, v1, hz, zr, zw, swm, bm; };
  auto ldlev = [&](int k, Lv& L) {
    const unsigned o = (unsigned)(k - 1) * lv, ow = (unsigned)k * lv;
    L.u0 = U.ld(vo, o); L.u1 = U.ld(vx, o); L.v0 = V.ld(vo, o); L.v1 = V.ld(vy, o);
    L.hz = Hz.ld(vo, o); L.zr = zr.ld(vo, o); L.zw = zw.ld(vo, ow);
    L.swm = sw.ld(vo, o); L.bm = bvf.ld(vo, o);
  };
  // k = N: FC(N) = 0, Cr(N) = Vtsq(N)
  const unsigned oN = (unsigned)(N - 1) * lv;
  double u0p = U.ld(vo, oN), u1p = U.ld(vx, oN);  // level k+1
  double v0p = V.ld(vo, oN), v1p = V.ld(vy, oN);
  double hzp = Hz.ld(vo, oN), zrp = zr.ld(vo, oN);
  double swc = sw.ld(vo, oN), bc = bvf.ld(vo, oN);   // sw, bvf at w level k (carried down)
  Lv cur{};
  if (N - 1 >= 1) ldlev(N - 1, cur);
  double FCk = 0.;
  fc_set(N, 0.);
  double Crp = FCk + vtsq(zrp, sw.ld(vo, (unsigned)N * lv), swc, bc);
  int kbls = Crp < 0. ? N : 0;
  double cr_k = Crp, cr_kp = 0., zr_k = zrp, zr_kp = 0.;
  for (int k = N - 1; k >= 1; k--) {
    Lv nxt = cur;
    if (k > 1) ldlev(k - 1, nxt);
    const unsigned ow = (unsigned)k * lv;
    const double u0 = cur.u0, u1 = cur.u1, v0 = cur.v0, v1 = cur.v1;
    const double hz = cur.hz, zrk = cur.zr, zwk = cur.zw, bk = bc;
    // raw gradient Richardson number (lmd_vmix.F:157-165), LMD_RIMIX only
    if (P.lmd_rimix) {
      const double cff = 0.5 / (zrp - zrk);
      const double dudz = cff * (u0p - u0 + u1p - u1);
      const double dvdz = cff * (v0p - v0 + v1p - v1);
      rig.st(bk / (kRi0 * dmax(dudz * dudz + dvdz * dvdz, 1.E-10)), vo, ow);
    }
    // bulk Richardson integral (lmd_kpp.F:200-215)
    {
      const double cu = zwN - zwk, cd = zwk - zw0;
      const double cff_up = cu * cu, cff_dn = cd * cd;
      const double Kern = cff_up * cff_dn / ((cff_up + eh2) * (cff_dn + eb2));
      const double du = u0p + u1p - u0 - u1;
      const double dv = v0p + v1p - v0 - v1;
      const double hh = hz + hzp;
      FCk = FCk + Kern * (0.5 * (du * du + dv * dv) / hh - 0.5 * hh * (Ri_inv * bk + kC_Ek * ff * ff));
      fc_set(k, FCk);
    }
    const double Cr = FCk + vtsq(zrk, swc, cur.swm, cur.bm);
    if (kbls == 0 && Cr < 0.) {
      kbls = k;
      cr_k = Cr; cr_kp = Crp; zr_k = zrk; zr_kp = zrp;
    }
    Crp = Cr;
    u0p = u0; u1p = u1; v0p = v0; v1p = v1; hzp = hz; zrp = zrk;
    swc = cur.swm; bc = cur.bm;
    cur = nxt;
  }
  // FC(0) (lmd_kpp.F:216-229): level-1 values are the carried ones, FCk is FC(1)
  double fc0;
  {
    const double hz1 = hzp;
    const double z_bl = zw0 + 0.25 * hz1;
    const double cu = zwN - z_bl, cd = z_bl - zw0;
    const double cff_up = cu * cu, cff_dn = cd * cd;
    const double Kern = cff_up * cff_dn / ((cff_up + eh2) * (cff_dn + eb2));
    const double su = u0p + u1p, sv = v0p + v1p;
    fc0 = FCk + Kern * (0.5 * (su * su + sv * sv) / hz1 - 0.5 * hz1 * (Ri_inv * bvf.ld(vo, lv) + kC_Ek * ff * ff));
    fc_set(0, fc0);
  }
  double hbl;
  if (kbls > 0) {
    if (kbls == N) hbl = zwN - zr.ld(vo, oN);
    else hbl = zwN - (zr_k * cr_kp - zr_kp * cr_k) / (cr_kp - cr_k);
  } else {
    hbl = zwN - zw0;
  }
  F.lmd_hbl[ij] = hbl * rm;
  // bottom layer (lmd_kpp.F:276-305): Cr(k) = FC(k) - FC(0), first k upward with Cr > 0
  const double FC0 = fc0;
  double bbl = zwN - zw0;
  // the first k upward with Cr(k) > 0 and Cr(k-1) (0 below k = 1): FC read
  // kKblsG levels at a time, the scan ends once every lane of the wave has
  // its level (one load per iteration waited on a round trip per level)
  int kb = 0;
  double crk = 0., crmk = 0.;
  {
    constexpr int G = kKblsG;
    double crm = 0.;
    for (int k0 = 1; k0 <= N; k0 += G) {   // k0 wave-uniform
      double c[G];
#pragma unroll
      for (int q = 0; q < G; q++) c[q] = fc_get(k0 + q <= N ? k0 + q : N);
#pragma unroll
      for (int q = 0; q < G; q++) {
        if (kb == 0 && k0 + q <= N) {
          const double cr = c[q] - FC0;
          if (cr > 0.) { kb = k0 + q; crk = cr; crmk = crm; }
          crm = cr;
        }
      }
      if (__all(kb != 0)) break;
    }
  }
  if (kb == 1) bbl = zr.ld(vo, 0) - zw0;
  else if (kb > 1) {   // per-lane level: VGPR offsets
    const double zrm = zr.ld(vo + (unsigned)(kb - 2) * lv, 0u), zrk = zr.ld(vo + (unsigned)(kb - 1) * lv, 0u);
    bbl = (zrm * crk - zrk * crmk) / (crk - crmk) - zw0;
  }
  F.lmd_bbl[ij] = bbl * rm;
}

// ---- pass 2: interior ----
// kDD: LMD_DDMIX (its T/S loads and registers only where it is on).
// TY > 0 (LMD_RIMIX only): blocks of 64 x TY columns stage each level's
// smoothed-Rig stencil window ((64+2) x (TY+2) raw Rig values, clamped at
// the edges like load3x3) in LDS once, double-buffered with one barrier per
// level, instead of nine global loads per lane; lanes past the range walk
// the levels too (barriers) and store nothing.  Same values bitwise.
template <bool kDD, int TY = 0, int MW = 1>   // MW: minimum waves per SIMD (VGPR cap)
__global__ void __launch_bounds__(TY > 0 ? kCX * TY : 64, MW) k_kpp_int(Dev d, Range R, EdgeClamp ec, int tind, int nstp,
                                                                   int first, KppConst kc) {
  constexpr bool STG = TY > 0;
  constexpr int TYB = STG ? TY : 1, WW = kCX + 2, WN = WW * (TYB + 2), NTH = kCX * TYB, WQ = (WN + NTH - 1) / NTH;
  const uint3 bI = xcd_tile();
  const int ti0 = tile_i0(R.i0);
  int i = ti0 + (int)(bI.x * kCX + threadIdx.x);
  int j = R.j0 + (int)(bI.y * TYB + threadIdx.y);
  const bool act = i >= R.i0 && i <= R.i1 && j <= R.j1;
  if (!STG && !act) return;
  if (!act) { i = i < R.i0 ? R.i0 : (i < R.i1 ? i : R.i1); j = j < R.j1 ? j : R.j1; }
  __shared__ double sW[STG ? 2 : 1][STG ? WN : 1];
  const int tid = threadIdx.x + kCX * threadIdx.y;
  const int wi0 = ti0 + (int)bI.x * kCX - 1, wj0 = R.j0 + (int)bI.y * TYB - 1;   // (EdgeClamp keeps i >= -1)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const long n2 = b.n2, ij = IJ(b, i, j), sj = b.nx2;
  const double vonKar = P.vonKar, Zob = P.Zob;
  const double akv = P.Akv_bak, akt = P.Akt_bak[0], aks = P.Akt_bak[b.nTS - 1];
  const double rm = F.rmask[ij];
  const SmoothMasks m = smooth_masks(b, F, i, j);
  // SMOOTH_HBL (lmd_kpp_smooth_hbl.h), then the two-step average (lmd_kpp.F:327-338)
  double w[3][3];
  load3x3(b, ec, F.lmd_hbl, i, j, w);
  double hbl = smooth_point(w, m) * rm;
  load3x3(b, ec, F.lmd_bbl, i, j, w);
  double bbl = smooth_point(w, m) * rm;
  if (!first) {
    hbl = 0.5 * (hbl + F.hbls[ij]);
    bbl = 0.5 * (bbl + F.hbbl[ij]);
  }
  // buffer accesses: the column in one VGPR offset, the level in an SGPR
  const unsigned vo = (unsigned)ij * 8u, lv = (unsigned)n2 * 8u;
  const BufF64 zw(F.z_w), sw(F.swr_frac);
  const double zwN = zw.ld(vo, (unsigned)N * lv), zw0 = zw.ld(vo, 0);
  // kbls and the buoyancy forcing at the boundary-layer depth (lmd_kpp.F:348-372)
  // (the downward scan keeps its last hit: kbls is the smallest k in 1..N-1
  // with z_w(k) > zwN - hbl, else N).  Levels are loaded kKblsG at a time --
  // a scan with one load per iteration waited on 99 round trips per column.
  int kbls = N;
  {
    constexpr int G = kKblsG;
    for (int k0 = N - 1; k0 >= 1; k0 -= G) {   // k0 wave-uniform: scalar level offsets
      double z[G];
#pragma unroll
      for (int q = 0; q < G; q++) z[q] = zw.ld(vo, (unsigned)(k0 - q >= 1 ? k0 - q : 1) * lv);
#pragma unroll
      for (int q = 0; q < G; q++)
        if (k0 - q >= 1 && z[q] > zwN - hbl) kbls = k0 - q;
    }
  }
  const double Bo = F.lmd_Bo[ij], Bosol = F.lmd_Bosol[ij], ustar = F.lmd_ustar[ij];
  double Bfsfc;
  {
    const double z_bl = zwN - hbl;
    // kbls differs between lanes: its level offsets go in the VGPR offset
    // (an SGPR offset would be a loop over the wave's distinct values)
    const unsigned ok = vo + (unsigned)kbls * lv, om = vo + (unsigned)(kbls - 1) * lv;
    const double swm = sw.ld(om, 0u), swk = sw.ld(ok, 0u);
    const double zwk = zw.ld(ok, 0u), zwm = zw.ld(om, 0u);
    if (swm > 0.)
      Bfsfc = Bo + Bosol * (1. - swm * swk * (zwk - zwm) / (swk * (zwk - z_bl) + swm * (z_bl - zwm)));
    else
      Bfsfc = Bo + Bosol;
  }
  // BKPP friction velocity (lmd_kpp.F:472-480)
  double wmb;
  {
    const long o = (long)(nstp - 1) * b.n3 + ij;
    const double u0 = F.u[o], u1 = F.u[o + 1], v0 = F.v[o], v1 = F.v[o + sj];
    wmb = vonKar * vonKar * sqrt(0.333333333333 * (u0 * u0 + u1 * u1 + u0 * u1 + v0 * v0 + v1 * v1 + v0 * v1)) /
          log(1. + 0.5 * F.Hz[ij] / Zob);
  }
  const double wsb = wmb;

  // raw interior Kv, Kt (= Ks) at level k from the smoothed Rig (lmd_vmix.F:249-272, 338-353)
  const double* __restrict__ rig = F.lmd_rig;
  const BufF64 Rg(F.lmd_rig);
  // the staged window's entries of this thread: column offsets (level-independent)
  unsigned wo[STG ? WQ : 1];
  if constexpr (STG) {
#pragma unroll
    for (int m = 0; m < WQ; m++) {
      const int q = tid + m * NTH;
      wo[m] = q < WN ? (unsigned)ec.at(b, wi0 + q % WW, wj0 + q / WW) * 8u : kBufOff;
    }
  }
  const bool rimix = P.lmd_rimix, convec = P.lmd_convec, nonlocal = P.lmd_nonlocal;
  // raw_k split into its loads (rload) and its arithmetic (rcomp), so the
  // loads of level k+2 can be issued ahead of level k's stores (which would
  // otherwise hold them back: the compiler cannot prove the arrays apart)
  // LMD_DDMIX: T and S at levels k, k+1 (tind)
  constexpr bool dd = kDD;
  const double* __restrict__ Tt = F.t + (long)(tind - 1) * b.n3 + ij;
  const double* __restrict__ St = Tt + 3 * b.n3;
  struct RL { double r[3][3]; double zw, t0, t1, s0, s1; double win[STG ? WQ : 1]; int k; };
  auto rload = [&](int k, RL& L) {
    L.k = k;
    if (STG) {   // this thread's entries of the level's window (rimix is on)
#pragma unroll
      for (int m = 0; m < WQ; m++) L.win[m] = Rg.ld(wo[m], (unsigned)k * lv);   // kBufOff entries read 0
    } else if (rimix) {
      load3x3(b, ec, rig + (long)k * n2, i, j, L.r);
    }
    L.zw = zw.ld(vo, (unsigned)k * lv);
    if (dd) {
      const long o = (long)(k - 1) * n2;
      L.t0 = Tt[o]; L.t1 = Tt[o + n2]; L.s0 = St[o]; L.s1 = St[o + n2];
    }
  };
  auto rcomp = [&](const RL& L, double& kv, double& kt, double& ks) {
    if (rimix) {
      double Rig;
      if (STG) {
        double* buf = sW[STG ? (L.k & 1) : 0];
#pragma unroll
        for (int mq = 0; mq < WQ; mq++) {
          const int q = tid + mq * NTH;
          if (q < WN) buf[q] = L.win[mq];
        }
        __syncthreads();
        double w[3][3];
#pragma unroll
        for (int dj = 0; dj < 3; dj++)
#pragma unroll
          for (int di = 0; di < 3; di++) w[dj][di] = buf[(threadIdx.y + dj) * WW + threadIdx.x + di];
        Rig = smooth_point(w, m);
      } else {
        Rig = smooth_point(L.r, m);
      }
      const double cff = dmin(1., dmax(0., Rig));
      double nu_sx = 1. - cff * cff;
      nu_sx = nu_sx * nu_sx * nu_sx;
      kv = kNuwm + kNu0m * nu_sx;
      kt = kNuws + kNu0s * nu_sx;
      if (convec && Rig < 0.) {   // LMD_CONVEC (lmd_vmix.F:269-274)
        kv = kv + kNu0c;
        kt = kt + kNu0c;
      }
    } else {                      // internal waves only (lmd_vmix.F:262-264)
      kv = kNuwm;
      kt = kNuws;
    }
    ks = kt;
    if (dd) ddmix(L.t0, L.t1, L.s0, L.s1, L.zw, kt, ks);
    const double zwk = L.zw;
    const double dist = zwk - zw0;
    if (dist < kLturb) {
      const double mult = sin(0.5 * kPi * (zwk - zw0) / kLturb);
      kv = kv * mult;
      kt = kt * mult;
      ks = ks * mult;
    }
  };
  const BufF64 Akv(F.Akv), AktT(F.Akt), AktS(F.Akt + b.n3w), ghat(F.ghat);
  const unsigned vs = act ? vo : kBufOff;   // lanes past the range store nothing
  const bool wet = rm > 0.5;
  // KPP shape functions (lmd_kpp.F:374-446), BKPP (:447-495), masked copy (:496-528)
  auto finish = [&](int k, double Kv, double Kt, double Ks, double zwk) {
    const double ssgm = (zwN - zwk) / dmax(hbl, kEPS);
    double gh = 0.;
    if (ssgm < 1.) {
      // the turbulent velocity scales are only used inside the boundary layer
      // (lmd_kpp.F:407-441 forms them at every level and discards them below)
      double wm, ws;
      wscale_wm_ws(zwN - zwk, Bfsfc, hbl, ustar, rm, vonKar, wm, ws);
      double cff;
      if (ssgm < 0.07) cff = 0.5 * ((ssgm - 0.07) * (ssgm - 0.07)) / 0.07;
      else cff = 0.;
      cff = cff + ssgm * ((1. - ssgm) * (1. - ssgm));
      const double amp = ssgm * ssgm;
      double a, q;
      a = amp * Kv; q = wm * hbl * cff;
      Kv = sqrt(a * a + q * q);
      a = amp * Kt; q = ws * hbl * cff;
      Kt = sqrt(a * a + q * q);
      a = amp * Ks;
      Ks = sqrt(a * a + q * q);
      if (Bfsfc < 0.) gh = -(kc.Cg * ssgm * ((1. - ssgm) * (1. - ssgm)));
    }
    const unsigned ow = (unsigned)k * lv;
    if (nonlocal) ghat.st(gh, vs, ow);   // LMD_NONLOCAL (lmd_kpp.F:436-446)
    const double sgmb = (zwk - zw0 + Zob) / (bbl + Zob);
    if (sgmb < 1.) {
      const double cff1 = sgmb * ((1. - sgmb) * (1. - sgmb));
      double q = wmb * bbl * cff1;
      Kv = sqrt(Kv * Kv + q * q);
      q = wsb * bbl * cff1;
      Kt = sqrt(Kt * Kt + q * q);
      Ks = sqrt(Ks * Ks + q * q);
    }
    Akv.st(wet ? Kv : 0., vs, ow);
    AktT.st(wet ? Kt : 0., vs, ow);
    if (b.nTS > 1) AktS.st(wet ? Ks : 0., vs, ow);
  };
  // bottom-up stream: padding (lmd_vmix.F:359-370) and the in-place ascending
  // 1-2-1 filter Kv(k) = 0.5 Kv(k) + 0.25 Kv(k-1)[filtered] + 0.25 Kv(k+1)[raw] + bak
  double rv, rt, rs;  // raw level k (rs = rt unless LMD_DDMIX)
  // PD levels' loads in flight ahead of the one formed (a ring of RL)
  constexpr int PD = kKppPfd;
  RL La, Lr[PD];
  rload(1, La);
#pragma unroll
  for (int q = 0; q < PD; q++)
    if (N - 1 >= 2 + q) rload(2 + q, Lr[q]);
  rcomp(La, rv, rt, rs);
  double zk = La.zw;  // z_w of level k
  double rvN = rv, rtN = rt, rsN = rs;  // raw level N-1 (known once reached)
  double sv = rv + akv, st = rt + akt, ss = rs + aks;  // level 0 (padded)
  finish(0, sv, st, ss, zw0);
  for (int k = 1; k <= N - 1; k++) {
    double nv, nt, ns;  // level k+1 before filtering
    double rvn = 0., rtn = 0., rsn = 0., zk1 = 0.;
    if (k + 1 <= N - 1) {
      const RL cur = Lr[0];
#pragma unroll
      for (int q = 0; q + 1 < PD; q++) Lr[q] = Lr[q + 1];
      if (k + 1 + PD <= N - 1) rload(k + 1 + PD, Lr[PD - 1]);
      rcomp(cur, rvn, rtn, rsn);
      zk1 = cur.zw;
      nv = rvn; nt = rtn; ns = rsn;
    } else {
      rvN = rv; rtN = rt; rsN = rs;
      nv = rv + akv; nt = rt + akt; ns = rs + aks;
    }
    sv = 0.5 * rv + 0.25 * sv + 0.25 * nv + akv;
    st = 0.5 * rt + 0.25 * st + 0.25 * nt + akt;
    ss = 0.5 * rs + 0.25 * ss + 0.25 * ns + aks;
    finish(k, sv, st, ss, zk);
    rv = rvn; rt = rtn; rs = rsn; zk = zk1;
  }
  finish(N, rvN + akv, rtN + akt, rsN + aks, zwN);
  // hbls/hbbl and their closed-wall ghost copies (lmd_kpp.F:530-620)
  if (!act) return;
  F.hbls[ij] = hbl;
  F.hbbl[ij] = bbl;
  const bool W = !b.ew_periodic && b.west_edge && i == b.istr, E = !b.ew_periodic && b.east_edge && i == b.iend;
  const bool S = !b.ns_periodic && b.south_edge && j == b.jstr, Nn = !b.ns_periodic && b.north_edge && j == b.jend;
  if (W) { F.hbls[ij - 1] = hbl; F.hbbl[ij - 1] = bbl; }
  if (E) { F.hbls[ij + 1] = hbl; F.hbbl[ij + 1] = bbl; }
  if (S) { F.hbls[ij - sj] = hbl; F.hbbl[ij - sj] = bbl; }
  if (Nn) { F.hbls[ij + sj] = hbl; F.hbbl[ij + sj] = bbl; }
  if (W && S) { F.hbls[ij - 1 - sj] = hbl; F.hbbl[ij - 1 - sj] = bbl; }
  if (W && Nn) { F.hbls[ij - 1 + sj] = hbl; F.hbbl[ij - 1 + sj] = bbl; }
  if (E && S) { F.hbls[ij + 1 - sj] = hbl; F.hbbl[ij + 1 - sj] = bbl; }
  if (E && Nn) { F.hbls[ij + 1 + sj] = hbl; F.hbbl[ij + 1 + sj] = bbl; }
}

}  // namespace

void launch_swr_frac(const Dev& d, hipStream_t s) {
  const Bounds& b = d.b;
  const Range R{b.istr, b.iend, b.jstr, b.jend};
  hipLaunchKernelGGL(k_swr_frac, grid_of(R), dim3(kBX, kBY), 0, s, d, R);
  ExchList L{};
  L.p[0] = d.f.swr_frac; L.nlev[0] = b.N + 1; L.n = 1;
  launch_exchange_list(d, s, L);
}

void launch_lmd_vmix(const Dev& d, hipStream_t s, const Tlev& t, int tind) {
  const Bounds& b = d.b;
  // lmd_kpp.F:97-123 (== lmd_vmix.F:105-141): I_EXT_RANGE x J_EXT_RANGE
  Range E;
  E.i0 = (b.ew_periodic || !b.west_edge) ? b.istr - 1 : b.istr;
  E.i1 = (b.ew_periodic || !b.east_edge) ? b.iend + 1 : b.iend;
  E.j0 = (b.ns_periodic || !b.south_edge) ? b.jstr - 1 : b.jstr;
  E.j1 = (b.ns_periodic || !b.north_edge) ? b.jend + 1 : b.jend;
  const Range R{b.istr, b.iend, b.jstr, b.jend};
  // Cg, Vtc (lmd_kpp.F:137-138) with host libm, like the reference's own runtime pow
  const double vonKar = d.p.vonKar, Cstar = 10., c_s = kC_s, epssfc = kEpssfc, Cv = 1.8, betaT = -0.2;
  KppConst kc;
  kc.Cg = Cstar * vonKar * std::pow(c_s * vonKar * epssfc, 1. / 3.);
  kc.Vtc = Cv * std::sqrt(-betaT / (c_s * epssfc)) / (kRicr * (vonKar * vonKar));
  const int first = t.iic == t.forw_start;  // FIRST_TIME_STEP with EXACT_RESTART
  if (d.f.colscr)
    hipLaunchKernelGGL(k_kpp_ext<ColGlb>, gridc_of(E), dim3(kCX), 0, s, d, E, tind, t.nstp, kc);
  else
    hipLaunchKernelGGL(k_kpp_ext<ColLds>, gridc_of(E), dim3(kCX), col_lds_bytes(1, b.N), s, d, E, tind, t.nstp, kc);
  if (d.p.kpp_ty && d.p.lmd_rimix) {   // staged Rig windows on 64 x TY column blocks
    const int ty = d.p.lmd_ddmix ? 4 : (d.p.kpp_ty == 8 || d.p.kpp_ty == 2) ? d.p.kpp_ty : 4;   // the DDMIX form is instantiated on 64x4 only
    dim3 g = gridc_of(R);
    g.y = (g.y + ty - 1) / ty;
    const EdgeClamp ec = edge_clamp(b);
    if (d.p.lmd_ddmix)
      hipLaunchKernelGGL((k_kpp_int<true, 4>), g, dim3(kCX, 4), 0, s, d, R, ec, tind, t.nstp, first, kc);
    else if (d.p.kpp_ty == 2)
      hipLaunchKernelGGL((k_kpp_int<false, 2>), g, dim3(kCX, 2), 0, s, d, R, ec, tind, t.nstp, first, kc);
    else if (d.p.kpp_ty == 8)
      hipLaunchKernelGGL((k_kpp_int<false, 8>), g, dim3(kCX, 8), 0, s, d, R, ec, tind, t.nstp, first, kc);
    else if (d.p.kpp_ty == 43)
      hipLaunchKernelGGL((k_kpp_int<false, 4, 3>), g, dim3(kCX, 4), 0, s, d, R, ec, tind, t.nstp, first, kc);
    else
      hipLaunchKernelGGL((k_kpp_int<false, 4>), g, dim3(kCX, 4), 0, s, d, R, ec, tind, t.nstp, first, kc);
  } else if (d.p.lmd_ddmix) {
    hipLaunchKernelGGL(k_kpp_int<true>, gridc_of(R), dim3(kCX), 0, s, d, R, edge_clamp(b), tind, t.nstp, first, kc);
  } else {
    hipLaunchKernelGGL(k_kpp_int<false>, gridc_of(R), dim3(kCX), 0, s, d, R, edge_clamp(b), tind, t.nstp, first, kc);
  }
  // lmd_kpp.F:631-649: Akv, hbls, hbbl, Akt(itemp), Akt(isalt)
  ExchList L{};
  L.p[0] = d.f.Akv; L.nlev[0] = b.N + 1;
  L.p[1] = d.f.hbls; L.nlev[1] = 1;
  L.p[2] = d.f.hbbl; L.nlev[2] = 1;
  L.p[3] = d.f.Akt; L.nlev[3] = (b.N + 1) * b.nTS;
  L.n = 4;
  launch_exchange_list(d, s, L);
}

}  // namespace roms
