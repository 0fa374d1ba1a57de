/*
 * oracle_lmd.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 *
 * Plain-C restatement of the LMD/KPP vertical mixing of the reference for
 * the switch set of tests/Pipes_ana and the C3 basin (LMD_MIXING, LMD_KPP,
 * LMD_BKPP, LMD_RIMIX, LMD_CONVEC, LMD_NONLOCAL, LMD_DDMIX, SALINITY,
 * MASKING; no MERGE_OVERLAP, no LIMIT_UNSTABLE_ONLY):
 *   or_swr_frac       lmd_swr_frac.F:13-88   (Jerlov type 1, at init)
 *   lmd_vmix_tile     lmd_vmix.F:31-433      (SMOOTH_RIG)
 *   lmd_kpp_tile      lmd_kpp.F:7-651        (INT_AT_RHO_POINTS, SMOOTH_HBL)
 *   alfabeta          alfabeta.F:4-79
 *   wscale            lmd_wscale_ws_only.h, lmd_wscale_wm_and_ws.h
 *   smooth_hbl        lmd_kpp_smooth_hbl.h
 * Fortran x**2 / x**3 are products (as gfortran expands integer powers);
 * real exponents (**r2, **r3, **r4, **(1./3.)) go through pow().
 */
#include <math.h>
#include <stdio.h>
#include "oracle_core.h"

#define KV(i, j, k) W3(S->lmdKv, i, j, k)
#define KT(i, j, k) W3(S->lmdKt, i, j, k)
#define KS(i, j, k) W3(S->lmdKs, i, j, k)
#define RIG(i, j, k) W3(S->lmdRig, i, j, k)
#define BVF(i, j, k) W3(S->bvf, i, j, k)
#define SWR(i, j, k) W3(S->swr_frac, i, j, k)
#define GHAT(i, j, k) W3(S->ghat, i, j, k)

void or_lmd_alloc(or_state *S) {
  S->lmdKv = calloc(S->n3w, sizeof(double));
  S->lmdKt = calloc(S->n3w, sizeof(double));
  S->lmdKs = calloc(S->n3w, sizeof(double));
  S->lmdRig = calloc(S->n3w, sizeof(double));
  for (int q = 0; q < 9; q++) S->lmd2[q] = calloc(S->n2, sizeof(double));
}

/* lmd_swr_frac.F:31-85, Jwt=1 */
void or_swr_frac(or_state *S) {
  const double mu1 = 0.35, mu2 = 23.0, r1 = 0.58;
  const double attn1 = -1. / mu1, attn2 = -1. / mu2;
  const int N = S->N;
  for (int j = S->jstr; j <= S->jend; j++)
    for (int i = S->istr; i <= S->iend; i++) {
      double swdk1 = r1, swdk2 = 1. - swdk1;
      SWR(i, j, N) = 1.;
      for (int k = N; k >= 1; k--) {
        const double xi1 = attn1 * HZ(i, j, k);
        if (xi1 > -20.) swdk1 = swdk1 * exp(xi1);
        else swdk1 = 0.;
        const double xi2 = attn2 * HZ(i, j, k);
        if (xi2 > -20.) swdk2 = swdk2 * exp(xi2);
        else swdk2 = 0.;
        SWR(i, j, k - 1) = swdk1 + swdk2;
      }
    }
  or_exch3(S, S->swr_frac, N + 1);
}

/* extended ranges of the smoothing operators (lmd_vmix.F:88-127, lmd_kpp.F:98-133) */
static void ext_range(const or_state *S, int *imin, int *imax, int *jmin, int *jmax) {
  if (S->c.ew_periodic) { *imin = S->istr - 1; *imax = S->iend + 1; }
  else { *imin = S->west_edge ? S->istr : S->istr - 1; *imax = S->east_edge ? S->iend : S->iend + 1; }
  if (S->c.ns_periodic) { *jmin = S->jstr - 1; *jmax = S->jend + 1; }
  else { *jmin = S->south_edge ? S->jstr : S->jstr - 1; *jmax = S->north_edge ? S->jend : S->jend + 1; }
}

/* closed-edge ghost copies of a 2-D field over the extended ranges */
static void edge_pad(or_state *S, double *w, int imin, int imax, int jmin, int jmax) {
  const int is = S->istr, ie = S->iend, js = S->jstr, je = S->jend;
  if (!S->c.ew_periodic) {
    if (S->west_edge) for (int j = jmin; j <= jmax; j++) A2(w, is - 1, j) = A2(w, is, j);
    if (S->east_edge) for (int j = jmin; j <= jmax; j++) A2(w, ie + 1, j) = A2(w, ie, j);
  }
  if (!S->c.ns_periodic) {
    if (S->south_edge) for (int i = imin; i <= imax; i++) A2(w, i, js - 1) = A2(w, i, js);
    if (S->north_edge) for (int i = imin; i <= imax; i++) A2(w, i, je + 1) = A2(w, i, je);
    if (!S->c.ew_periodic) {
      if (S->west_edge && S->south_edge) A2(w, is - 1, js - 1) = A2(w, is, js);
      if (S->west_edge && S->north_edge) A2(w, is - 1, je + 1) = A2(w, is, je);
      if (S->east_edge && S->south_edge) A2(w, ie + 1, js - 1) = A2(w, ie, js);
      if (S->east_edge && S->north_edge) A2(w, ie + 1, je + 1) = A2(w, ie, je);
    }
  }
}

/* isotropic masked smoother (lmd_vmix.F:206-241 and lmd_kpp_smooth_hbl.h:63-102);
   rmask_after: the KPP version re-masks the result */
static void smooth2(or_state *S, double *w, int rmask_after) {
  double *FX = S->lmd2[0], *FE = S->lmd2[1], *FE1 = S->lmd2[2];
  const double cff = 1. / 12., cff1 = 3. / 16.;
  const int is = S->istr, ie = S->iend, js = S->jstr, je = S->jend;
  for (int j = js - 1; j <= je + 1; j++)
    for (int i = is; i <= ie + 1; i++) A2(FX, i, j) = (A2(w, i, j) - A2(w, i - 1, j)) * A2(S->umask, i, j);
  for (int j = js; j <= je + 1; j++) {
    for (int i = is - 1; i <= ie + 1; i++) A2(FE1, i, j) = (A2(w, i, j) - A2(w, i, j - 1)) * A2(S->vmask, i, j);
    for (int i = is; i <= ie; i++)
      A2(FE, i, j) = A2(FE1, i, j) + cff * (A2(FX, i + 1, j) + A2(FX, i, j - 1) - A2(FX, i, j) - A2(FX, i + 1, j - 1));
  }
  for (int j = js; j <= je; j++) {
    for (int i = is; i <= ie + 1; i++)
      A2(FX, i, j) = A2(FX, i, j) + cff * (A2(FE1, i, j + 1) + A2(FE1, i - 1, j) - A2(FE1, i, j) - A2(FE1, i - 1, j + 1));
    for (int i = is; i <= ie; i++) {
      A2(w, i, j) = A2(w, i, j) + cff1 * (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j));
      if (rmask_after) A2(w, i, j) = A2(w, i, j) * A2(S->rmask, i, j);
    }
  }
}

/* LMD_DDMIX (lmd_vmix.F:95-101, 279-360): double-diffusive mixing added to
 * Kt and Ks at w-level k from t(k), t(k+1) at tind and z_w(k) */
static void ddmix(or_state *S, int i, int j, int k, int tind, double *kt, double *ks) {
  const double A0 = +0.665157E-01, A1 = +0.170907E-01, A2 = -0.203814E-03, A3 = +0.298357E-05,
               A4 = -0.255019E-07, B0 = +0.378110E-02, B1 = -0.846960E-04, C0 = -0.678662E-05,
               D0 = +0.380374E-04, D1 = -0.933746E-06, D2 = +0.791325E-08, E0 = -0.164759E-06,
               F0 = -0.251520E-11, G0 = +0.512857E-12, H0 = -0.302285E-13, Smean = 35.0;
  const double lmd_nu = 1.5e-6, lmd_Rrho0 = 1.9, lmd_nuf = 10.0e-4, lmd_fdd = 0.7, lmd_tdd1 = 0.909,
               lmd_tdd2 = 4.6, lmd_tdd3 = 0.54, lmd_sdd1 = 0.15, lmd_sdd2 = 1.85, lmd_sdd3 = 0.85, eps = 1.E-14;
  const double t0 = TT(i, j, k, tind, 1), t1 = TT(i, j, k + 1, tind, 1);
  const double s0 = TT(i, j, k, tind, 2), s1 = TT(i, j, k + 1, tind, 2);
  const double Tt = 0.5 * (t0 + t1);
  const double Ts = 0.5 * (s0 + s1) - Smean;
  const double Tp = -ZW(i, j, k);
  const double alfaobeta = A0 + Tt * (A1 + Tt * (A2 + Tt * (A3 + Tt * A4))) + Ts * (B0 + Tt * B1 + Ts * C0) +
                           Tp * (D0 + Tt * (D1 + Tt * D2) + Ts * E0 + Tp * (Ts * F0 + Tt * Tt * G0 + Tp * H0));
  const double ddDT = t1 - t0;
  double ddDS = s1 - s0;
  ddDS = copysign(1., ddDS) * dmax(fabs(ddDS), eps);
  double Rrho = alfaobeta * ddDT / ddDS;
  double nu_dds, nu_ddt;
  if (Rrho > 1. && ddDS > 0.) {  /* salt fingering */
    Rrho = dmin(Rrho, lmd_Rrho0);
    const double x = (Rrho - 1.) / (lmd_Rrho0 - 1.);
    nu_dds = 1. - x * x;
    nu_dds = lmd_nuf * nu_dds * nu_dds * nu_dds;
    nu_ddt = lmd_fdd * nu_dds;
  } else if (Rrho < 1. && Rrho > 0. && ddDS < 0.) {  /* diffusive convection */
    nu_ddt = lmd_nu * lmd_tdd1 * exp(lmd_tdd2 * exp(-lmd_tdd3 * ((1. / Rrho) - 1.)));
    if (Rrho < 0.5) nu_dds = nu_ddt * lmd_sdd1 * Rrho;
    else nu_dds = nu_ddt * (lmd_sdd2 * Rrho - lmd_sdd3);
  } else {
    nu_ddt = 0.;
    nu_dds = 0.;
  }
  *kt = *kt + nu_ddt;
  *ks = *ks + nu_dds;
}

/* lmd_vmix_tile (lmd_vmix.F:31-433): interior Kv, Kt, Ks at w-levels 0..N */
static void lmd_vmix_tile(or_state *S, int tind) {
  const int N = S->N;
  const double Ri0 = 0.7, nu0m = 1.e-2, nu0s = 1.e-2, nuwm = 1.0e-4, nuws = 0.1e-4, nu0c = 0.1, Lturb = 10.;
  const double pi = 3.14159265358979323;
  int imin, imax, jmin, jmax;
  ext_range(S, &imin, &imax, &jmin, &jmax);
  double *Rk = S->lmd2[3];
  const int rimix = (S->c.lmd & OR_LMD_RIMIX) != 0, convec = (S->c.lmd & OR_LMD_CONVEC) != 0;
  const int dd = (S->c.lmd & OR_LMD_DDMIX) != 0 && S->c.salinity;
  for (int k = 1; k <= N - 1; k++) {
    if (!rimix) {  /* internal waves only (lmd_vmix.F:262-264) */
      for (int j = S->jstr; j <= S->jend; j++)
        for (int i = S->istr; i <= S->iend; i++) {
          double kt = nuws, ks = nuws;
          if (dd) ddmix(S, i, j, k, tind, &kt, &ks);
          KV(i, j, k) = nuwm;
          KT(i, j, k) = kt;
          KS(i, j, k) = ks;
        }
      continue;
    }
    for (int j = jmin; j <= jmax; j++)
      for (int i = imin; i <= imax; i++) {
        const double cff = 0.5 / (ZR(i, j, k + 1) - ZR(i, j, k));
        const double dudz = cff * (U(i, j, k + 1, tind) - U(i, j, k, tind) + U(i + 1, j, k + 1, tind) - U(i + 1, j, k, tind));
        const double dvdz = cff * (V(i, j, k + 1, tind) - V(i, j, k, tind) + V(i, j + 1, k + 1, tind) - V(i, j + 1, k, tind));
        A2(Rk, i, j) = BVF(i, j, k) / (Ri0 * dmax(dudz * dudz + dvdz * dvdz, 1.E-10));
      }
    edge_pad(S, Rk, imin, imax, jmin, jmax);
    smooth2(S, Rk, 0);
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = S->istr; i <= S->iend; i++) {
        const double rig = A2(Rk, i, j);
        RIG(i, j, k) = rig;
        const double cff = dmin(1., dmax(0., rig));
        double nu_sx = 1. - cff * cff;
        nu_sx = nu_sx * nu_sx * nu_sx;
        double kv = nuwm + nu0m * nu_sx, kt = nuws + nu0s * nu_sx;
        if (convec && rig < 0.) { kv = kv + nu0c; kt = kt + nu0c; }  /* LMD_CONVEC (lmd_vmix.F:269-274) */
        double ks = kt;
        if (dd) ddmix(S, i, j, k, tind, &kt, &ks);
        KV(i, j, k) = kv;
        KT(i, j, k) = kt;
        KS(i, j, k) = ks;
      }
  }
  for (int k = 1; k <= N - 1; k++)
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = S->istr; i <= S->iend; i++) {
        const double dist = ZW(i, j, k) - ZW(i, j, 0);
        if (dist < Lturb) {
          const double mult = sin(0.5 * pi * (ZW(i, j, k) - ZW(i, j, 0)) / Lturb);
          KV(i, j, k) = KV(i, j, k) * mult;
          KT(i, j, k) = KT(i, j, k) * mult;
          KS(i, j, k) = KS(i, j, k) * mult;
        }
      }
  const double akv = S->c.Akv_bak, akt = S->c.Akt_bak[0], aks = S->c.Akt_bak[S->nTS - 1];
  for (int j = S->jstr; j <= S->jend; j++)
    for (int i = S->istr; i <= S->iend; i++) {
      KV(i, j, N) = KV(i, j, N - 1) + akv;
      KS(i, j, N) = KS(i, j, N - 1) + aks;
      KT(i, j, N) = KT(i, j, N - 1) + akt;
      KV(i, j, 0) = KV(i, j, 1) + akv;
      KS(i, j, 0) = KS(i, j, 1) + aks;
      KT(i, j, 0) = KT(i, j, 1) + akt;
    }
  /* vertical 1-2-1 smoothing, in place upward (uses the already smoothed k-1) */
  for (int k = 1; k <= N - 1; k++)
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = S->istr; i <= S->iend; i++) {
        KV(i, j, k) = 0.5 * KV(i, j, k) + 0.25 * KV(i, j, k - 1) + 0.25 * KV(i, j, k + 1) + akv;
        KT(i, j, k) = 0.5 * KT(i, j, k) + 0.25 * KT(i, j, k - 1) + 0.25 * KT(i, j, k + 1) + akt;
        KS(i, j, k) = 0.5 * KS(i, j, k) + 0.25 * KS(i, j, k - 1) + 0.25 * KS(i, j, k + 1) + aks;
      }
}

/* KPP constants (lmd_kpp.F:70-95) */
#define K_Ricr 0.15
#define K_epssfc 0.1
#define K_betaT (-0.2)
#define K_Cv 1.8
#define K_C_Ek 258.
#define K_Cstar 10.
#define K_zeta_m (-0.2)
#define K_a_m 1.257
#define K_c_m 8.360
#define K_zeta_s (-1.0)
#define K_a_s (-28.86)
#define K_c_s 98.96

/* lmd_wscale_ws_only.h */
static double wscale_ws(double zscale, double Bfsfc, double hbl, double ustar, double rmask, double vonKar) {
  const double r2 = 0.5, r3 = 1. / 3.;
  zscale = dmin(zscale, hbl * K_epssfc);
  zscale = zscale * rmask;
  const double zetahat = vonKar * zscale * Bfsfc;
  const double ustar3 = ustar * ustar * ustar;
  if (zetahat >= 0.) return vonKar * ustar * ustar3 / dmax(ustar3 + 5. * zetahat, 1.E-20);
  if (zetahat > K_zeta_s * ustar3) return vonKar * pow((ustar3 - 16. * zetahat) / ustar, r2);
  return vonKar * pow(K_a_s * ustar3 - K_c_s * zetahat, r3);
}
/* lmd_wscale_wm_and_ws.h */
static void wscale_wm_ws(double zscale, double Bfsfc, double hbl, double ustar, double rmask, double vonKar,
                         double *wm, double *ws) {
  const double r2 = 0.5, r3 = 1. / 3., r4 = 0.25;
  zscale = dmin(zscale, hbl * K_epssfc);
  zscale = zscale * rmask;
  const double zetahat = vonKar * zscale * Bfsfc;
  const double ustar3 = ustar * ustar * ustar;
  if (zetahat >= 0.) {
    *wm = vonKar * ustar * ustar3 / dmax(ustar3 + 5. * zetahat, 1.E-20);
    *ws = *wm;
  } else {
    if (zetahat > K_zeta_m * ustar3) *wm = vonKar * pow(ustar * (ustar3 - 16. * zetahat), r4);
    else *wm = vonKar * pow(K_a_m * ustar3 - K_c_m * zetahat, r3);
    if (zetahat > K_zeta_s * ustar3) *ws = vonKar * pow((ustar3 - 16. * zetahat) / ustar, r2);
    else *ws = vonKar * pow(K_a_s * ustar3 - K_c_s * zetahat, r3);
  }
}

/* lmd_kpp_tile (lmd_kpp.F:7-651) */
static void lmd_kpp_tile(or_state *S, int tind) {
  const int N = S->N;
  const double vonKar = S->vonKar, g = S->g, Zob = S->c.Zob;
  const double Ri_inv = 1. / K_Ricr, EPS = 1.E-20;
  const double Cg = K_Cstar * vonKar * pow(K_c_s * vonKar * K_epssfc, 1. / 3.);
  const double Vtc = K_Cv * sqrt(-K_betaT / (K_c_s * K_epssfc)) / (K_Ricr * (vonKar * vonKar));
  const int first = S->iic == S->forw_start;  /* FIRST_TIME_STEP, EXACT_RESTART (set_global_definitions.h:339) */
  int imin, imax, jmin, jmax;
  ext_range(S, &imin, &imax, &jmin, &jmax);
  double *ustar = S->lmd2[4], *Bo = S->lmd2[5], *Bosol = S->lmd2[6], *hbl = S->lmd2[7], *bbl = S->lmd2[8];
  double *FC = S->c1[0], *Cr = S->c1[1];
  int *kbls = malloc(sizeof(int) * (size_t)S->nx2), *kbbl = malloc(sizeof(int) * (size_t)S->nx2);
  double *Bfsfc_bl = malloc(sizeof(double) * (size_t)S->nx2);
#define KI(i) ((i) + 1)
  const int nstp = S->nstp;
  const double rho0 = S->rho0;
  const int nonlocal = (S->c.lmd & OR_LMD_NONLOCAL) != 0;
  for (int j = jmin; j <= jmax; j++) {
    for (int i = imin; i <= imax; i++) {
      /* alfabeta.F:46-78 (NONLIN_EOS, SALINITY) at t(N,nstp) */
      double alpha, beta;
      if (S->c.nonlin_eos) {
        const double r01 = 6.793952E-2, r02 = -9.095290E-3, r03 = +1.001685E-4, r04 = -1.120083E-6,
                     r05 = +6.536332E-9, r10 = +0.824493, r11 = -4.08990E-3, r12 = +7.64380E-5,
                     r13 = -8.24670E-7, r14 = +5.38750E-9, rS0 = -5.72466E-3, rS1 = +1.02270E-4,
                     rS2 = -1.65460E-6, r20 = +4.8314E-4;
        const double cff = 1. / rho0;
        const double Tt = TT(i, j, N, nstp, 1);
        const double Ts = S->c.salinity ? TT(i, j, N, nstp, 2) : 0.0, sqrtTs = sqrt(dmax(0., Ts));
        if (S->c.salinity) {
          alpha = -cff * (r01 + Tt * (2. * r02 + Tt * (3. * r03 + Tt * (4. * r04 + Tt * 5. * r05))) +
                          Ts * (r11 + Tt * (2. * r12 + Tt * (3. * r13 + Tt * 4. * r14)) + sqrtTs * (rS1 + Tt * 2. * rS2)));
          beta = cff * (r10 + Tt * (r11 + Tt * (r12 + Tt * (r13 + Tt * r14))) + 1.5 * (rS0 + Tt * (rS1 + Tt * rS2)) * sqrtTs +
                        2. * r20 * Ts);
        } else {
          alpha = -cff * (r01 + Tt * (2. * r02 + Tt * (3. * r03 + Tt * (4. * r04 + Tt * 5. * r05))));
          beta = 0.;
        }
      } else {
        alpha = fabs(S->c.Tcoef);
        beta = S->c.salinity ? fabs(S->c.Scoef) : 0.;
      }
      double bo = g * (alpha * (A2(S->stflx, i, j) - A2(S->srflx, i, j)));
      if (S->c.salinity) bo = g * (alpha * (A2(S->stflx, i, j) - A2(S->srflx, i, j)) - beta * S->stflx[O2(i, j) + S->n2]);
      A2(Bo, i, j) = bo;
      A2(Bosol, i, j) = g * alpha * A2(S->srflx, i, j);
      const double su0 = A2(S->sustr, i, j), su1 = A2(S->sustr, i + 1, j), sv0 = A2(S->svstr, i, j),
                   sv1 = A2(S->svstr, i, j + 1);
      if (S->c.bulk_frc)   /* BULK_FRC: rho-point stresses (lmd_kpp.F:173-174) */
        A2(ustar, i, j) = sqrt(sqrt(A2(S->sustr_r, i, j) * A2(S->sustr_r, i, j) + A2(S->svstr_r, i, j) * A2(S->svstr_r, i, j)));
      else
        A2(ustar, i, j) = sqrt(sqrt(0.333333333333 * (su0 * su0 + su1 * su1 + su0 * su1 + sv0 * sv0 + sv1 * sv1 + sv0 * sv1)));
      A2(hbl, i, j) = A2(S->hbls, i, j);
      A2(bbl, i, j) = A2(S->hbbl, i, j);
      kbls[KI(i)] = 0;
      C1(Cr, i, N) = 0.;
      C1(Cr, i, 0) = 0.;
      C1(FC, i, N) = 0.;
    }
    /* INT_AT_RHO_POINTS bulk Richardson integral */
    for (int k = N - 1; k >= 1; k--)
      for (int i = imin; i <= imax; i++) {
        const double cu = ZW(i, j, N) - ZW(i, j, k), cd = ZW(i, j, k) - ZW(i, j, 0);
        const double cff_up = cu * cu, cff_dn = cd * cd;
        const double eh = K_epssfc * A2(hbl, i, j), eb = K_epssfc * A2(bbl, i, j);
        const double Kern = cff_up * cff_dn / ((cff_up + eh * eh) * (cff_dn + eb * eb));
        const double du = U(i, j, k + 1, tind) + U(i + 1, j, k + 1, tind) - U(i, j, k, tind) - U(i + 1, j, k, tind);
        const double dv = V(i, j, k + 1, tind) + V(i, j + 1, k + 1, tind) - V(i, j, k, tind) - V(i, j + 1, k, tind);
        const double hh = HZ(i, j, k) + HZ(i, j, k + 1);
        const double ff = A2(S->f, i, j);
        C1(FC, i, k) = C1(FC, i, k + 1) +
                       Kern * (0.5 * (du * du + dv * dv) / hh - 0.5 * hh * (Ri_inv * BVF(i, j, k) + K_C_Ek * ff * ff));
      }
    for (int i = imin; i <= imax; i++) {
      const double z_bl = ZW(i, j, 0) + 0.25 * HZ(i, j, 1);
      const double cu = ZW(i, j, N) - z_bl, cd = z_bl - ZW(i, j, 0);
      const double cff_up = cu * cu, cff_dn = cd * cd;
      const double eh = K_epssfc * A2(hbl, i, j), eb = K_epssfc * A2(bbl, i, j);
      const double Kern = cff_up * cff_dn / ((cff_up + eh * eh) * (cff_dn + eb * eb));
      const double su = U(i, j, 1, tind) + U(i + 1, j, 1, tind), sv = V(i, j, 1, tind) + V(i, j + 1, 1, tind);
      const double ff = A2(S->f, i, j);
      C1(FC, i, 0) = C1(FC, i, 1) + Kern * (0.5 * (su * su + sv * sv) / HZ(i, j, 1) -
                                            0.5 * HZ(i, j, 1) * (Ri_inv * BVF(i, j, 1) + K_C_Ek * ff * ff));
    }
    for (int k = N; k >= 1; k--)
      for (int i = imin; i <= imax; i++) {
        const double swdk_r = sqrt(SWR(i, j, k) * SWR(i, j, k - 1));
        const double zscale = ZW(i, j, N) - ZR(i, j, k);
        const double Bfsfc = A2(Bo, i, j) + A2(Bosol, i, j) * (1. - swdk_r);
        const double ws = wscale_ws(zscale, Bfsfc, A2(hbl, i, j), A2(ustar, i, j), A2(S->rmask, i, j), vonKar);
        const double Vtsq = 1.8 * Vtc * ws * sqrt(dmax(1.e-5, BVF(i, j, k - 1)));
        C1(Cr, i, k) = C1(FC, i, k) + Vtsq;
        if (kbls[KI(i)] == 0 && C1(Cr, i, k) < 0.) kbls[KI(i)] = k;
      }
    for (int i = imin; i <= imax; i++) {
      double hb;
      if (kbls[KI(i)] > 0) {
        const int k = kbls[KI(i)];
        if (k == N) hb = ZW(i, j, N) - ZR(i, j, N);
        else
          hb = ZW(i, j, N) - (ZR(i, j, k) * C1(Cr, i, k + 1) - ZR(i, j, k + 1) * C1(Cr, i, k)) /
                                 (C1(Cr, i, k + 1) - C1(Cr, i, k));
      } else {
        hb = ZW(i, j, N) - ZW(i, j, 0);
      }
      A2(hbl, i, j) = hb * A2(S->rmask, i, j);
    }
    for (int i = imin; i <= imax; i++) {
      kbbl[KI(i)] = 0;
      C1(Cr, i, 0) = 0.;
    }
    for (int k = 1; k <= N; k++)
      for (int i = imin; i <= imax; i++) {
        C1(Cr, i, k) = C1(FC, i, k) - C1(FC, i, 0);
        if (kbbl[KI(i)] == 0 && C1(Cr, i, k) > 0.) kbbl[KI(i)] = k;
      }
    for (int i = imin; i <= imax; i++) {
      double bb;
      if (kbbl[KI(i)] > 0) {
        const int k = kbbl[KI(i)];
        if (k == 1) bb = ZR(i, j, 1) - ZW(i, j, 0);
        else
          bb = (ZR(i, j, k - 1) * C1(Cr, i, k) - ZR(i, j, k) * C1(Cr, i, k - 1)) / (C1(Cr, i, k) - C1(Cr, i, k - 1)) -
               ZW(i, j, 0);
      } else {
        bb = ZW(i, j, N) - ZW(i, j, 0);
      }
      A2(bbl, i, j) = bb * A2(S->rmask, i, j);
    }
  }
  /* SMOOTH_HBL (lmd_kpp_smooth_hbl.h) for hbl then bbl */
  edge_pad(S, hbl, imin, imax, jmin, jmax);
  smooth2(S, hbl, 1);
  edge_pad(S, bbl, imin, imax, jmin, jmax);
  smooth2(S, bbl, 1);

  for (int j = S->jstr; j <= S->jend; j++) {
    if (!first)
      for (int i = S->istr; i <= S->iend; i++) {
        A2(hbl, i, j) = 0.5 * (A2(hbl, i, j) + A2(S->hbls, i, j));
        A2(bbl, i, j) = 0.5 * (A2(bbl, i, j) + A2(S->hbbl, i, j));
      }
    for (int i = S->istr; i <= S->iend; i++) kbls[KI(i)] = N;
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istr; i <= S->iend; i++)
        if (ZW(i, j, k) > ZW(i, j, N) - A2(hbl, i, j)) kbls[KI(i)] = k;
    for (int i = S->istr; i <= S->iend; i++) {
      const int k = kbls[KI(i)];
      const double z_bl = ZW(i, j, N) - A2(hbl, i, j);
      const double zscale = A2(hbl, i, j);
      double Bfsfc;
      if (SWR(i, j, k - 1) > 0.)
        Bfsfc = A2(Bo, i, j) + A2(Bosol, i, j) *
                                   (1. - SWR(i, j, k - 1) * SWR(i, j, k) * (ZW(i, j, k) - ZW(i, j, k - 1)) /
                                             (SWR(i, j, k) * (ZW(i, j, k) - z_bl) + SWR(i, j, k - 1) * (z_bl - ZW(i, j, k - 1))));
      else
        Bfsfc = A2(Bo, i, j) + A2(Bosol, i, j);
      double wm, ws;
      wscale_wm_ws(zscale, Bfsfc, A2(hbl, i, j), A2(ustar, i, j), A2(S->rmask, i, j), vonKar, &wm, &ws);
      Bfsfc_bl[KI(i)] = Bfsfc;
    }
    for (int i = S->istr; i <= S->iend; i++)
      for (int k = N; k >= 0; k--) {
        const double Bfsfc = Bfsfc_bl[KI(i)];
        const double zscale = ZW(i, j, N) - ZW(i, j, k);
        double wm, ws;
        wscale_wm_ws(zscale, Bfsfc, A2(hbl, i, j), A2(ustar, i, j), A2(S->rmask, i, j), vonKar, &wm, &ws);
        const double ssgm = (ZW(i, j, N) - ZW(i, j, k)) / dmax(A2(hbl, i, j), EPS);
        if (ssgm < 1.) {
          double cff;
          if (ssgm < 0.07) cff = 0.5 * ((ssgm - 0.07) * (ssgm - 0.07)) / 0.07;
          else cff = 0.;
          cff = cff + ssgm * ((1. - ssgm) * (1. - ssgm));
          const double amp = ssgm * ssgm;
          const double hb = A2(hbl, i, j);
          double a, w;
          a = amp * KV(i, j, k); w = wm * hb * cff;
          KV(i, j, k) = sqrt(a * a + w * w);
          a = amp * KT(i, j, k); w = ws * hb * cff;
          KT(i, j, k) = sqrt(a * a + w * w);
          a = amp * KS(i, j, k);
          KS(i, j, k) = sqrt(a * a + w * w);
          if (nonlocal) {  /* LMD_NONLOCAL (lmd_kpp.F:436-442) */
            if (Bfsfc < 0.) GHAT(i, j, k) = -(Cg * ssgm * ((1. - ssgm) * (1. - ssgm)));
            else GHAT(i, j, k) = 0.;
          }
        } else {
          if (nonlocal) GHAT(i, j, k) = 0.;
        }
      }
    /* LMD_BKPP bottom layer */
    for (int i = S->istr; i <= S->iend; i++) {
      const double u0 = U(i, j, 1, nstp), u1 = U(i + 1, j, 1, nstp), v0 = V(i, j, 1, nstp), v1 = V(i, j + 1, 1, nstp);
      const double wmb = vonKar * vonKar * sqrt(0.333333333333 * (u0 * u0 + u1 * u1 + u0 * u1 + v0 * v0 + v1 * v1 + v0 * v1)) /
                         log(1. + 0.5 * HZ(i, j, 1) / Zob);
      const double wsb = wmb;
      for (int k = 0; k <= N; k++) {
        const double sgmb = (ZW(i, j, k) - ZW(i, j, 0) + Zob) / (A2(bbl, i, j) + Zob);
        if (sgmb < 1.) {
          const double cff1 = sgmb * ((1. - sgmb) * (1. - sgmb));
          double w = wmb * A2(bbl, i, j) * cff1;
          KV(i, j, k) = sqrt(KV(i, j, k) * KV(i, j, k) + w * w);
          w = wsb * A2(bbl, i, j) * cff1;
          KT(i, j, k) = sqrt(KT(i, j, k) * KT(i, j, k) + w * w);
          KS(i, j, k) = sqrt(KS(i, j, k) * KS(i, j, k) + w * w);
        }
      }
    }
    for (int i = S->istr; i <= S->iend; i++) {
      if (A2(S->rmask, i, j) > 0.5) {
        for (int k = 0; k <= N; k++) {
          AKV(i, j, k) = KV(i, j, k);
          AKT(i, j, k, 1) = KT(i, j, k);
          if (S->nTS > 1) AKT(i, j, k, 2) = KS(i, j, k);
        }
      } else {
        for (int k = 0; k <= N; k++) {
          AKV(i, j, k) = 0.;
          AKT(i, j, k, 1) = 0.;
          if (S->nTS > 1) AKT(i, j, k, 2) = 0.;
        }
      }
    }
  }
  for (int j = S->jstr; j <= S->jend; j++)
    for (int i = S->istr; i <= S->iend; i++) {
      A2(S->hbls, i, j) = A2(hbl, i, j);
      A2(S->hbbl, i, j) = A2(bbl, i, j);
    }
  edge_pad(S, S->hbls, S->istr, S->iend, S->jstr, S->jend);
  edge_pad(S, S->hbbl, S->istr, S->iend, S->jstr, S->jend);
  or_exch3(S, S->Akv, N + 1);
  or_exch2(S, S->hbls);
  or_exch2(S, S->hbbl);
  or_exch3(S, S->Akt, N + 1);
  if (S->nTS > 1) or_exch3(S, S->Akt + S->n3w, N + 1);
  free(kbls);
  free(kbbl);
  free(Bfsfc_bl);
#undef KI
}

void or_lmd_vmix_impl(or_state *S, int tind) {
  lmd_vmix_tile(S, tind);
  lmd_kpp_tile(S, tind);
}
