/*
 * oracle_bulk.c -- TEST INFRASTRUCTURE ONLY (parity checker, see roms_oracle.h).
 *
 * BULK_FRC surface fluxes: calc_all_bulk_forces (bulk_frc.F:143-913), the
 * COARE 3.0 bulk formulae with the surface-current feedback on the stress,
 * restated loop by loop over the extended bounds of compute_extended_bounds.h,
 * and the stability functions bulk_psiu / bulk_psit (bulk_frc.F:916-1036).
 * Inputs: uwnd, vwnd, tair, qair (Q), prate, swrad (short-wave data in W/m2,
 * read into srflx by set_frc_data in the reference), lwrad; t, u, v at nrhs.
 * Without QCORRECTION / SFLX_CORR / TAU_CORRECTION / SEA_ICE_NOFLUX.
 */
#include <math.h>

#include "oracle_core.h"

static double bulk_psiu(double ZoL, double pi) {   /* bulk_frc.F:916-976 */
  const double r3 = 1.0 / 3.0;
  double Fw, cff, psic, psik, x, y;
  if (ZoL < 0.0) {
    x = pow(1.0 - 15.0 * ZoL, 0.25);
    psik = 2.0 * log(0.5 * (1.0 + x)) + log(0.5 * (1.0 + x * x)) - 2.0 * atan(x) + 0.5 * pi;
    cff = sqrt(3.0);
    y = pow(1.0 - 10.15 * ZoL, r3);
    psic = 1.5 * log(r3 * (1.0 + y + y * y)) - cff * atan((1.0 + 2.0 * y) / cff) + pi / cff;
    cff = ZoL * ZoL;
    Fw = cff / (1.0 + cff);
    return (1.0 - Fw) * psik + Fw * psic;
  }
  cff = fmin(50.0, 0.35 * ZoL);
  return -((1.0 + ZoL) + 0.6667 * (ZoL - 14.28) / exp(cff) + 8.525);
}

static double bulk_psit(double ZoL, double pi) {   /* bulk_frc.F:978-1036 */
  const double r3 = 1.0 / 3.0;
  double Fw, cff, psic, psik, x, y;
  if (ZoL < 0.0) {
    x = pow(1.0 - 15.0 * ZoL, 0.5);
    psik = 2.0 * log(0.5 * (1.0 + x));
    cff = sqrt(3.0);
    y = pow(1.0 - 34.15 * ZoL, r3);
    psic = 1.5 * log(r3 * (1.0 + y + y * y)) - cff * atan((1.0 + 2.0 * y) / cff) + pi / cff;
    cff = ZoL * ZoL;
    Fw = cff / (1.0 + cff);
    return (1.0 - Fw) * psik + Fw * psic;
  }
  cff = fmin(50.0, 0.35 * ZoL);
  return -(pow(1.0 + 2.0 * ZoL, 1.5) + 0.6667 * (ZoL - 14.28) / exp(cff) + 8.525);
}

void or_bulk_flux(or_state *S) {
  const int N = S->N, nrhs = S->nrhs;
  const double pi = 3.14159265358979323846, Cp = 3985., cmday2ms = 0.01 / 86400.;   /* scalars.F:127-129 */
  const double g = S->g, vonKar = 0.41, rho0 = S->rho0;
  const double blk_Rgas = 287.1, blk_ZW = 10.0, blk_ZT = 10.0, blk_ZQ = 10.0, blk_Zabl = 600.0, blk_beta = 1.2,
               blk_Cpa = 1004.67;
  const double emiss_lw = 0.985, SigmaSB = 5.6697E-8, patm = 1010.0, eps = 1.e-20, r3 = 1.0 / 3.0;
  const double cpi = 1. / Cp;
  /* compute_extended_bounds.h: the R bounds of this routine */
  const int istrR = S->istrE, iendR = S->iendE, jstrR = S->jstrE, jendR = S->jendE;
  const double rho0i = 1.0 / rho0;
  for (int j = jstrR; j <= jendR; j++)
    for (int i = istrR; i <= iendR; i++) A2(S->srflx, i, j) = A2(S->swrad, i, j) / (rho0 * Cp);
  for (int j = jstrR; j <= jendR; j++)
    for (int i = istrR; i <= iendR; i++) {
      const double uw = A2(S->uwnd, i, j), vw = A2(S->vwnd, i, j);
      const double wspd_used = sqrt(uw * uw + vw * vw);
      const double radlw = A2(S->lwrad, i, j) / (rho0 * Cp);
      double wspd0 = wspd_used;
      const double TairC = A2(S->tair, i, j);
      const double TairK = TairC + 273.16;
      const double TseaC = TT(i, j, N, nrhs, 1);
      const double TseaK = TseaC + 273.16;
      const double Q = A2(S->qair, i, j);
      const double hflw = radlw - emiss_lw * rho0i * cpi * SigmaSB * TseaK * TseaK * TseaK * TseaK;
      double cff = (1.0007 + 3.46e-6 * patm) * 6.1121 * exp(17.502 * TseaC / (240.97 + TseaC));
      cff = cff * 0.98;
      const double Qsea = 0.62197 * (cff / (patm - 0.378 * cff));
      const double rhoAir = patm * 100.0 / (blk_Rgas * TairK * (1.0 + 0.61 * Q));
      const double VisAir = 1.326E-5 * (1.0 + TairC * (6.542E-3 + TairC * (8.301e-6 - 4.84e-9 * TairC)));
      const double Hlv = (2.501 - 0.00237 * TseaC) * 1.0e+6;
      double Wgus = 0.5;
      double delW = sqrt(wspd0 * wspd0 + Wgus * Wgus);
      const double delQ = Qsea - Q;
      const double delT = TseaC - TairC;
      double ZoW = 0.0001;
      const double u10 = delW * log(10.0 / ZoW) / log(blk_ZW / ZoW);
      double Wstar = 0.035 * u10;
      const double Zo10 = 0.011 * Wstar * Wstar / g + 0.11 * VisAir / Wstar;
      const double c10 = vonKar / log(10.0 / Zo10), Cd10 = c10 * c10;
      const double Ch10 = 0.00115;
      const double Ct10 = Ch10 / sqrt(Cd10);
      const double ZoT10 = 10.0 / exp(vonKar / Ct10);
      const double cW = vonKar / log(blk_ZW / Zo10);
      double Cd = cW * cW;
      const double Ct = vonKar / log(blk_ZT / ZoT10);
      const double CC = vonKar * Ct / Cd;
      const double Ribcu = -blk_ZW / (blk_Zabl * 0.004 * (blk_beta * blk_beta * blk_beta));
      const double Ri = -g * blk_ZW * (delT + 0.61 * TairK * delQ) / (TairK * delW * delW);
      double Zetu;
      if (Ri < 0.0) Zetu = CC * Ri / (1.0 + Ri / Ribcu);
      else Zetu = CC * Ri / (1.0 + 3.0 * Ri / CC);
      const double L10 = blk_ZW / Zetu;
      const int IterMax = Zetu > 50.0 ? 1 : 3;
      Wstar = delW * vonKar / (log(blk_ZW / Zo10) - bulk_psiu(blk_ZW / L10, pi));
      double Tstar = -delT * vonKar / (log(blk_ZT / ZoT10) - bulk_psit(blk_ZT / L10, pi));
      double Qstar = -delQ * vonKar / (log(blk_ZQ / ZoT10) - bulk_psit(blk_ZQ / L10, pi));
      double charn;
      if (delW > 18.0) charn = 0.018;
      else if ((10.0 < delW) && (delW <= 18.0)) charn = 0.011 + 0.125 * (0.018 - 0.011) * (delW - 10.);
      else charn = 0.011;
      for (int iter = 1; iter <= IterMax; iter++) {
        ZoW = charn * Wstar * Wstar / g + 0.11 * VisAir / (Wstar + eps);
        const double Rr = ZoW * Wstar / VisAir;
        const double ZoQ = fmin(1.15e-4, 5.5e-5 / pow(Rr, 0.6));
        const double ZoT = ZoQ;
        const double ZoL = vonKar * g * blk_ZW * (Tstar * (1.0 + 0.61 * Q) + 0.61 * TairK * Qstar) /
                           (TairK * Wstar * Wstar * (1.0 + 0.61 * Q) + eps);
        const double L = blk_ZW / (ZoL + eps);
        const double Wpsi = bulk_psiu(ZoL, pi);
        const double Tpsi = bulk_psit(blk_ZT / L, pi);
        const double Qpsi = bulk_psit(blk_ZQ / L, pi);
        Wstar = fmax(eps, delW * vonKar / (log(blk_ZW / ZoW) - Wpsi));
        Tstar = -delT * vonKar / (log(blk_ZT / ZoT) - Tpsi);
        Qstar = -delQ * vonKar / (log(blk_ZQ / ZoQ) - Qpsi);
        const double Bff = -g / TairK * Wstar * (Tstar + 0.61 * TairK * Qstar);
        if (Bff > 0.0) Wgus = blk_beta * pow(Bff * blk_Zabl, r3);
        else Wgus = 0.2;
        delW = sqrt(wspd0 * wspd0 + Wgus * Wgus);
      }
      wspd0 = sqrt(wspd0 * wspd0 + Wgus * Wgus);
      Cd = Wstar * Wstar / (wspd0 * wspd0 + eps);
      double hfsen = -blk_Cpa * rhoAir * Wstar * Tstar;
      double hflat = -Hlv * rhoAir * Wstar * Qstar;
      const double upvel = -1.61 * Wstar * Qstar - (1.0 + 1.61 * Q) * Wstar * Tstar / TairK;
      hflat = hflat + rhoAir * Hlv * upvel * Q;
      hflat = -hflat * rho0i * cpi;
      hfsen = -hfsen * rho0i * cpi;
      A2(S->stflx, i, j) = A2(S->srflx, i, j) + hflw + hflat + hfsen;
      if (S->c.salinity) {
        const double evap = -Cp * hflat / Hlv;
        A2(S->swflx, i, j) = A2(S->prate, i, j) * cmday2ms - evap;
      }
      A2(S->stflx, i, j) = A2(S->stflx, i, j) * A2(S->rmask, i, j);
      if (S->c.salinity) S->stflx[O2(i, j) + S->n2] = S->stflx[O2(i, j) + S->n2] * A2(S->rmask, i, j);
      const double aer = rhoAir * wspd0 * rho0i, cer = Cd;
      A2(S->sustr_r, i, j) = aer * cer * uw * A2(S->rmask, i, j);
      A2(S->svstr_r, i, j) = aer * cer * vw * A2(S->rmask, i, j);
    }
  /* surface-current feedback and rho -> u, v points (bulk_frc.F:823-910) */
  const double Wspd_min = 3., stau_ref = -0.0027, cfb_slope = -0.0029, cfb_offset = 0.008;
  for (int j = jstrR; j <= jendR; j++)
    for (int i = istrR; i <= S->iend + 1; i++) {
      const double uw = A2(S->uwnd, i, j), vw = A2(S->vwnd, i, j);
      const double wspd = sqrt(uw * uw + vw * vw);
      double cff;
      if (wspd > Wspd_min) cff = cfb_slope * wspd + cfb_offset;
      else cff = stau_ref;
      A2(S->sustr_r, i, j) = A2(S->sustr_r, i, j) + cff * 0.5 * (U(i, j, N, nrhs) + U(i + 1, j, N, nrhs)) / rho0;
      if (i >= istrR + 1) A2(S->sustr, i, j) = (A2(S->sustr_r, i - 1, j) + A2(S->sustr_r, i, j)) / 2 * A2(S->umask, i, j);
    }
  for (int j = jstrR; j <= S->jend + 1; j++)
    for (int i = istrR; i <= iendR; i++) {
      const double uw = A2(S->uwnd, i, j), vw = A2(S->vwnd, i, j);
      const double wspd = sqrt(uw * uw + vw * vw);
      double cff;
      if (wspd > Wspd_min) cff = cfb_slope * wspd + cfb_offset;
      else cff = stau_ref;
      A2(S->svstr_r, i, j) = A2(S->svstr_r, i, j) + cff * 0.5 * (V(i, j, N, nrhs) + V(i, j + 1, N, nrhs)) / rho0;
      if (j >= jstrR + 1) A2(S->svstr, i, j) = (A2(S->svstr_r, i, j - 1) + A2(S->svstr_r, i, j)) / 2 * A2(S->vmask, i, j);
    }
}
