/*
 * oracle_step.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 *
 * Plain-C restatement of the UCLA-ROMS split-explicit hot path, one function
 * per reference routine, loop bounds and arithmetic order kept as in the
 * reference so the FP64 results are reproducible.  Every function cites the
 * reference file:line it restates (paths relative to /root/reference/src).
 */
#include "oracle_core.h"

/* ---------------------------------------------------------------------- */
/* halo exchange for a single rank: mpi_exchanges.F:528-670 with the rank   */
/* as its own periodic neighbour (mpi_setup.F:65-67,223-236).  The packed   */
/* message is a snapshot of the pre-exchange array; the final state is the  */
/* periodic wrap of the interior over the message extents.                  */
/* ---------------------------------------------------------------------- */
static void exch_lev(or_state *S, double *a) {
  const int Lm = S->Lm, Mm = S->Mm;
  if (S->c.ew_periodic) {
    /* E/W strips cover jl0..jl1 = 0..Mm+1 (single rank in eta) */
    for (int j = 0; j <= Mm + 1; j++) {
      A2(a, -1, j) = A2(a, Lm - 1, j);
      A2(a, 0, j) = A2(a, Lm, j);
      A2(a, Lm + 1, j) = A2(a, 1, j);
      A2(a, Lm + 2, j) = A2(a, 2, j);
    }
  }
  if (S->c.ns_periodic) {
    for (int i = 0; i <= Lm + 1; i++) {
      int is = i;
      if (S->c.ew_periodic) { if (i == 0) is = Lm; if (i == Lm + 1) is = 1; }
      A2(a, i, -1) = A2(a, is, Mm - 1);
      A2(a, i, 0) = A2(a, is, Mm);
      A2(a, i, Mm + 1) = A2(a, is, 1);
      A2(a, i, Mm + 2) = A2(a, is, 2);
    }
  }
  if (S->c.ew_periodic && S->c.ns_periodic) {
    for (int dj = 0; dj < 2; dj++)
      for (int di = 0; di < 2; di++) {
        A2(a, -1 + di, -1 + dj) = A2(a, Lm - 1 + di, Mm - 1 + dj);
        A2(a, Lm + 1 + di, -1 + dj) = A2(a, 1 + di, Mm - 1 + dj);
        A2(a, -1 + di, Mm + 1 + dj) = A2(a, Lm - 1 + di, 1 + dj);
        A2(a, Lm + 1 + di, Mm + 1 + dj) = A2(a, 1 + di, 1 + dj);
      }
  }
}
void or_exch2(or_state *S, double *a) { exch_lev(S, a); }
void or_exch3(or_state *S, double *a, int nlev) {
  for (int k = 0; k < nlev; k++) exch_lev(S, a + (size_t)k * S->n2);
}

/* ---------------------------------------------------------------------- */
/* set_depth_tile (set_depth.F:16-186)                                     */
/* ---------------------------------------------------------------------- */
static void set_depth_tile(or_state *S) {
  const int N = S->N, kn = S->knew;
  const double hc = S->c.hc;
  if (S->iic == 0) {
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istrR; i <= S->iendR; i++) A2(S->hinv, i, j) = 1.0 / (A2(S->h, i, j) + hc);
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istr; i <= S->iendR; i++)
        A2(S->DU_avg1, i, j) = 0.5 * (A2(S->h, i - 1, j) + A2(S->h, i, j) + ZETA(i, j, 1) + ZETA(i - 1, j, 1)) *
                               A2(S->dn_u, i, j) * (UBAR(i, j, 1));
    for (int j = S->jstr; j <= S->jendR; j++)
      for (int i = S->istrR; i <= S->iendR; i++)
        A2(S->DV_avg1, i, j) = 0.5 * (A2(S->h, i, j) + A2(S->h, i, j - 1) + ZETA(i, j, 1) + ZETA(i, j - 1, 1)) *
                               A2(S->dm_v, i, j) * (VBAR(i, j, 1));
  }
  const double ds = 1.0 / (double)N;
  for (int j = S->jstrR; j <= S->jendR; j++) {
    for (int i = S->istrR; i <= S->iendR; i++) ZW(i, j, 0) = -A2(S->h, i, j);
    for (int k = 1; k <= N; k++) {
      const double cff_w = hc * ds * (double)(k - N);
      const double cff_r = hc * ds * ((double)(k - N) - 0.5);
      const double cff1_w = S->Cs_w[k], cff1_r = S->Cs_r[k];
      for (int i = S->istrR; i <= S->iendR; i++) {
        const double z = ZETA(i, j, kn), hh = A2(S->h, i, j), hi = A2(S->hinv, i, j);
        ZW(i, j, k) = z + (z + hh) * (cff_w + cff1_w * hh) * hi;
        ZR(i, j, k) = z + (z + hh) * (cff_r + cff1_r * hh) * hi;
        HZ(i, j, k) = ZW(i, j, k) - ZW(i, j, k - 1);
      }
    }
  }
  if (S->iic == 0) or_exch2(S, S->hinv);
  or_exch3(S, S->z_w, N + 1);
  or_exch3(S, S->z_r, N);
  or_exch3(S, S->Hz, N);
}
void or_set_depth(or_state *S) { set_depth_tile(S); }

/* ---------------------------------------------------------------------- */
/* set_HUV_tile (set_depth.F:190-234)                                      */
/* ---------------------------------------------------------------------- */
void or_set_HUV(or_state *S) {
  const int N = S->N, nr = S->nrhs;
  for (int k = 1; k <= N; k++) {
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istr; i <= S->iendR; i++) {
        FLXU(i, j, k) = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j) * (U(i, j, k, nr));
        R3(S->Hz_u, i, j, k) = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k));
      }
    for (int j = S->jstr; j <= S->jendR; j++)
      for (int i = S->istrR; i <= S->iendR; i++) {
        FLXV(i, j, k) = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j) * (V(i, j, k, nr));
        R3(S->Hz_v, i, j, k) = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k));
      }
  }
  or_exch3(S, S->FlxU, N);
  or_exch3(S, S->FlxV, N);
}

/* ---------------------------------------------------------------------- */
/* set_HUV1_tile (set_depth.F:239-422), CORR_COUPLED_MODE+EXTRAP_BAR_FLUXES */
/* ---------------------------------------------------------------------- */
void or_set_HUV1(or_state *S) {
  const int N = S->N, nn = S->nnew;
  const double NOW = 3.63, MID = 4.47, BAK = 2.05;
  double *DC = S->c1[0], *FC = S->c1[1];
  const int first = (S->iic == S->forw_start);
  for (int j = S->jstrR; j <= S->jendR; j++) {
    for (int i = S->istr; i <= S->iendR; i++) {
      C1(DC, i, N) = 0.5 * (HZ(i, j, N) + HZ(i - 1, j, N)) * A2(S->dn_u, i, j);
      C1(DC, i, 0) = C1(DC, i, N);
      C1(FC, i, 0) = C1(DC, i, N) * U(i, j, N, nn);
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istr; i <= S->iendR; i++) {
        C1(DC, i, k) = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j);
        C1(DC, i, 0) = C1(DC, i, 0) + C1(DC, i, k);
        C1(FC, i, 0) = C1(FC, i, 0) + C1(DC, i, k) * U(i, j, k, nn);
      }
    for (int i = S->istr; i <= S->iendR; i++) {
      if (first)
        C1(FC, i, 0) = (C1(FC, i, 0) - A2(S->DU_avg1, i, j)) / C1(DC, i, 0);
      else
        C1(FC, i, 0) = (C1(FC, i, 0) - NOW * A2(S->DU_avg1, i, j) + MID * A2(S->DU_avg2, i, j) -
                        BAK * A2(S->DU_avg_bak, i, j)) / C1(DC, i, 0);
    }
    for (int k = 1; k <= N; k++)
      for (int i = S->istr; i <= S->iendR; i++) {
        U(i, j, k, nn) = (U(i, j, k, nn) - C1(FC, i, 0)) * A2(S->umask, i, j);
        FLXU(i, j, k) = C1(DC, i, k) * (U(i, j, k, nn));
      }
    if (j >= S->jstr) {
      for (int i = S->istrR; i <= S->iendR; i++) {
        C1(DC, i, N) = 0.5 * (HZ(i, j, N) + HZ(i, j - 1, N)) * A2(S->dm_v, i, j);
        C1(DC, i, 0) = C1(DC, i, N);
        C1(FC, i, 0) = C1(DC, i, N) * V(i, j, N, nn);
      }
      for (int k = N - 1; k >= 1; k--)
        for (int i = S->istrR; i <= S->iendR; i++) {
          C1(DC, i, k) = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j);
          C1(DC, i, 0) = C1(DC, i, 0) + C1(DC, i, k);
          C1(FC, i, 0) = C1(FC, i, 0) + C1(DC, i, k) * V(i, j, k, nn);
        }
      for (int i = S->istrR; i <= S->iendR; i++) {
        if (first)
          C1(FC, i, 0) = (C1(FC, i, 0) - A2(S->DV_avg1, i, j)) / C1(DC, i, 0);
        else
          C1(FC, i, 0) = (C1(FC, i, 0) - NOW * A2(S->DV_avg1, i, j) + MID * A2(S->DV_avg2, i, j) -
                          BAK * A2(S->DV_avg_bak, i, j)) / C1(DC, i, 0);
      }
      for (int k = 1; k <= N; k++)
        for (int i = S->istrR; i <= S->iendR; i++) {
          V(i, j, k, nn) = (V(i, j, k, nn) - C1(FC, i, 0)) * A2(S->vmask, i, j);
          FLXV(i, j, k) = C1(DC, i, k) * (V(i, j, k, nn));
        }
    }
  }
  or_exch3(S, S->FlxU, N);
  or_exch3(S, S->FlxV, N);
  or_exch3(S, S->u + (size_t)(nn - 1) * S->n3, N);
  or_exch3(S, S->v + (size_t)(nn - 1) * S->n3, N);
}

/* ---------------------------------------------------------------------- */
/* omega_tile (omega.F:17-236)                                             */
/* ---------------------------------------------------------------------- */
void or_omega(or_state *S) {
  const int N = S->N;
  const double cu_min = 0.6, cu_max = 1.0, cmnx_ratio = cu_min / cu_max, cutoff = 2.0 - cmnx_ratio,
               r4cmx = 0.25 / (1.0 - cmnx_ratio);
  double *CX = S->c1[0], *wrk = S->c1[1];
  double dtau;
  if (S->nrhs == 3) dtau = S->dt;
  else if (S->iic == S->forw_start) dtau = 0.5 * S->dt;
  else dtau = 0.6 * S->dt;
  for (int j = 1; j <= S->Mm; j++)
    for (int i = 1; i <= S->Lm; i++) WI(i, j, 0) = 0.0;
  for (int j = S->jstr; j <= S->jend; j++) {
    for (int k = 1; k <= N; k++)
      for (int i = S->istr; i <= S->iend; i++) {
        WI(i, j, k) = WI(i, j, k - 1) - FLXU(i + 1, j, k) + FLXU(i, j, k) - FLXV(i, j + 1, k) + FLXV(i, j, k);
        if (S->pipe_source && A2(S->pipe_idx, i, j) > 0) {  /* omega.F:102-108: pipe_prf(pidx,k) */
          const int pidx = (int)A2(S->pipe_idx, i, j);
          WI(i, j, k) = WI(i, j, k) + A2(S->pipe_flx, i, j) * S->pipe_prf[(pidx - 1) + (size_t)S->npip * (k - 1)];
        }
        C1(CX, i, k) = fmax0(FLXU(i + 1, j, k)) - fmin0(FLXU(i, j, k)) + fmax0(FLXV(i, j + 1, k)) -
                       fmin0(FLXV(i, j, k));
      }
    for (int i = 1; i <= S->Lm; i++)
      WI(i, j, N) = WI(i, j, N) + A2(S->swflx, i, j) * A2(S->dm_r, i, j) * A2(S->dn_r, i, j);
    for (int i = S->istr; i <= S->iend; i++) {
      C1(wrk, i, 0) = WI(i, j, N) / (ZW(i, j, N) - ZW(i, j, 0));
      WI(i, j, N) = 0.0;
      WE(i, j, N) = 0.0;
      WE(i, j, 0) = 0.0;
      C1(CX, i, 0) = dtau * A2(S->pm, i, j) * A2(S->pn, i, j);
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istr; i <= S->iend; i++) {
        WI(i, j, k) = WI(i, j, k) - C1(wrk, i, 0) * (ZW(i, j, k) - ZW(i, j, 0));
        const double c2d = dmax(C1(CX, i, k), C1(CX, i, k + 1));
        const double dh = dmin(HZ(i, j, k), HZ(i, j, k + 1));
        const double cw_max = cu_max * dh - c2d * C1(CX, i, 0);
        if (cw_max > 0.0) {
          const double cw_max2 = cw_max * cw_max;
          const double cw_min = cw_max * cmnx_ratio;
          const double cw = fabs(WI(i, j, k)) * C1(CX, i, 0);
          double cff;
          if (cw < cw_min) cff = cw_max2;
          else if (cw < cutoff * cw_max) cff = cw_max2 + r4cmx * ((cw - cw_min) * (cw - cw_min));
          else cff = cw_max * cw;
          WE(i, j, k) = cw_max2 * WI(i, j, k) / cff;
          WI(i, j, k) = WI(i, j, k) - WE(i, j, k);
        } else {
          WE(i, j, k) = 0.0;
        }
      }
  }
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  for (int k = 0; k <= N; k++) {
    if (S->west_edge) for (int j = jstr; j <= jend; j++) { WE(istr - 1, j, k) = WE(istr, j, k); WI(istr - 1, j, k) = WI(istr, j, k); }
    if (S->east_edge) for (int j = jstr; j <= jend; j++) { WE(iend + 1, j, k) = WE(iend, j, k); WI(iend + 1, j, k) = WI(iend, j, k); }
    if (S->south_edge) for (int i = istr; i <= iend; i++) { WE(i, jstr - 1, k) = WE(i, jstr, k); WI(i, jstr - 1, k) = WI(i, jstr, k); }
    if (S->north_edge) for (int i = istr; i <= iend; i++) { WE(i, jend + 1, k) = WE(i, jend, k); WI(i, jend + 1, k) = WI(i, jend, k); }
    if (S->west_edge && S->south_edge) { WE(istr - 1, jstr - 1, k) = WE(istr, jstr, k); WI(istr - 1, jstr - 1, k) = WI(istr, jstr, k); }
    if (S->west_edge && S->north_edge) { WE(istr - 1, jend + 1, k) = WE(istr, jend, k); WI(istr - 1, jend + 1, k) = WI(istr, jend, k); }
    if (S->east_edge && S->south_edge) { WE(iend + 1, jstr - 1, k) = WE(iend, jstr, k); WI(iend + 1, jstr - 1, k) = WI(iend, jstr, k); }
    if (S->east_edge && S->north_edge) { WE(iend + 1, jend + 1, k) = WE(iend, jend, k); WI(iend + 1, jend + 1, k) = WI(iend, jend, k); }
  }
  or_exch3(S, S->We, N + 1);
  or_exch3(S, S->Wi, N + 1);
}

/* ---------------------------------------------------------------------- */
/* rho_eos_tile (rho_eos.F:24-409): linear EOS or JM95 split EOS (DUKO_2001) */
/* ---------------------------------------------------------------------- */
void or_rho_eos(or_state *S, int tidx) {
  const int N = S->N;
  const double rho0 = S->rho0, g = S->g, qp2 = S->qp2;
  const int lmd = S->c.lmd;
  if (S->c.nonlin_eos) {
    const double r00 = 999.842594, r01 = 6.793952E-2, r02 = -9.095290E-3, r03 = 1.001685E-4,
                 r04 = -1.120083E-6, r05 = 6.536332E-9, r10 = 0.824493, r11 = -4.08990E-3,
                 r12 = 7.64380E-5, r13 = -8.24670E-7, r14 = 5.38750E-9, rS0 = -5.72466E-3,
                 rS1 = 1.02270E-4, rS2 = -1.65460E-6, r20 = 4.8314E-4, K00 = 19092.56,
                 K01 = 209.8925, K02 = -3.041638, K03 = -1.852732e-3, K04 = -1.361629e-5,
                 K10 = 104.4077, K11 = -6.500517, K12 = 0.1553190, K13 = 2.326469e-4,
                 KS0 = -5.587545, KS1 = +0.7390729, KS2 = -1.909078e-2;
    double Tt = 3.8, Ts = 34.5, sqrtTs = sqrt(Ts);
    const double K0_Duk = Tt * (K01 + Tt * (K02 + Tt * (K03 + Tt * K04))) +
                          Ts * (K10 + Tt * (K11 + Tt * (K12 + Tt * K13)) + sqrtTs * (KS0 + Tt * (KS1 + Tt * KS2)));
    const double dr00 = r00 - rho0;
    for (int j = S->jstrE; j <= S->jendE; j++) {
      for (int k = 1; k <= N; k++)
        for (int i = S->istrE; i <= S->iendE; i++) {
          Tt = TT(i, j, k, tidx, 1);
          Ts = TT(i, j, k, tidx, 2);
          sqrtTs = sqrt(dmax(0.0, Ts));
          const double rm = A2(S->rmask, i, j);
          R3(S->rho1, i, j, k) =
              (dr00 + Tt * (r01 + Tt * (r02 + Tt * (r03 + Tt * (r04 + Tt * r05)))) +
               Ts * (r10 + Tt * (r11 + Tt * (r12 + Tt * (r13 + Tt * r14))) + sqrtTs * (rS0 + Tt * (rS1 + Tt * rS2)) +
                     Ts * r20)) *
              rm;
          const double K0 = Tt * (K01 + Tt * (K02 + Tt * (K03 + Tt * K04))) +
                            Ts * (K10 + Tt * (K11 + Tt * (K12 + Tt * K13)) + sqrtTs * (KS0 + Tt * (KS1 + Tt * KS2)));
          R3(S->qp1, i, j, k) =
              0.1 * (rho0 + R3(S->rho1, i, j, k)) * (K0_Duk - K0) / ((K00 + K0) * (K00 + K0_Duk)) * rm;
        }
      if (lmd) {
        const double cff = g / rho0;
        for (int k = 1; k <= N - 1; k++)
          for (int i = S->istrE; i <= S->iendE; i++) {
            const double dpth = -0.5 * (ZR(i, j, k + 1) + ZR(i, j, k));
            W3(S->bvf, i, j, k) = -cff *
                                  (R3(S->rho1, i, j, k + 1) - R3(S->rho1, i, j, k) +
                                   (R3(S->qp1, i, j, k + 1) - R3(S->qp1, i, j, k)) * dpth * (1.0 - qp2 * dpth)) /
                                  (ZR(i, j, k + 1) - ZR(i, j, k)) * A2(S->rmask, i, j);
          }
        for (int i = S->istrE; i <= S->iendE; i++) {
          W3(S->bvf, i, j, N) = W3(S->bvf, i, j, N - 1);
          W3(S->bvf, i, j, 0) = W3(S->bvf, i, j, 1);
        }
      }
      /* VAR_RHO_2D */
      for (int i = S->istrE; i <= S->iendE; i++) {
        const double dpth = -ZR(i, j, N);
        const double cff =
            HZ(i, j, N) * (R3(S->rho1, i, j, N) + R3(S->qp1, i, j, N) * dpth * (1.0 - qp2 * dpth));
        A2(S->rhoS, i, j) = 0.5 * cff * HZ(i, j, N);
        A2(S->rhoA, i, j) = cff;
      }
      for (int k = N - 1; k >= 1; k--)
        for (int i = S->istrE; i <= S->iendE; i++) {
          const double dpth = -ZR(i, j, k);
          const double cff =
              HZ(i, j, k) * (R3(S->rho1, i, j, k) + R3(S->qp1, i, j, k) * dpth * (1.0 - qp2 * dpth));
          A2(S->rhoS, i, j) = A2(S->rhoS, i, j) + HZ(i, j, k) * (A2(S->rhoA, i, j) + 0.5 * cff);
          A2(S->rhoA, i, j) = A2(S->rhoA, i, j) + cff;
        }
      const double cff1 = 1.0 / rho0;
      for (int i = S->istrE; i <= S->iendE; i++) {
        const double cff = 1.0 / (ZW(i, j, N) - ZW(i, j, 0));
        A2(S->rhoA, i, j) = cff * cff1 * A2(S->rhoA, i, j);
        A2(S->rhoS, i, j) = 2.0 * cff * cff * cff1 * A2(S->rhoS, i, j);
      }
    }
    return;
  }
  /* linear EOS, rho (no SPLIT_EOS) */
  const int sal = S->c.salinity;
  for (int j = S->jstrE; j <= S->jendE; j++) {
    const double cff0 = sal ? (S->c.Tcoef * S->c.T0 - S->c.Scoef * S->c.S0) : (S->c.Tcoef * S->c.T0);
    for (int k = 1; k <= N; k++)
      for (int i = S->istrE; i <= S->iendE; i++) {
        double r = cff0 - S->c.Tcoef * TT(i, j, k, tidx, 1);
        if (sal) r = r + S->c.Scoef * TT(i, j, k, tidx, 2);
        R3(S->rho, i, j, k) = r;
        R3(S->rho, i, j, k) = R3(S->rho, i, j, k) * A2(S->rmask, i, j);
      }
    if (lmd) {
      const double cff = g / rho0;
      for (int k = 1; k <= N - 1; k++)
        for (int i = S->istrE; i <= S->iendE; i++)
          W3(S->bvf, i, j, k) = cff * (R3(S->rho, i, j, k) - R3(S->rho, i, j, k + 1)) / (ZR(i, j, k + 1) - ZR(i, j, k));
      for (int i = S->istrE; i <= S->iendE; i++) {
        W3(S->bvf, i, j, N) = W3(S->bvf, i, j, N - 1);
        W3(S->bvf, i, j, 0) = W3(S->bvf, i, j, 1);
      }
    }
    for (int i = S->istrE; i <= S->iendE; i++) {
      const double cff = HZ(i, j, N) * R3(S->rho, i, j, N);
      A2(S->rhoS, i, j) = 0.5 * cff * HZ(i, j, N);
      A2(S->rhoA, i, j) = cff;
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istrE; i <= S->iendE; i++) {
        const double cff = HZ(i, j, k) * R3(S->rho, i, j, k);
        A2(S->rhoS, i, j) = A2(S->rhoS, i, j) + HZ(i, j, k) * (A2(S->rhoA, i, j) + 0.5 * cff);
        A2(S->rhoA, i, j) = A2(S->rhoA, i, j) + cff;
      }
    const double cff1 = 1.0 / rho0;
    for (int i = S->istrE; i <= S->iendE; i++) {
      const double cff = 1.0 / (ZW(i, j, N) - ZW(i, j, 0));
      A2(S->rhoA, i, j) = cff * cff1 * A2(S->rhoA, i, j);
      A2(S->rhoS, i, j) = 2.0 * cff * cff * cff1 * A2(S->rhoS, i, j);
    }
  }
}

/* ---------------------------------------------------------------------- */
/* prsgrd_tile (prsgrd.F:25-510): SM03 density-Jacobian pressure gradient  */
/* ---------------------------------------------------------------------- */
void or_prsgrd(or_state *S) {
  const int N = S->N, nx = S->Lm, ny = S->Mm;
  const int split = S->c.nonlin_eos;
  const double g = S->g, rho0 = S->rho0, qp2 = S->qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0, epsil = 0.0;
  double *dR = S->c1[0], *dZ = S->c1[1];
  double *FC = S->s2[0], *dZx = S->s2[1], *rx = S->s2[2], *dRx = S->s2[3];
  double *P = S->P, *ru = S->ru, *rv = S->rv;
  double *rho = split ? S->rhos3 : S->rho;
  int imin, imax, jmin, jmax;
  if (!S->c.ew_periodic) {
    imin = S->west_edge ? S->istrU : S->istrU - 1;
    imax = S->east_edge ? S->iend : S->iend + 1;
  } else {
    imin = S->istr - 1;
    imax = S->iend + 1;
  }
  if (!S->c.ns_periodic) {
    jmin = S->south_edge ? S->jstrV : S->jstrV - 1;
    jmax = S->north_edge ? S->jend : S->jend + 1;
  } else {
    jmin = S->jstr - 1;
    jmax = S->jend + 1;
  }
  const double grho = g / rho0, HalfGRho = 0.5 * grho;
  for (int j = 0; j <= ny; j++) {
    for (int k = 1; k <= N - 1; k++)
      for (int i = 0; i <= nx; i++) {
        C1(dZ, i, k) = ZR(i, j, k + 1) - ZR(i, j, k);
        if (split) {
          const double dpth = -0.5 * (ZR(i, j, k + 1) + ZR(i, j, k));
          C1(dR, i, k) = R3(S->rho1, i, j, k + 1) - R3(S->rho1, i, j, k) +
                         (R3(S->qp1, i, j, k + 1) - R3(S->qp1, i, j, k)) * dpth * (1.0 - qp2 * dpth);
        } else {
          C1(dR, i, k) = R3(S->rho, i, j, k + 1) - R3(S->rho, i, j, k);
        }
      }
    for (int i = 0; i <= nx; i++) {
      C1(dR, i, N) = C1(dR, i, N - 1);
      C1(dR, i, 0) = C1(dR, i, 1);
      C1(dZ, i, N) = C1(dZ, i, N - 1);
      C1(dZ, i, 0) = C1(dZ, i, 1);
    }
    for (int k = N; k >= 1; k--)
      for (int i = 0; i <= nx; i++) {
        const double cff = 2.0 * C1(dZ, i, k) * C1(dZ, i, k - 1);
        C1(dZ, i, k) = cff / (C1(dZ, i, k) + C1(dZ, i, k - 1));
        const double cfr = 2.0 * C1(dR, i, k) * C1(dR, i, k - 1);
        if (cfr > epsil) C1(dR, i, k) = cfr / (C1(dR, i, k) + C1(dR, i, k - 1));
        else C1(dR, i, k) = 0.0;
        if (split) {
          const double dpth = -ZR(i, j, k);
          C1(dR, i, k) = C1(dR, i, k) - R3(S->qp1, i, j, k) * C1(dZ, i, k) * (1.0 - 2.0 * qp2 * dpth);
          R3(rho, i, j, k) = R3(S->rho1, i, j, k) + R3(S->qp1, i, j, k) * dpth * (1.0 - qp2 * dpth);
        }
      }
    for (int i = S->istrU - 1; i <= S->iend; i++) {
      R3(P, i, j, N) = g * ZW(i, j, N) +
                       grho * (R3(rho, i, j, N) + 0.5 * (R3(rho, i, j, N) - R3(rho, i, j, N - 1)) *
                                                       (ZW(i, j, N) - ZR(i, j, N)) / (ZR(i, j, N) - ZR(i, j, N - 1))) *
                           (ZW(i, j, N) - ZR(i, j, N));
      if (S->c.pot_tides) R3(P, i, j, N) = R3(P, i, j, N) - g * A2(S->ptide, i, j);  /* prsgrd.F:209-211 */
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        R3(P, i, j, k) =
            R3(P, i, j, k + 1) +
            HalfGRho * ((R3(rho, i, j, k + 1) + R3(rho, i, j, k)) * (ZR(i, j, k + 1) - ZR(i, j, k)) -
                        OneFifth * ((C1(dR, i, k + 1) - C1(dR, i, k)) *
                                        (ZR(i, j, k + 1) - ZR(i, j, k) - OneTwelfth * (C1(dZ, i, k + 1) + C1(dZ, i, k))) -
                                    (C1(dZ, i, k + 1) - C1(dZ, i, k)) *
                                        (R3(rho, i, j, k + 1) - R3(rho, i, j, k) -
                                         OneTwelfth * (C1(dR, i, k + 1) + C1(dR, i, k)))));
      }
  }
  for (int k = N; k >= 1; k--) {
    /* XI component */
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = imin; i <= imax; i++) {
        A2(FC, i, j) = (ZR(i, j, k) - ZR(i - 1, j, k)) * A2(S->umask, i, j);
        if (split) {
          const double dpth = -0.5 * (ZR(i, j, k) + ZR(i - 1, j, k));
          A2(rx, i, j) = (R3(S->rho1, i, j, k) - R3(S->rho1, i - 1, j, k) +
                          (R3(S->qp1, i, j, k) - R3(S->qp1, i - 1, j, k)) * dpth * (1.0 - qp2 * dpth)) *
                         A2(S->umask, i, j);
        } else {
          A2(rx, i, j) = (R3(S->rho, i, j, k) - R3(S->rho, i - 1, j, k)) * A2(S->umask, i, j);
        }
      }
    if (!S->c.ew_periodic) {
      if (S->west_edge)
        for (int j = S->jstr; j <= S->jend; j++) { A2(FC, imin - 1, j) = A2(FC, imin, j); A2(rx, imin - 1, j) = A2(rx, imin, j); }
      if (S->east_edge)
        for (int j = S->jstr; j <= S->jend; j++) { A2(FC, imax + 1, j) = A2(FC, imax, j); A2(rx, imax + 1, j) = A2(rx, imax, j); }
    }
    for (int j = S->jstr; j <= S->jend; j++) {
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        const double cff = 2.0 * A2(FC, i, j) * A2(FC, i + 1, j);
        if (cff > epsil) A2(dZx, i, j) = cff / (A2(FC, i, j) + A2(FC, i + 1, j));
        else A2(dZx, i, j) = 0.0;
        const double cfr = 2.0 * A2(rx, i, j) * A2(rx, i + 1, j);
        if (cfr > epsil) A2(dRx, i, j) = cfr / (A2(rx, i, j) + A2(rx, i + 1, j));
        else A2(dRx, i, j) = 0.0;
        if (split) A2(dRx, i, j) = A2(dRx, i, j) - R3(S->qp1, i, j, k) * A2(dZx, i, j) * (1.0 + 2.0 * qp2 * ZR(i, j, k));
      }
      for (int i = S->istrU; i <= S->iend; i++) {
        R3(ru, i, j, k) =
            0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j) *
            (R3(P, i - 1, j, k) - R3(P, i, j, k) -
             HalfGRho * ((R3(rho, i, j, k) + R3(rho, i - 1, j, k)) * (ZR(i, j, k) - ZR(i - 1, j, k)) -
                         OneFifth * ((A2(dRx, i, j) - A2(dRx, i - 1, j)) *
                                         (ZR(i, j, k) - ZR(i - 1, j, k) - OneTwelfth * (A2(dZx, i, j) + A2(dZx, i - 1, j))) -
                                     (A2(dZx, i, j) - A2(dZx, i - 1, j)) *
                                         (R3(rho, i, j, k) - R3(rho, i - 1, j, k) -
                                          OneTwelfth * (A2(dRx, i, j) + A2(dRx, i - 1, j))))));
      }
    }
    /* ADV_ISONEUTRAL, corrector stage: slopes dRdx from this k's rx (prsgrd.F:307-338) */
    const int iso = S->c.adv_isoneutral && S->nrhs == 3;
    if (iso) or_iso_dRdx(S, k, rx, imin, imax);
    /* ETA component */
    for (int j = jmin; j <= jmax; j++)
      for (int i = S->istr; i <= S->iend; i++) {
        A2(FC, i, j) = (ZR(i, j, k) - ZR(i, j - 1, k)) * A2(S->vmask, i, j);
        if (split) {
          const double dpth = -0.5 * (ZR(i, j, k) + ZR(i, j - 1, k));
          A2(rx, i, j) = (R3(S->rho1, i, j, k) - R3(S->rho1, i, j - 1, k) +
                          (R3(S->qp1, i, j, k) - R3(S->qp1, i, j - 1, k)) * dpth * (1.0 - qp2 * dpth)) *
                         A2(S->vmask, i, j);
        } else {
          A2(rx, i, j) = (R3(S->rho, i, j, k) - R3(S->rho, i, j - 1, k)) * A2(S->vmask, i, j);
        }
      }
    if (!S->c.ns_periodic) {
      if (S->south_edge)
        for (int i = S->istr; i <= S->iend; i++) { A2(FC, i, jmin - 1) = A2(FC, i, jmin); A2(rx, i, jmin - 1) = A2(rx, i, jmin); }
      if (S->north_edge)
        for (int i = S->istr; i <= S->iend; i++) { A2(FC, i, jmax + 1) = A2(FC, i, jmax); A2(rx, i, jmax + 1) = A2(rx, i, jmax); }
    }
    for (int j = S->jstrV - 1; j <= S->jend; j++) {
      for (int i = S->istr; i <= S->iend; i++) {
        const double cff = 2.0 * A2(FC, i, j) * A2(FC, i, j + 1);
        if (cff > epsil) A2(dZx, i, j) = cff / (A2(FC, i, j) + A2(FC, i, j + 1));
        else A2(dZx, i, j) = 0.0;
        const double cfr = 2.0 * A2(rx, i, j) * A2(rx, i, j + 1);
        if (cfr > epsil) A2(dRx, i, j) = cfr / (A2(rx, i, j) + A2(rx, i, j + 1));
        else A2(dRx, i, j) = 0.0;
        if (split) A2(dRx, i, j) = A2(dRx, i, j) - R3(S->qp1, i, j, k) * A2(dZx, i, j) * (1.0 + 2.0 * qp2 * ZR(i, j, k));
      }
      if (j >= S->jstrV)
        for (int i = S->istr; i <= S->iend; i++) {
          R3(rv, i, j, k) =
              0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j) *
              (R3(P, i, j - 1, k) - R3(P, i, j, k) -
               HalfGRho * ((R3(rho, i, j, k) + R3(rho, i, j - 1, k)) * (ZR(i, j, k) - ZR(i, j - 1, k)) -
                           OneFifth * ((A2(dRx, i, j) - A2(dRx, i, j - 1)) *
                                           (ZR(i, j, k) - ZR(i, j - 1, k) - OneTwelfth * (A2(dZx, i, j) + A2(dZx, i, j - 1))) -
                                       (A2(dZx, i, j) - A2(dZx, i, j - 1)) *
                                           (R3(rho, i, j, k) - R3(rho, i, j - 1, k) -
                                            OneTwelfth * (A2(dRx, i, j) + A2(dRx, i, j - 1))))));
        }
    }
    if (iso) or_iso_dRde(S, k, rx, jmin, jmax);   /* prsgrd.F:423-453 */
  }
  if (S->c.adv_isoneutral && S->nrhs == 3) or_iso_exch_slopes(S);   /* step3d_uv1.F:529-532 */
}

/* ---------------------------------------------------------------------- */
/* compute_horiz_tracer_fluxes.h (4th-order centred, or UPSTREAM_TS)       */
/* ---------------------------------------------------------------------- */
static void horiz_tracer_fluxes(or_state *S, int k, int itrc, int tl, int upstream, double *FX, double *FE,
                                double *wrk) {
  int imin, imax, jmin, jmax;
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  if (!S->c.ew_periodic) {
    imin = S->west_edge ? istr : istr - 1;
    imax = S->east_edge ? iend : iend + 1;
  } else { imin = istr - 1; imax = iend + 1; }
  for (int j = jstr; j <= jend; j++)
    for (int i = imin; i <= imax + 1; i++)
      A2(FX, i, j) = (TT(i, j, k, tl, itrc) - TT(i - 1, j, k, tl, itrc)) * A2(S->umask, i, j);
  if (!S->c.ew_periodic) {
    if (S->west_edge) for (int j = jstr; j <= jend; j++) A2(FX, istr - 1, j) = A2(FX, istr, j);
    if (S->east_edge) for (int j = jstr; j <= jend; j++) A2(FX, iend + 2, j) = A2(FX, iend + 1, j);
  }
  for (int j = jstr; j <= jend; j++)
    for (int i = istr - 1; i <= iend + 1; i++) {
      if (upstream) A2(wrk, i, j) = A2(FX, i + 1, j) - A2(FX, i, j);
      else A2(wrk, i, j) = 0.5 * (A2(FX, i + 1, j) + A2(FX, i, j));
    }
  for (int j = jstr; j <= jend; j++)
    for (int i = istr; i <= iend + 1; i++) {
      const double t0 = TT(i, j, k, tl, itrc), tm = TT(i - 1, j, k, tl, itrc), F = FLXU(i, j, k);
      if (upstream)
        A2(FX, i, j) = 0.5 * (t0 + tm) * F - 0.1666666666666666 * (A2(wrk, i - 1, j) * fmax0(F) + A2(wrk, i, j) * fmin0(F));
      else
        A2(FX, i, j) = 0.5 * (t0 + tm - 0.3333333333333333 * (A2(wrk, i, j) - A2(wrk, i - 1, j))) * F;
    }
  if (!S->c.ns_periodic) {
    jmin = S->south_edge ? jstr : jstr - 1;
    jmax = S->north_edge ? jend : jend + 1;
  } else { jmin = jstr - 1; jmax = jend + 1; }
  for (int j = jmin; j <= jmax + 1; j++)
    for (int i = istr; i <= iend; i++)
      A2(FE, i, j) = (TT(i, j, k, tl, itrc) - TT(i, j - 1, k, tl, itrc)) * A2(S->vmask, i, j);
  if (!S->c.ns_periodic) {
    if (S->south_edge) for (int i = istr; i <= iend; i++) A2(FE, i, jstr - 1) = A2(FE, i, jstr);
    if (S->north_edge) for (int i = istr; i <= iend; i++) A2(FE, i, jend + 2) = A2(FE, i, jend + 1);
  }
  for (int j = jstr - 1; j <= jend + 1; j++)
    for (int i = istr; i <= iend; i++) {
      if (upstream) A2(wrk, i, j) = A2(FE, i, j + 1) - A2(FE, i, j);
      else A2(wrk, i, j) = 0.5 * (A2(FE, i, j + 1) + A2(FE, i, j));
    }
  for (int j = jstr; j <= jend + 1; j++)
    for (int i = istr; i <= iend; i++) {
      const double t0 = TT(i, j, k, tl, itrc), tm = TT(i, j - 1, k, tl, itrc), F = FLXV(i, j, k);
      if (upstream)
        A2(FE, i, j) = 0.5 * (t0 + tm) * F - 0.1666666666666666 * (A2(wrk, i, j - 1) * fmax0(F) + A2(wrk, i, j) * fmin0(F));
      else
        A2(FE, i, j) = 0.5 * (t0 + tm - 0.3333333333333333 * (A2(wrk, i, j) - A2(wrk, i, j - 1))) * F;
    }  if (S->river_source) {  /* compute_horiz_tracer_fluxes.h:217-246: river tracer inflow */
    const int N = S->N;
    for (int j = jstr; j <= jend; j++)
      for (int i = istr; i <= iend + 1; i++)
        if (fabs(A2(S->riv_uflx, i, j)) > 1e-3) {
          const double riv_depth = 0.5 * (ZW(i - 1, j, N) - ZW(i - 1, j, 0) + ZW(i, j, N) - ZW(i, j, 0));
          const int iriver = (int)lround(A2(S->riv_uflx, i, j) / 10);
          const double riv_uvel = S->riv_vol[iriver - 1] * (A2(S->riv_uflx, i, j) - 10 * iriver) / riv_depth;
          A2(FX, i, j) = S->riv_trc[(iriver - 1) + (itrc - 1) * S->nriv] * 0.5 * (HZ(i - 1, j, k) + HZ(i, j, k)) * riv_uvel;
        }
    for (int j = jstr; j <= jend + 1; j++)
      for (int i = istr; i <= iend; i++)
        if (fabs(A2(S->riv_vflx, i, j)) > 1e-3) {
          const double riv_depth = 0.5 * (ZW(i, j - 1, N) - ZW(i, j - 1, 0) + ZW(i, j, N) - ZW(i, j, 0));
          const int iriver = (int)lround(A2(S->riv_vflx, i, j) / 10);
          const double riv_vvel = S->riv_vol[iriver - 1] * (A2(S->riv_vflx, i, j) - 10 * iriver) / riv_depth;
          A2(FE, i, j) = S->riv_trc[(iriver - 1) + (itrc - 1) * S->nriv] * 0.5 * (HZ(i, j - 1, k) + HZ(i, j, k)) * riv_vvel;
        }
  }
}

/* compute_vert_tracer_fluxes.h, SPLINE_TS with natural b.c. */
static void vert_tracer_fluxes(or_state *S, int j, int itrc, int tl, double *FC, double *CF, const double *Hz) {
  const int N = S->N;
  for (int i = S->istr; i <= S->iend; i++) {
    C1(CF, i, 1) = 1.0;
    C1(FC, i, 0) = 2.0 * TT(i, j, 1, tl, itrc);
  }
  for (int k = 1; k <= N - 1; k++)
    for (int i = S->istr; i <= S->iend; i++) {
      const double hk = R3(Hz, i, j, k), hk1 = R3(Hz, i, j, k + 1);
      const double cff = 1.0 / (2.0 * hk + hk1 * (2.0 - C1(CF, i, k)));
      C1(CF, i, k + 1) = cff * hk;
      C1(FC, i, k) = cff * (3.0 * (hk * TT(i, j, k + 1, tl, itrc) + hk1 * TT(i, j, k, tl, itrc)) - hk1 * C1(FC, i, k - 1));
    }
  for (int i = S->istr; i <= S->iend; i++)
    C1(FC, i, N) = (2.0 * TT(i, j, N, tl, itrc) - C1(FC, i, N - 1)) / (1.0 - C1(CF, i, N));
  for (int k = N - 1; k >= 0; k--)
    for (int i = S->istr; i <= S->iend; i++) {
      C1(FC, i, k) = C1(FC, i, k) - C1(CF, i, k + 1) * C1(FC, i, k + 1);
      C1(FC, i, k + 1) = C1(FC, i, k + 1) * WE(i, j, k + 1);
    }
  for (int i = S->istr; i <= S->iend; i++) {
    C1(FC, i, N) = 0.0;
    C1(FC, i, 0) = 0.0;
  }
}

/* compute_horiz_rhs_uv_terms.h (UV_COR + UV_ADV; centred or UPSTREAM_UV)  */
static void horiz_rhs_uv(or_state *S, int k, int upstream, double *ru, double *rv) {
  const int nr = S->nrhs, istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const int istrU = S->istrU, jstrV = S->jstrV;
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  double *UFx = S->s2[4], *UFe = S->s2[5], *VFx = S->s2[6], *VFe = S->s2[7], *wrk1 = S->s2[8], *wrk2 = S->s2[9];
  int imin, imax, jmin, jmax;
  const int ucor = S->c.uv_cor, curv = S->c.curvgrid && S->c.uv_adv;
  /* Coriolis (UV_COR) and/or the CURVGRID && UV_ADV curvature terms */
  if (ucor || curv) {
    for (int j = jstrV - 1; j <= jend; j++)
      for (int i = istrU - 1; i <= iend; i++) {
        /* compute_horiz_rhs_uv_terms.h:4-12 */
        double cff;
        if (curv) {
          const double ct = 0.5 * ((V(i, j, k, nr) + V(i, j + 1, k, nr)) * A2(S->dndx, i, j) -
                                   (U(i, j, k, nr) + U(i + 1, j, k, nr)) * A2(S->dmde, i, j));
          cff = 0.5 * HZ(i, j, k) * (ucor ? A2(S->fomn, i, j) + ct : ct);
        } else {
          cff = 0.5 * HZ(i, j, k) * (A2(S->fomn, i, j));
        }
        A2(UFx, i, j) = cff * (V(i, j, k, nr) + V(i, j + 1, k, nr));
        A2(VFe, i, j) = cff * (U(i, j, k, nr) + U(i + 1, j, k, nr));
      }
    for (int j = jstr; j <= jend; j++)
      for (int i = istrU; i <= iend; i++) R3(ru, i, j, k) = R3(ru, i, j, k) + 0.5 * (A2(UFx, i, j) + A2(UFx, i - 1, j));
    for (int j = jstrV; j <= jend; j++)
      for (int i = istr; i <= iend; i++) R3(rv, i, j, k) = R3(rv, i, j, k) - 0.5 * (A2(VFe, i, j) + A2(VFe, i, j - 1));
  }
  if (!S->c.uv_adv) return;  /* compute_horiz_rhs_uv_terms.h:42 */
  /* advection: UFx */
  if (!S->c.ew_periodic) {
    imin = S->west_edge ? istrU : istrU - 1;
    imax = S->east_edge ? iend : iend + 1;
  } else { imin = istr - 1; imax = iend + 1; }
  double *uxx = wrk1, *Huxx = wrk2;
  for (int j = jstr; j <= jend; j++)
    for (int i = imin; i <= imax; i++) {
      A2(uxx, i, j) = U(i - 1, j, k, nr) - 2.0 * U(i, j, k, nr) + U(i + 1, j, k, nr);
      A2(Huxx, i, j) = FLXU(i - 1, j, k) - 2.0 * FLXU(i, j, k) + FLXU(i + 1, j, k);
    }
  if (!S->c.ew_periodic) {
    if (S->west_edge) for (int j = jstr; j <= jend; j++) { A2(uxx, istrU - 1, j) = A2(uxx, istrU, j); A2(Huxx, istrU - 1, j) = A2(Huxx, istrU, j); }
    if (S->east_edge) for (int j = jstr; j <= jend; j++) { A2(uxx, iend + 1, j) = A2(uxx, iend, j); A2(Huxx, iend + 1, j) = A2(Huxx, iend, j); }
  }
  for (int j = jstr; j <= jend; j++)
    for (int i = istrU - 1; i <= iend; i++) {
      if (upstream) {
        const double cff = FLXU(i, j, k) + FLXU(i + 1, j, k) - delta * (A2(Huxx, i, j) + A2(Huxx, i + 1, j));
        A2(UFx, i, j) = 0.25 * (cff * (U(i, j, k, nr) + U(i + 1, j, k, nr)) -
                                gamma * (fmax0(cff) * A2(uxx, i, j) + fmin0(cff) * A2(uxx, i + 1, j)));
      } else {
        A2(UFx, i, j) = 0.25 * (U(i, j, k, nr) + U(i + 1, j, k, nr) - delta * (A2(uxx, i, j) + A2(uxx, i + 1, j))) *
                        (FLXU(i, j, k) + FLXU(i + 1, j, k) - delta * (A2(Huxx, i, j) + A2(Huxx, i + 1, j)));
      }
    }
  /* VFe */
  if (!S->c.ns_periodic) {
    jmin = S->south_edge ? jstrV : jstrV - 1;
    jmax = S->north_edge ? jend : jend + 1;
  } else { jmin = jstr - 1; jmax = jend + 1; }
  double *vee = wrk1, *Hvee = wrk2;
  for (int j = jmin; j <= jmax; j++)
    for (int i = istr; i <= iend; i++) {
      A2(vee, i, j) = V(i, j - 1, k, nr) - 2.0 * V(i, j, k, nr) + V(i, j + 1, k, nr);
      A2(Hvee, i, j) = FLXV(i, j - 1, k) - 2.0 * FLXV(i, j, k) + FLXV(i, j + 1, k);
    }
  if (!S->c.ns_periodic) {
    if (S->south_edge) for (int i = istr; i <= iend; i++) { A2(vee, i, jstrV - 1) = A2(vee, i, jstrV); A2(Hvee, i, jstrV - 1) = A2(Hvee, i, jstrV); }
    if (S->north_edge) for (int i = istr; i <= iend; i++) { A2(vee, i, jend + 1) = A2(vee, i, jend); A2(Hvee, i, jend + 1) = A2(Hvee, i, jend); }
  }
  for (int j = jstrV - 1; j <= jend; j++)
    for (int i = istr; i <= iend; i++) {
      if (upstream) {
        const double cff = FLXV(i, j, k) + FLXV(i, j + 1, k) - delta * (A2(Hvee, i, j) + A2(Hvee, i, j + 1));
        A2(VFe, i, j) = 0.25 * (cff * (V(i, j, k, nr) + V(i, j + 1, k, nr)) -
                                gamma * (fmax0(cff) * A2(vee, i, j) + fmin0(cff) * A2(vee, i, j + 1)));
      } else {
        A2(VFe, i, j) = 0.25 * (V(i, j, k, nr) + V(i, j + 1, k, nr) - delta * (A2(vee, i, j) + A2(vee, i, j + 1))) *
                        (FLXV(i, j, k) + FLXV(i, j + 1, k) - delta * (A2(Hvee, i, j) + A2(Hvee, i, j + 1)));
      }
    }
  /* UFe */
  if (!S->c.ns_periodic) {
    jmin = S->south_edge ? jstr : jstr - 1;
    jmax = S->north_edge ? jend : jend + 1;
  } else { jmin = jstr - 1; jmax = jend + 1; }
  double *uee = wrk1, *Hvxx = wrk2;
  for (int j = jmin; j <= jmax; j++)
    for (int i = istrU; i <= iend; i++)
      A2(uee, i, j) = U(i, j - 1, k, nr) - 2.0 * U(i, j, k, nr) + U(i, j + 1, k, nr);
  if (!S->c.ns_periodic) {
    if (S->south_edge) for (int i = istrU; i <= iend; i++) A2(uee, i, jstr - 1) = A2(uee, i, jstr);
    if (S->north_edge) for (int i = istrU; i <= iend; i++) A2(uee, i, jend + 1) = A2(uee, i, jend);
  }
  for (int j = jstr; j <= jend + 1; j++)
    for (int i = istrU - 1; i <= iend; i++)
      A2(Hvxx, i, j) = FLXV(i - 1, j, k) - 2.0 * FLXV(i, j, k) + FLXV(i + 1, j, k);
  for (int j = jstr; j <= jend + 1; j++)
    for (int i = istrU; i <= iend; i++) {
      if (upstream) {
        const double cff = FLXV(i, j, k) + FLXV(i - 1, j, k) - delta * (A2(Hvxx, i, j) + A2(Hvxx, i - 1, j));
        A2(UFe, i, j) = 0.25 * (cff * (U(i, j, k, nr) + U(i, j - 1, k, nr)) -
                                gamma * (fmax0(cff) * A2(uee, i, j - 1) + fmin0(cff) * A2(uee, i, j)));
      } else {
        A2(UFe, i, j) = 0.25 * (U(i, j, k, nr) + U(i, j - 1, k, nr) - delta * (A2(uee, i, j) + A2(uee, i, j - 1))) *
                        (FLXV(i, j, k) + FLXV(i - 1, j, k) - delta * (A2(Hvxx, i, j) + A2(Hvxx, i - 1, j)));
      }
    }
  /* VFx */
  if (!S->c.ew_periodic) {
    imin = S->west_edge ? istr : istr - 1;
    imax = S->east_edge ? iend : iend + 1;
  } else { imin = istr - 1; imax = iend + 1; }
  double *vxx = wrk1, *Huee = wrk2;
  for (int j = jstrV; j <= jend; j++)
    for (int i = imin; i <= imax; i++)
      A2(vxx, i, j) = V(i - 1, j, k, nr) - 2.0 * V(i, j, k, nr) + V(i + 1, j, k, nr);
  if (!S->c.ew_periodic) {
    if (S->west_edge) for (int j = jstrV; j <= jend; j++) A2(vxx, istr - 1, j) = A2(vxx, istr, j);
    if (S->east_edge) for (int j = jstrV; j <= jend; j++) A2(vxx, iend + 1, j) = A2(vxx, iend, j);
  }
  for (int j = jstrV - 1; j <= jend; j++)
    for (int i = istr; i <= iend + 1; i++)
      A2(Huee, i, j) = FLXU(i, j - 1, k) - 2.0 * FLXU(i, j, k) + FLXU(i, j + 1, k);
  for (int j = jstrV; j <= jend; j++)
    for (int i = istr; i <= iend + 1; i++) {
      if (upstream) {
        const double cff = FLXU(i, j, k) + FLXU(i, j - 1, k) - delta * (A2(Huee, i, j) + A2(Huee, i, j - 1));
        A2(VFx, i, j) = 0.25 * (cff * (V(i, j, k, nr) + V(i - 1, j, k, nr)) -
                                gamma * (fmax0(cff) * A2(vxx, i - 1, j) + fmin0(cff) * A2(vxx, i, j)));
      } else {
        A2(VFx, i, j) = 0.25 * (V(i, j, k, nr) + V(i - 1, j, k, nr) - delta * (A2(vxx, i, j) + A2(vxx, i - 1, j))) *
                        (FLXU(i, j, k) + FLXU(i, j - 1, k) - delta * (A2(Huee, i, j) + A2(Huee, i, j - 1)));
      }
    }
  for (int j = jstr; j <= jend; j++)
    for (int i = istrU; i <= iend; i++)
      R3(ru, i, j, k) = R3(ru, i, j, k) - A2(UFx, i, j) + A2(UFx, i - 1, j) - A2(UFe, i, j + 1) + A2(UFe, i, j);
  for (int j = jstrV; j <= jend; j++)
    for (int i = istr; i <= iend; i++)
      R3(rv, i, j, k) = R3(rv, i, j, k) - A2(VFx, i + 1, j) + A2(VFx, i, j) - A2(VFe, i, j) + A2(VFe, i, j - 1);
}

/* compute_vert_rhs_uv_terms.h, SPLINE_UV, MASKING                         */
static void vert_rhs_uv(or_state *S, int j, double *ru, double *rv) {
  const int N = S->N, nr = S->nrhs;
  if (!S->c.uv_adv) return;  /* compute_vert_rhs_uv_terms.h:1 */
  double *DC = S->c1[3], *CF = S->c1[2], *FC = S->c1[1];
  for (int i = S->istrU; i <= S->iend; i++) {
    C1(DC, i, 1) = 0.5625 * (HZ(i, j, 1) + HZ(i - 1, j, 1)) - 0.0625 * (HZ(i + 1, j, 1) + HZ(i - 2, j, 1));
    C1(CF, i, 1) = 1.0;
    C1(FC, i, 0) = 2.0 * U(i, j, 1, nr);
  }
  for (int k = 1; k <= N - 1; k++)
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(DC, i, k + 1) = 0.5625 * (HZ(i, j, k + 1) + HZ(i - 1, j, k + 1)) - 0.0625 * (HZ(i + 1, j, k + 1) + HZ(i - 2, j, k + 1));
      const double cff = 1.0 / (2.0 * C1(DC, i, k) + C1(DC, i, k + 1) * (2.0 - C1(CF, i, k)));
      C1(CF, i, k + 1) = cff * C1(DC, i, k);
      C1(FC, i, k) = cff * (3.0 * (C1(DC, i, k) * U(i, j, k + 1, nr) + C1(DC, i, k + 1) * U(i, j, k, nr)) -
                            C1(DC, i, k + 1) * C1(FC, i, k - 1));
    }
  for (int i = S->istrU; i <= S->iend; i++) {
    C1(FC, i, N) = (2.0 * U(i, j, N, nr) - C1(FC, i, N - 1)) / (1.0 - C1(CF, i, N));
    C1(DC, i, N) = 0.0;
  }
  for (int k = N - 1; k >= 1; k--)
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(FC, i, k) = C1(FC, i, k) - C1(CF, i, k + 1) * C1(FC, i, k + 1);
      C1(DC, i, k) = C1(FC, i, k) * 0.5 *
                     (WE(i, j, k) + WE(i - 1, j, k) -
                      0.125 * ((WE(i + 1, j, k) - WE(i, j, k)) * A2(S->umask, i + 1, j) -
                               (WE(i - 1, j, k) - WE(i - 2, j, k)) * A2(S->umask, i - 1, j)));
      R3(ru, i, j, k + 1) = R3(ru, i, j, k + 1) - C1(DC, i, k + 1) + C1(DC, i, k);
    }
  for (int i = S->istrU; i <= S->iend; i++) R3(ru, i, j, 1) = R3(ru, i, j, 1) - C1(DC, i, 1);
  if (j >= S->jstrV) {
    for (int i = S->istr; i <= S->iend; i++) {
      C1(DC, i, 1) = 0.5625 * (HZ(i, j, 1) + HZ(i, j - 1, 1)) - 0.0625 * (HZ(i, j + 1, 1) + HZ(i, j - 2, 1));
      C1(CF, i, 1) = 1.0;
      C1(FC, i, 0) = 2.0 * V(i, j, 1, nr);
    }
    for (int k = 1; k <= N - 1; k++)
      for (int i = S->istr; i <= S->iend; i++) {
        C1(DC, i, k + 1) = 0.5625 * (HZ(i, j, k + 1) + HZ(i, j - 1, k + 1)) - 0.0625 * (HZ(i, j + 1, k + 1) + HZ(i, j - 2, k + 1));
        const double cff = 1.0 / (2.0 * C1(DC, i, k) + C1(DC, i, k + 1) * (2.0 - C1(CF, i, k)));
        C1(CF, i, k + 1) = cff * C1(DC, i, k);
        C1(FC, i, k) = cff * (3.0 * (C1(DC, i, k) * V(i, j, k + 1, nr) + C1(DC, i, k + 1) * V(i, j, k, nr)) -
                              C1(DC, i, k + 1) * C1(FC, i, k - 1));
      }
    for (int i = S->istr; i <= S->iend; i++) {
      C1(FC, i, N) = (2.0 * V(i, j, N, nr) - C1(FC, i, N - 1)) / (1.0 - C1(CF, i, N));
      C1(DC, i, N) = 0.0;
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istr; i <= S->iend; i++) {
        C1(FC, i, k) = C1(FC, i, k) - C1(CF, i, k + 1) * C1(FC, i, k + 1);
        C1(DC, i, k) = C1(FC, i, k) * 0.5 *
                       (WE(i, j, k) + WE(i, j - 1, k) -
                        0.125 * ((WE(i, j + 1, k) - WE(i, j, k)) * A2(S->vmask, i, j + 1) -
                                 (WE(i, j - 1, k) - WE(i, j - 2, k)) * A2(S->vmask, i, j - 1)));
        R3(rv, i, j, k + 1) = R3(rv, i, j, k + 1) - C1(DC, i, k + 1) + C1(DC, i, k);
      }
    for (int i = S->istr; i <= S->iend; i++) R3(rv, i, j, 1) = R3(rv, i, j, 1) - C1(DC, i, 1);
  }
}

/* ---------------------------------------------------------------------- */
/* pre_step3d_tile (pre_step3d4S.F:23-742), includes compute_rd_bott_drag.h */
/* ---------------------------------------------------------------------- */
/* river velocities in u,v(nnew) over the whole column (pre_step3d4S.F:493-522,
 * step3d_uv2.F:689-717; the u range is istrU..iend in the predictor and
 * istr..iend in the corrector, which differ only at a western wall face) */
static void river_uv(or_state *S, int nnew, int iu0) {
  const int N = S->N;
  for (int j = S->jstr; j <= S->jend; j++)
    for (int i = iu0; i <= S->iend; i++)
      if (fabs(A2(S->riv_uflx, i, j)) > 1e-3) {
        const double riv_depth = 0.5 * (ZW(i - 1, j, N) - ZW(i - 1, j, 0) + ZW(i, j, N) - ZW(i, j, 0));
        const int iriver = (int)lround(A2(S->riv_uflx, i, j) / 10);
        const double riv_uvel = S->riv_vol[iriver - 1] * (A2(S->riv_uflx, i, j) - 10 * iriver) / (A2(S->dn_u, i, j) * riv_depth);
        for (int k = 1; k <= N; k++) U(i, j, k, nnew) = riv_uvel;
      }
  for (int j = (iu0 == S->istrU ? S->jstrV : S->jstr); j <= S->jend; j++)
    for (int i = S->istr; i <= S->iend; i++)
      if (fabs(A2(S->riv_vflx, i, j)) > 1e-3) {
        const double riv_depth = 0.5 * (ZW(i, j - 1, N) - ZW(i, j - 1, 0) + ZW(i, j, N) - ZW(i, j, 0));
        const int iriver = (int)lround(A2(S->riv_vflx, i, j) / 10);
        const double riv_vvel = S->riv_vol[iriver - 1] * (A2(S->riv_vflx, i, j) - 10 * iriver) / (A2(S->dm_v, i, j) * riv_depth);
        for (int k = 1; k <= N; k++) V(i, j, k, nnew) = riv_vvel;
      }
}

void or_pre_step3d(or_state *S) {
  const int N = S->N, NT = S->NT, nstp = S->nstp, nnew = S->nnew, indx = 3 - nstp;
  const double AM3_crv = 1.0 / 6.0;
  double dtau, cf_stp, cf_bak;
  double *ru = S->ru, *rv = S->rv;
  double *Hz_bak = S->P, *Hz_fwd = S->rhos3; /* scratch A3d(:,3..4) */
  double *FX = S->s2[4], *FE = S->s2[7], *wrk1 = S->s2[8], *rd = S->s2[10];
  double *WC = S->c1[0], *FC = S->c1[1], *CF = S->c1[2], *DC = S->c1[3];
  if (S->iic == S->forw_start) { dtau = 0.5 * S->dt; cf_stp = 1.0; cf_bak = 0.0; }
  else { dtau = S->dt * (1.0 - AM3_crv); cf_stp = 0.5 + AM3_crv; cf_bak = 0.5 - AM3_crv; }
  for (int k = 1; k <= N; k++) {
    const double cff = 0.5 * dtau;
    for (int j = S->jstrV - 1; j <= S->jend; j++)
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        const double FlxDiv = cff * A2(S->pm, i, j) * A2(S->pn, i, j) *
                              (FLXU(i + 1, j, k) - FLXU(i, j, k) + FLXV(i, j + 1, k) - FLXV(i, j, k) + WE(i, j, k) +
                               WI(i, j, k) - WE(i, j, k - 1) - WI(i, j, k - 1));
        R3(Hz_bak, i, j, k) = HZ(i, j, k) + FlxDiv;
        R3(Hz_fwd, i, j, k) = HZ(i, j, k) - FlxDiv;
      }
    for (int itrc = 1; itrc <= NT; itrc++) {
      horiz_tracer_fluxes(S, k, itrc, S->nrhs, 0, FX, FE, wrk1);
      for (int j = S->jstr; j <= S->jend; j++)
        for (int i = S->istr; i <= S->iend; i++) {
          TT(i, j, k, nnew, itrc) =
              R3(Hz_bak, i, j, k) * (cf_stp * TT(i, j, k, nstp, itrc) + cf_bak * TT(i, j, k, indx, itrc)) -
              dtau * A2(S->pm, i, j) * A2(S->pn, i, j) *
                  (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j));
          TT(i, j, k, indx, itrc) = HZ(i, j, k) * TT(i, j, k, nstp, itrc);
        }
    }
    horiz_rhs_uv(S, k, 0, ru, rv);
  }
  /* compute_rd_bott_drag.h */
  if (S->c.Zob > 0.0) {
    for (int j = S->jstrV - 1; j <= S->jend; j++)
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        const double u0 = U(i, j, 1, nstp), u1 = U(i + 1, j, 1, nstp), v0 = V(i, j, 1, nstp), v1 = V(i, j + 1, 1, nstp);
        const double cff = sqrt(0.333333333333 * (u0 * u0 + u1 * u1 + u0 * u1 + v0 * v0 + v1 * v1 + v0 * v1));
        const double q = S->vonKar / log(1.0 + 0.5 * HZ(i, j, 1) / S->c.Zob);
        A2(rd, i, j) = cff * (q * q);
      }
  } else {
    for (int j = S->jstrV - 1; j <= S->jend; j++)
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        A2(rd, i, j) = S->c.rdrg;
        A2(rd, i, j) = dmin(A2(rd, i, j), 0.8 * HZ(i, j, 1) / S->dt);
      }
  }
  /* ext_copy_prv2shr_2d_tile: r_D over extended range (only the computed part is ever read) */
  for (int j = S->jstrE; j <= S->jendE; j++)
    for (int i = S->istrE; i <= S->iendE; i++) A2(S->r_D, i, j) = A2(rd, i, j);

  for (int j = S->jstr; j <= S->jend; j++) {
    for (int itrc = 1; itrc <= NT; itrc++) {
      vert_tracer_fluxes(S, j, itrc, S->nrhs, FC, CF, S->Hz);
      for (int k = 1; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, k, nnew, itrc) =
              TT(i, j, k, nnew, itrc) - dtau * A2(S->pm, i, j) * A2(S->pn, i, j) * (C1(FC, i, k) - C1(FC, i, k - 1));
      const int iAkt = itrc < S->nTS ? itrc : S->nTS;
      for (int i = S->istr; i <= S->iend; i++) {
        C1(FC, i, 1) = 2.0 * dtau * AKT(i, j, 1, iAkt) / (R3(Hz_fwd, i, j, 2) + R3(Hz_fwd, i, j, 1));
        C1(DC, i, 0) = dtau * A2(S->pm, i, j) * A2(S->pn, i, j);
        C1(WC, i, 1) = C1(DC, i, 0) * WI(i, j, 1);
        const double cff = 1.0 / (R3(Hz_fwd, i, j, 1) + C1(FC, i, 1) + fmax0(C1(WC, i, 1)));
        C1(CF, i, 1) = cff * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)));
        C1(DC, i, 1) = cff * TT(i, j, 1, nnew, itrc);
      }
      for (int k = 2; k <= N - 1; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(FC, i, k) = 2.0 * dtau * AKT(i, j, k, iAkt) / (R3(Hz_fwd, i, j, k + 1) + R3(Hz_fwd, i, j, k));
          C1(WC, i, k) = C1(DC, i, 0) * WI(i, j, k);
          const double cff = 1.0 / (R3(Hz_fwd, i, j, k) + C1(FC, i, k) + fmax0(C1(WC, i, k)) + C1(FC, i, k - 1) -
                                    fmin0(C1(WC, i, k - 1)) - C1(CF, i, k - 1) * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1))));
          C1(CF, i, k) = cff * (C1(FC, i, k) - fmin0(C1(WC, i, k)));
          C1(DC, i, k) = cff * (TT(i, j, k, nnew, itrc) + C1(DC, i, k - 1) * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1))));
        }
      for (int i = S->istr; i <= S->iend; i++)
        TT(i, j, N, nnew, itrc) =
            (TT(i, j, N, nnew, itrc) + C1(DC, i, N - 1) * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)))) /
            (R3(Hz_fwd, i, j, N) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)) -
             C1(CF, i, N - 1) * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1))));
      for (int k = N - 1; k >= 1; k--)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, k, nnew, itrc) = C1(DC, i, k) + C1(CF, i, k) * TT(i, j, k + 1, nnew, itrc);
    }
    vert_rhs_uv(S, j, ru, rv);
    /* u(nnew): implicit viscosity + no-slip bottom */
    for (int i = S->istrU; i <= S->iend; i++)
      C1(DC, i, 0) = dtau * 0.25 * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) * (A2(S->pn, i, j) + A2(S->pn, i - 1, j));
    for (int k = 1; k <= N; k++)
      for (int i = S->istrU; i <= S->iend; i++) {
        C1(DC, i, k) = 0.5 * (R3(Hz_bak, i, j, k) + R3(Hz_bak, i - 1, j, k)) *
                           (cf_stp * U(i, j, k, nstp) + cf_bak * U(i, j, k, indx)) +
                       C1(DC, i, 0) * R3(ru, i, j, k);
        U(i, j, k, indx) = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * U(i, j, k, nstp);
      }
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(FC, i, N - 1) = 2.0 * dtau * (AKV(i, j, N - 1) + AKV(i - 1, j, N - 1)) /
                         (R3(Hz_fwd, i, j, N) + R3(Hz_fwd, i - 1, j, N) + R3(Hz_fwd, i, j, N - 1) + R3(Hz_fwd, i - 1, j, N - 1));
      C1(WC, i, N - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, N - 1) + WI(i - 1, j, N - 1));
      const double cff = 1.0 / (0.5 * (R3(Hz_fwd, i, j, N) + R3(Hz_fwd, i - 1, j, N)) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)));
      C1(CF, i, N - 1) = cff * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)));
      C1(DC, i, N) = cff * (C1(DC, i, N) + dtau * A2(S->sustr, i, j));
    }
    for (int k = N - 1; k >= 2; k--)
      for (int i = S->istrU; i <= S->iend; i++) {
        C1(FC, i, k - 1) = 2.0 * dtau * (AKV(i, j, k - 1) + AKV(i - 1, j, k - 1)) /
                           (R3(Hz_fwd, i, j, k) + R3(Hz_fwd, i - 1, j, k) + R3(Hz_fwd, i, j, k - 1) + R3(Hz_fwd, i - 1, j, k - 1));
        C1(WC, i, k - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, k - 1) + WI(i - 1, j, k - 1));
        const double cff = 1.0 / (0.5 * (R3(Hz_fwd, i, j, k) + R3(Hz_fwd, i - 1, j, k)) + C1(FC, i, k - 1) -
                                  fmin0(C1(WC, i, k - 1)) + C1(FC, i, k) + fmax0(C1(WC, i, k)) -
                                  C1(CF, i, k) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
        C1(CF, i, k - 1) = cff * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1)));
        C1(DC, i, k) = cff * (C1(DC, i, k) + C1(DC, i, k + 1) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
      }
    for (int i = S->istrU; i <= S->iend; i++)
      U(i, j, 1, nnew) = (C1(DC, i, 1) + C1(DC, i, 2) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)))) /
                         (0.5 * (R3(Hz_fwd, i, j, 1) + R3(Hz_fwd, i - 1, j, 1)) + 0.5 * dtau * (A2(rd, i, j) + A2(rd, i - 1, j)) +
                          C1(FC, i, 1) + fmax0(C1(WC, i, 1)) - C1(CF, i, 1) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1))));
    for (int k = 2; k <= N; k++)
      for (int i = S->istrU; i <= S->iend; i++) U(i, j, k, nnew) = C1(DC, i, k) + C1(CF, i, k - 1) * U(i, j, k - 1, nnew);
    if (j >= S->jstrV) {
      for (int i = S->istr; i <= S->iend; i++)
        C1(DC, i, 0) = dtau * 0.25 * (A2(S->pm, i, j) + A2(S->pm, i, j - 1)) * (A2(S->pn, i, j) + A2(S->pn, i, j - 1));
      for (int k = 1; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(DC, i, k) = 0.5 * (R3(Hz_bak, i, j, k) + R3(Hz_bak, i, j - 1, k)) *
                             (cf_stp * V(i, j, k, nstp) + cf_bak * V(i, j, k, indx)) +
                         C1(DC, i, 0) * R3(rv, i, j, k);
          V(i, j, k, indx) = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * V(i, j, k, nstp);
        }
      for (int i = S->istr; i <= S->iend; i++) {
        C1(FC, i, N - 1) = 2.0 * dtau * (AKV(i, j, N - 1) + AKV(i, j - 1, N - 1)) /
                           (R3(Hz_fwd, i, j, N) + R3(Hz_fwd, i, j - 1, N) + R3(Hz_fwd, i, j, N - 1) + R3(Hz_fwd, i, j - 1, N - 1));
        C1(WC, i, N - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, N - 1) + WI(i, j - 1, N - 1));
        const double cff = 1.0 / (0.5 * (R3(Hz_fwd, i, j, N) + R3(Hz_fwd, i, j - 1, N)) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)));
        C1(CF, i, N - 1) = cff * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)));
        C1(DC, i, N) = cff * (C1(DC, i, N) + dtau * A2(S->svstr, i, j));
      }
      for (int k = N - 1; k >= 2; k--)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(FC, i, k - 1) = 2.0 * dtau * (AKV(i, j, k - 1) + AKV(i, j - 1, k - 1)) /
                             (R3(Hz_fwd, i, j, k) + R3(Hz_fwd, i, j - 1, k) + R3(Hz_fwd, i, j, k - 1) + R3(Hz_fwd, i, j - 1, k - 1));
          C1(WC, i, k - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, k - 1) + WI(i, j - 1, k - 1));
          const double cff = 1.0 / (0.5 * (R3(Hz_fwd, i, j, k) + R3(Hz_fwd, i, j - 1, k)) + C1(FC, i, k - 1) -
                                    fmin0(C1(WC, i, k - 1)) + C1(FC, i, k) + fmax0(C1(WC, i, k)) -
                                    C1(CF, i, k) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
          C1(CF, i, k - 1) = cff * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1)));
          C1(DC, i, k) = cff * (C1(DC, i, k) + C1(DC, i, k + 1) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
        }
      for (int i = S->istr; i <= S->iend; i++)
        V(i, j, 1, nnew) = (C1(DC, i, 1) + C1(DC, i, 2) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)))) /
                           (0.5 * (R3(Hz_fwd, i, j, 1) + R3(Hz_fwd, i, j - 1, 1)) + 0.5 * dtau * (A2(rd, i, j) + A2(rd, i, j - 1)) +
                            C1(FC, i, 1) + fmax0(C1(WC, i, 1)) - C1(CF, i, 1) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1))));
      for (int k = 2; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++) V(i, j, k, nnew) = C1(DC, i, k) + C1(CF, i, k - 1) * V(i, j, k - 1, nnew);
    }
  }
  if (S->river_source) river_uv(S, nnew, S->istrU);
  or_u3dbc(S);
  or_v3dbc(S);
  for (int itrc = 1; itrc <= NT; itrc++) {
    or_t3dbc(S, itrc);
    or_exch3(S, S->t + (size_t)(nnew - 1) * S->n3 + (size_t)(itrc - 1) * 3 * S->n3, N);
  }
}

/* ---------------------------------------------------------------------- */
/* step3d_uv1_tile (step3d_uv1.F:23-534), UPSTREAM_UV, IMPLICIT_BOTTOM_DRAG */
/* ---------------------------------------------------------------------- */
void or_step3d_uv1(or_state *S) {
  const int N = S->N, nnew = S->nnew;
  const double dt = S->dt;
  double *ru = S->ru, *rv = S->rv;
  double *WC = S->c1[0], *FC = S->c1[1], *CF = S->c1[2], *DC = S->c1[3];
  for (int k = 1; k <= N; k++) horiz_rhs_uv(S, k, 1, ru, rv);
  for (int j = S->jstr; j <= S->jend; j++) {
    vert_rhs_uv(S, j, ru, rv);
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(DC, i, 0) = dt * 0.25 * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) * (A2(S->pn, i, j) + A2(S->pn, i - 1, j));
      C1(FC, i, N - 1) = 2.0 * dt * (AKV(i, j, N - 1) + AKV(i - 1, j, N - 1)) /
                         (HZ(i, j, N) + HZ(i - 1, j, N) + HZ(i, j, N - 1) + HZ(i - 1, j, N - 1));
      C1(WC, i, N - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, N - 1) + WI(i - 1, j, N - 1));
      const double cff = 1.0 / (0.5 * (HZ(i, j, N) + HZ(i - 1, j, N)) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)));
      C1(CF, i, N - 1) = cff * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)));
      C1(DC, i, N) = cff * (U(i, j, N, nnew) + C1(DC, i, 0) * R3(ru, i, j, N) + dt * A2(S->sustr, i, j));
    }
    for (int k = N - 1; k >= 2; k--)
      for (int i = S->istrU; i <= S->iend; i++) {
        C1(FC, i, k - 1) = 2.0 * dt * (AKV(i, j, k - 1) + AKV(i - 1, j, k - 1)) /
                           (HZ(i, j, k) + HZ(i - 1, j, k) + HZ(i, j, k - 1) + HZ(i - 1, j, k - 1));
        C1(WC, i, k - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, k - 1) + WI(i - 1, j, k - 1));
        const double cff = 1.0 / (0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) + C1(FC, i, k - 1) - fmin0(C1(WC, i, k - 1)) +
                                  C1(FC, i, k) + fmax0(C1(WC, i, k)) - C1(CF, i, k) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
        C1(CF, i, k - 1) = cff * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1)));
        C1(DC, i, k) = cff * (U(i, j, k, nnew) + C1(DC, i, 0) * R3(ru, i, j, k) +
                              C1(DC, i, k + 1) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
      }
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(DC, i, 1) = (U(i, j, 1, nnew) + C1(DC, i, 0) * R3(ru, i, j, 1) + C1(DC, i, 2) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)))) /
                     (0.5 * (HZ(i, j, 1) + HZ(i - 1, j, 1)) + 0.5 * dt * (A2(S->r_D, i, j) + A2(S->r_D, i - 1, j)) +
                      C1(FC, i, 1) + fmax0(C1(WC, i, 1)) - C1(CF, i, 1) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1))));
      U(i, j, 1, nnew) = C1(DC, i, 1) * 0.5 * (HZ(i, j, 1) + HZ(i - 1, j, 1));
      A2(S->rufrc, i, j) = R3(ru, i, j, 1) + A2(S->dm_u, i, j) * A2(S->dn_u, i, j) *
                                                 (A2(S->sustr, i, j) - 0.5 * (A2(S->r_D, i - 1, j) + A2(S->r_D, i, j)) * C1(DC, i, 1));
    }
    for (int k = 2; k <= N; k++)
      for (int i = S->istrU; i <= S->iend; i++) {
        C1(DC, i, k) = C1(DC, i, k) + C1(CF, i, k - 1) * C1(DC, i, k - 1);
        U(i, j, k, nnew) = C1(DC, i, k) * 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k));
        A2(S->rufrc, i, j) = A2(S->rufrc, i, j) + R3(ru, i, j, k);
      }
    if (j >= S->jstrV) {
      for (int i = S->istr; i <= S->iend; i++) {
        C1(DC, i, 0) = dt * 0.25 * (A2(S->pm, i, j) + A2(S->pm, i, j - 1)) * (A2(S->pn, i, j) + A2(S->pn, i, j - 1));
        C1(FC, i, N - 1) = 2.0 * dt * (AKV(i, j, N - 1) + AKV(i, j - 1, N - 1)) /
                           (HZ(i, j, N) + HZ(i, j - 1, N) + HZ(i, j, N - 1) + HZ(i, j - 1, N - 1));
        C1(WC, i, N - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, N - 1) + WI(i, j - 1, N - 1));
        const double cff = 1.0 / (0.5 * (HZ(i, j, N) + HZ(i, j - 1, N)) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)));
        C1(CF, i, N - 1) = cff * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)));
        C1(DC, i, N) = cff * (V(i, j, N, nnew) + C1(DC, i, 0) * R3(rv, i, j, N) + dt * A2(S->svstr, i, j));
      }
      for (int k = N - 1; k >= 2; k--)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(FC, i, k - 1) = 2.0 * dt * (AKV(i, j, k - 1) + AKV(i, j - 1, k - 1)) /
                             (HZ(i, j, k) + HZ(i, j - 1, k) + HZ(i, j, k - 1) + HZ(i, j - 1, k - 1));
          C1(WC, i, k - 1) = C1(DC, i, 0) * 0.5 * (WI(i, j, k - 1) + WI(i, j - 1, k - 1));
          const double cff = 1.0 / (0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) + C1(FC, i, k - 1) - fmin0(C1(WC, i, k - 1)) +
                                    C1(FC, i, k) + fmax0(C1(WC, i, k)) - C1(CF, i, k) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
          C1(CF, i, k - 1) = cff * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1)));
          C1(DC, i, k) = cff * (V(i, j, k, nnew) + C1(DC, i, 0) * R3(rv, i, j, k) +
                                C1(DC, i, k + 1) * (C1(FC, i, k) - fmin0(C1(WC, i, k))));
        }
      for (int i = S->istr; i <= S->iend; i++) {
        C1(DC, i, 1) = (V(i, j, 1, nnew) + C1(DC, i, 0) * R3(rv, i, j, 1) + C1(DC, i, 2) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)))) /
                       (0.5 * (HZ(i, j, 1) + HZ(i, j - 1, 1)) + 0.5 * dt * (A2(S->r_D, i, j) + A2(S->r_D, i, j - 1)) +
                        C1(FC, i, 1) + fmax0(C1(WC, i, 1)) - C1(CF, i, 1) * (C1(FC, i, 1) - fmin0(C1(WC, i, 1))));
        V(i, j, 1, nnew) = C1(DC, i, 1) * 0.5 * (HZ(i, j, 1) + HZ(i, j - 1, 1));
        A2(S->rvfrc, i, j) = R3(rv, i, j, 1) + A2(S->dm_v, i, j) * A2(S->dn_v, i, j) *
                                                   (A2(S->svstr, i, j) - 0.5 * (A2(S->r_D, i, j - 1) + A2(S->r_D, i, j)) * C1(DC, i, 1));
      }
      for (int k = 2; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(DC, i, k) = C1(DC, i, k) + C1(CF, i, k - 1) * C1(DC, i, k - 1);
          V(i, j, k, nnew) = C1(DC, i, k) * 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k));
          A2(S->rvfrc, i, j) = A2(S->rvfrc, i, j) + R3(rv, i, j, k);
        }
    }
  }
}

/* ---------------------------------------------------------------------- */
/* visc3d_tile (visc3d_S.F:18-131): Laplacian viscosity along S            */
/* ---------------------------------------------------------------------- */
void or_visc3d(or_state *S) {
  const int N = S->N, nstp = S->nstp, indx = 3 - nstp;
  double *UFx = S->s2[4], *UFe = S->s2[5], *VFx = S->s2[6], *VFe = S->s2[7];
  const double *pm = S->pm, *pn = S->pn;
  for (int k = 1; k <= N; k++) {
    for (int j = S->jstrV - 1; j <= S->jend; j++)
      for (int i = S->istrU - 1; i <= S->iend; i++) {
        const double cff =
            0.5 * HZ(i, j, k) * A2(S->visc2_r, i, j) *
            (A2(S->dn_r, i, j) * A2(pm, i, j) *
                 ((A2(pn, i, j) + A2(pn, i + 1, j)) * U(i + 1, j, k, nstp) - (A2(pn, i - 1, j) + A2(pn, i, j)) * U(i, j, k, nstp)) -
             A2(S->dm_r, i, j) * A2(pn, i, j) *
                 ((A2(pm, i, j) + A2(pm, i, j + 1)) * V(i, j + 1, k, nstp) - (A2(pm, i, j - 1) + A2(pm, i, j)) * V(i, j, k, nstp)));
        A2(UFx, i, j) = cff * A2(S->dn_r, i, j) * A2(S->dn_r, i, j);
        A2(VFe, i, j) = -cff * A2(S->dm_r, i, j) * A2(S->dm_r, i, j);
      }
    for (int j = S->jstr; j <= S->jend + 1; j++)
      for (int i = S->istr; i <= S->iend + 1; i++) {
        const double cff =
            0.125 * (HZ(i - 1, j, k) + HZ(i, j, k) + HZ(i - 1, j - 1, k) + HZ(i, j - 1, k)) * A2(S->visc2_p, i, j) *
            (0.25 * (A2(pm, i - 1, j) + A2(pm, i, j) + A2(pm, i - 1, j - 1) + A2(pm, i, j - 1)) * A2(S->dn_p, i, j) *
                 ((A2(pn, i, j - 1) + A2(pn, i, j)) * V(i, j, k, nstp) - (A2(pn, i - 1, j - 1) + A2(pn, i - 1, j)) * V(i - 1, j, k, nstp)) +
             0.25 * (A2(pn, i - 1, j) + A2(pn, i, j) + A2(pn, i - 1, j - 1) + A2(pn, i, j - 1)) * A2(S->dm_p, i, j) *
                 ((A2(pm, i - 1, j) + A2(pm, i, j)) * U(i, j, k, nstp) - (A2(pm, i - 1, j - 1) + A2(pm, i, j - 1)) * U(i, j - 1, k, nstp))) *
            A2(S->pmask, i, j);
        A2(UFe, i, j) = cff * A2(S->dm_p, i, j) * A2(S->dm_p, i, j);
        A2(VFx, i, j) = cff * A2(S->dn_p, i, j) * A2(S->dn_p, i, j);
      }
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = S->istrU; i <= S->iend; i++) {
        const double cff = 0.125 * (A2(pm, i - 1, j) + A2(pm, i, j)) * (A2(pn, i - 1, j) + A2(pn, i, j)) *
                           ((A2(pn, i - 1, j) + A2(pn, i, j)) * (A2(UFx, i, j) - A2(UFx, i - 1, j)) +
                            (A2(pm, i - 1, j) + A2(pm, i, j)) * (A2(UFe, i, j + 1) - A2(UFe, i, j)));
        A2(S->rufrc, i, j) = A2(S->rufrc, i, j) + cff;
        U(i, j, k, indx) = U(i, j, k, indx) + S->dt * cff;
      }
    for (int j = S->jstrV; j <= S->jend; j++)
      for (int i = S->istr; i <= S->iend; i++) {
        const double cff = 0.125 * (A2(pm, i, j) + A2(pm, i, j - 1)) * (A2(pn, i, j) + A2(pn, i, j - 1)) *
                           ((A2(pn, i, j - 1) + A2(pn, i, j)) * (A2(VFx, i + 1, j) - A2(VFx, i, j)) +
                            (A2(pm, i, j - 1) + A2(pm, i, j)) * (A2(VFe, i, j) - A2(VFe, i, j - 1)));
        A2(S->rvfrc, i, j) = A2(S->rvfrc, i, j) + cff;
        V(i, j, k, indx) = V(i, j, k, indx) + S->dt * cff;
      }
  }
}

/* ---------------------------------------------------------------------- */
/* step2d_FB_tile (step2d_FB.F:24-576): generalized FB AB3-AM4 fast step   */
/* ---------------------------------------------------------------------- */
void or_step2d(or_state *S) {
  const int kstp = S->kstp, knew = S->knew, iif = S->iif;
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const int istrU = S->istrU, jstrV = S->jstrV;
  double *zeta_new = S->s2[0], *Dnew = S->s2[1], *rubar = S->s2[2], *rvbar = S->s2[3], *urhs = S->s2[4],
         *vrhs = S->s2[5], *DUon = S->s2[6], *DVom = S->s2[7], *Drhs = S->s2[8], *UFx = S->s2[9],
         *UFe = S->s2[10], *VFx = S->s2[11], *VFe = S->s2[12];
  const double *h = S->h;
  int kbak, kold;
  double fwd, fwd1, fwd2, bkw_new, bkw, bkw1, bkw2;
  if (iif == 1) {
    kbak = kstp; kold = kstp;
    fwd = 1.0; fwd1 = 0.0; fwd2 = 0.0;
    bkw_new = 0.0; bkw = 1.0; bkw1 = 0.0; bkw2 = 0.0;
  } else if (iif == 2) {
    kbak = kstp - 1; if (kbak < 1) kbak = 4;
    kold = kbak;
    fwd = 1.0; fwd1 = 0.0; fwd2 = 0.0;
    bkw_new = 1.0833333333333; bkw = -0.1666666666666; bkw1 = 0.0833333333333; bkw2 = 0.0;
  } else {
    kbak = kstp - 1; if (kbak < 1) kbak = 4;
    kold = kbak - 1; if (kold < 1) kold = 4;
    fwd = 1.781105; fwd1 = -1.06221; fwd2 = 0.281105;
    bkw_new = 0.614; bkw = 0.285; bkw1 = 0.088; bkw2 = 0.013;
  }
  for (int j = jstrV - 2; j <= jend + 1; j++)
    for (int i = istrU - 2; i <= iend + 1; i++)
      A2(Drhs, i, j) = A2(h, i, j) + fwd * ZETA(i, j, kstp) + fwd1 * ZETA(i, j, kbak) + fwd2 * ZETA(i, j, kold);
  for (int j = jstr - 1; j <= jend + 1; j++)
    for (int i = istrU - 1; i <= iend + 1; i++) {
      A2(urhs, i, j) = fwd * UBAR(i, j, kstp) + fwd1 * UBAR(i, j, kbak) + fwd2 * UBAR(i, j, kold);
      A2(DUon, i, j) = 0.5 * (A2(Drhs, i, j) + A2(Drhs, i - 1, j)) * A2(S->dn_u, i, j) * (A2(urhs, i, j));
    }
  for (int j = jstrV - 1; j <= jend + 1; j++)
    for (int i = istr - 1; i <= iend + 1; i++) {
      A2(vrhs, i, j) = fwd * VBAR(i, j, kstp) + fwd1 * VBAR(i, j, kbak) + fwd2 * VBAR(i, j, kold);
      A2(DVom, i, j) = 0.5 * (A2(Drhs, i, j) + A2(Drhs, i, j - 1)) * A2(S->dm_v, i, j) * (A2(vrhs, i, j));
    }
  double *zwrk = UFx, *rzeta = UFe, *rzeta2 = VFe, *rzetaSA = VFx;
  for (int j = jstrV - 1; j <= jend; j++)
    for (int i = istrU - 1; i <= iend; i++) {
      A2(zeta_new, i, j) = ZETA(i, j, kstp) + S->dtfast * A2(S->pm, i, j) * A2(S->pn, i, j) *
                                                  (A2(DUon, i, j) - A2(DUon, i + 1, j) + A2(DVom, i, j) - A2(DVom, i, j + 1)) +
                           S->dtfast * A2(S->swflx, i, j);
      if (S->pipe_source && A2(S->pipe_idx, i, j) > 0.)  /* step2d_FB.F:155-159 */
        A2(zeta_new, i, j) = A2(zeta_new, i, j) + S->dtfast * A2(S->pm, i, j) * A2(S->pn, i, j) * A2(S->pipe_flx, i, j);
      A2(zeta_new, i, j) = A2(zeta_new, i, j) * A2(S->rmask, i, j);
      A2(Dnew, i, j) = A2(zeta_new, i, j) + A2(h, i, j);
      A2(zwrk, i, j) = bkw_new * A2(zeta_new, i, j) + bkw * ZETA(i, j, kstp) + bkw1 * ZETA(i, j, kbak) + bkw2 * ZETA(i, j, kold);
      A2(rzeta, i, j) = (1.0 + A2(S->rhoS, i, j)) * A2(zwrk, i, j);
      A2(rzetaSA, i, j) = A2(zwrk, i, j) * (A2(S->rhoS, i, j) - A2(S->rhoA, i, j));
      A2(rzeta2, i, j) = A2(rzeta, i, j) * A2(zwrk, i, j);
    }
  or_zetabc(S, zeta_new);
  for (int j = S->jstrR; j <= S->jendR; j++)
    for (int i = S->istrR; i <= S->iendR; i++) ZETA(i, j, knew) = A2(zeta_new, i, j);
  {
    const double cff1 = S->weight[0][iif - 1], cff2 = S->weight[1][iif - 1];
    if (iif == 1) {
      for (int j = S->jstrR; j <= S->jendR; j++)
        for (int i = S->istrR; i <= S->iendR; i++) {
          A2(S->DU_avg_bak, i, j) = A2(S->DU_avg1, i, j) - 0.1024390243902439 * A2(S->DU_avg2, i, j);
          A2(S->DV_avg_bak, i, j) = A2(S->DV_avg1, i, j) - 0.1024390243902439 * A2(S->DV_avg2, i, j);
          A2(S->Zt_avg1, i, j) = cff1 * ZETA(i, j, knew);
          A2(S->DU_avg1, i, j) = 0.0;
          A2(S->DV_avg1, i, j) = 0.0;
          A2(S->DU_avg2, i, j) = cff2 * A2(DUon, i, j);
          A2(S->DV_avg2, i, j) = cff2 * A2(DVom, i, j);
        }
    } else {
      for (int j = S->jstrR; j <= S->jendR; j++)
        for (int i = S->istrR; i <= S->iendR; i++) {
          A2(S->Zt_avg1, i, j) = A2(S->Zt_avg1, i, j) + cff1 * ZETA(i, j, knew);
          A2(S->DU_avg2, i, j) = A2(S->DU_avg2, i, j) + cff2 * A2(DUon, i, j);
          A2(S->DV_avg2, i, j) = A2(S->DV_avg2, i, j) + cff2 * A2(DVom, i, j);
        }
    }
  }
  {
    const double cff = 0.5 * S->g;
    for (int j = jstr; j <= jend; j++)
      for (int i = istr; i <= iend; i++) {
        A2(rubar, i, j) =
            cff * A2(S->dn_u, i, j) *
            ((A2(h, i - 1, j) + A2(h, i, j)) * (A2(rzeta, i - 1, j) - A2(rzeta, i, j)) + A2(rzeta2, i - 1, j) - A2(rzeta2, i, j) +
             (A2(h, i - 1, j) - A2(h, i, j)) * (A2(rzetaSA, i - 1, j) + A2(rzetaSA, i, j) +
                                                0.333333333333 * (A2(S->rhoA, i - 1, j) - A2(S->rhoA, i, j)) *
                                                    (A2(zwrk, i - 1, j) - A2(zwrk, i, j))));
        A2(rvbar, i, j) =
            cff * A2(S->dm_v, i, j) *
            ((A2(h, i, j - 1) + A2(h, i, j)) * (A2(rzeta, i, j - 1) - A2(rzeta, i, j)) + A2(rzeta2, i, j - 1) - A2(rzeta2, i, j) +
             (A2(h, i, j - 1) - A2(h, i, j)) * (A2(rzetaSA, i, j - 1) + A2(rzetaSA, i, j) +
                                                0.333333333333 * (A2(S->rhoA, i, j - 1) - A2(S->rhoA, i, j)) *
                                                    (A2(zwrk, i, j - 1) - A2(zwrk, i, j))));
      }
  }
  if (iif == 1) {
    for (int j = jstr; j <= jend; j++)
      for (int i = istr; i <= iend; i++) {
        A2(S->rufrc, i, j) = A2(S->rufrc, i, j) - A2(rubar, i, j);
        A2(S->rvfrc, i, j) = A2(S->rvfrc, i, j) - A2(rvbar, i, j);
      }
    for (int j = jstrV - 1; j <= jend; j++)
      for (int i = istrU - 1; i <= iend; i++) {
        A2(zwrk, i, j) = A2(zeta_new, i, j) - ZETA(i, j, kstp);
        A2(rzeta, i, j) = (1.0 + A2(S->rhoS, i, j)) * A2(zwrk, i, j);
        A2(rzeta2, i, j) = A2(rzeta, i, j) * (A2(zeta_new, i, j) + ZETA(i, j, kstp));
        A2(rzetaSA, i, j) = A2(zwrk, i, j) * (A2(S->rhoS, i, j) - A2(S->rhoA, i, j));
      }
    const double cff = 0.5 * S->g;
    for (int j = jstr; j <= jend; j++)
      for (int i = istr; i <= iend; i++) {
        A2(rubar, i, j) =
            A2(rubar, i, j) +
            cff * A2(S->dn_u, i, j) *
                ((A2(h, i - 1, j) + A2(h, i, j)) * (A2(rzeta, i - 1, j) - A2(rzeta, i, j)) + A2(rzeta2, i - 1, j) - A2(rzeta2, i, j) +
                 (A2(h, i - 1, j) - A2(h, i, j)) * (A2(rzetaSA, i - 1, j) + A2(rzetaSA, i, j) +
                                                    0.333333333333 * (A2(S->rhoA, i - 1, j) - A2(S->rhoA, i, j)) *
                                                        (A2(zwrk, i - 1, j) - A2(zwrk, i, j))));
        A2(rvbar, i, j) =
            A2(rvbar, i, j) +
            cff * A2(S->dm_v, i, j) *
                ((A2(h, i, j - 1) + A2(h, i, j)) * (A2(rzeta, i, j - 1) - A2(rzeta, i, j)) + A2(rzeta2, i, j - 1) - A2(rzeta2, i, j) +
                 (A2(h, i, j - 1) - A2(h, i, j)) * (A2(rzetaSA, i, j - 1) + A2(rzetaSA, i, j) +
                                                    0.333333333333 * (A2(S->rhoA, i, j - 1) - A2(S->rhoA, i, j)) *
                                                        (A2(zwrk, i, j - 1) - A2(zwrk, i, j))));
      }
  }
  double *Dstp = DUon;
  for (int j = jstrV - 1; j <= jend; j++)
    for (int i = istrU - 1; i <= iend; i++) A2(Dstp, i, j) = ZETA(i, j, kstp) + A2(h, i, j);
  {
    const double cff = 0.5 * S->dtfast, cff1 = 0.5 * S->weight[0][iif - 1];
    for (int j = jstr; j <= jend; j++)
      for (int i = istrU; i <= iend; i++) {
        const double DUnew = ((A2(Dstp, i, j) + A2(Dstp, i - 1, j)) * UBAR(i, j, kstp) +
                              cff * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) * (A2(S->pn, i, j) + A2(S->pn, i - 1, j)) *
                                  (A2(rubar, i, j) + A2(S->rufrc, i, j))) *
                             A2(S->umask, i, j);
        UBAR(i, j, knew) = DUnew / (A2(Dnew, i, j) + A2(Dnew, i - 1, j));
        A2(S->DU_avg1, i, j) = A2(S->DU_avg1, i, j) + cff1 * A2(S->dn_u, i, j) * (DUnew);
      }
    for (int j = jstrV; j <= jend; j++)
      for (int i = istr; i <= iend; i++) {
        const double DVnew = ((A2(Dstp, i, j) + A2(Dstp, i, j - 1)) * VBAR(i, j, kstp) +
                              cff * (A2(S->pm, i, j) + A2(S->pm, i, j - 1)) * (A2(S->pn, i, j) + A2(S->pn, i, j - 1)) *
                                  (A2(rvbar, i, j) + A2(S->rvfrc, i, j))) *
                             A2(S->vmask, i, j);
        VBAR(i, j, knew) = DVnew / (A2(Dnew, i, j) + A2(Dnew, i, j - 1));
        A2(S->DV_avg1, i, j) = A2(S->DV_avg1, i, j) + cff1 * A2(S->dm_v, i, j) * (DVnew);
      }
  }
  or_u2dbc(S);
  or_v2dbc(S);
  /* fast-time-averaged barotropic fluxes along physical boundaries */
  if (S->west_edge) for (int j = jstr - 1; j <= S->jendR; j++) A2(Dnew, istr - 1, j) = A2(h, istr - 1, j) + A2(zeta_new, istr - 1, j);
  if (S->east_edge) for (int j = jstr - 1; j <= S->jendR; j++) A2(Dnew, iend + 1, j) = A2(h, iend + 1, j) + A2(zeta_new, iend + 1, j);
  if (S->south_edge) for (int i = istr - 1; i <= S->iendR; i++) A2(Dnew, i, jstr - 1) = A2(h, i, jstr - 1) + A2(zeta_new, i, jstr - 1);
  if (S->north_edge) for (int i = istr - 1; i <= S->iendR; i++) A2(Dnew, i, jend + 1) = A2(h, i, jend + 1) + A2(zeta_new, i, jend + 1);
  {
    const double cff1 = 0.5 * S->weight[0][iif - 1];
    if (S->west_edge) {
      for (int j = S->jstrR; j <= S->jendR; j++)
        A2(S->DU_avg1, istrU - 1, j) = A2(S->DU_avg1, istrU - 1, j) + cff1 * (A2(Dnew, istrU - 1, j) + A2(Dnew, istrU - 2, j)) *
                                                                       (UBAR(istrU - 1, j, knew)) * A2(S->dn_u, istrU - 1, j);
      for (int j = jstrV; j <= jend; j++)
        A2(S->DV_avg1, istr - 1, j) = A2(S->DV_avg1, istr - 1, j) + cff1 * (A2(Dnew, istr - 1, j) + A2(Dnew, istr - 1, j - 1)) *
                                                                     (VBAR(istr - 1, j, knew)) * A2(S->dm_v, istr - 1, j);
    }
    if (S->east_edge) {
      for (int j = S->jstrR; j <= S->jendR; j++)
        A2(S->DU_avg1, iend + 1, j) = A2(S->DU_avg1, iend + 1, j) + cff1 * (A2(Dnew, iend + 1, j) + A2(Dnew, iend, j)) *
                                                                     (UBAR(iend + 1, j, knew)) * A2(S->dn_u, iend + 1, j);
      for (int j = jstrV; j <= jend; j++)
        A2(S->DV_avg1, iend + 1, j) = A2(S->DV_avg1, iend + 1, j) + cff1 * (A2(Dnew, iend + 1, j) + A2(Dnew, iend + 1, j - 1)) *
                                                                     (VBAR(iend + 1, j, knew)) * A2(S->dm_v, iend + 1, j);
    }
    if (S->south_edge) {
      for (int i = istrU; i <= iend; i++)
        A2(S->DU_avg1, i, jstr - 1) = A2(S->DU_avg1, i, jstr - 1) + cff1 * (A2(Dnew, i, jstr - 1) + A2(Dnew, i - 1, jstr - 1)) *
                                                                     (UBAR(i, jstr - 1, knew)) * A2(S->dn_u, i, jstr - 1);
      for (int i = S->istrR; i <= S->iendR; i++)
        A2(S->DV_avg1, i, jstrV - 1) = A2(S->DV_avg1, i, jstrV - 1) + cff1 * (A2(Dnew, i, jstrV - 1) + A2(Dnew, i, jstrV - 2)) *
                                                                       (VBAR(i, jstrV - 1, knew)) * A2(S->dm_v, i, jstrV - 1);
    }
    if (S->north_edge) {
      for (int i = istrU; i <= iend; i++)
        A2(S->DU_avg1, i, jend + 1) = A2(S->DU_avg1, i, jend + 1) + cff1 * (A2(Dnew, i, jend + 1) + A2(Dnew, i - 1, jend + 1)) *
                                                                     (UBAR(i, jend + 1, knew)) * A2(S->dn_u, i, jend + 1);
      for (int i = S->istrR; i <= S->iendR; i++)
        A2(S->DV_avg1, i, jend + 1) = A2(S->DV_avg1, i, jend + 1) + cff1 * (A2(Dnew, i, jend + 1) + A2(Dnew, i, jend)) *
                                                                     (VBAR(i, jend + 1, knew)) * A2(S->dm_v, i, jend + 1);
    }
  }
  if (S->river_source) {  /* step2d_FB.F:531-554: river inflow sets ubar, vbar(knew) and the fast-time flux */
    for (int j = jstr; j <= jend; j++)
      for (int i = istrU; i <= iend; i++)
        if (fabs(A2(S->riv_uflx, i, j)) > 1e-3) {
          const int iriver = (int)lround(A2(S->riv_uflx, i, j) / 10);
          const double river_flux = S->riv_vol[iriver - 1] * (A2(S->riv_uflx, i, j) - 10 * iriver);
          UBAR(i, j, knew) = river_flux * 2 / (A2(S->dn_u, i, j) * (A2(Dnew, i - 1, j) + A2(Dnew, i, j)));
          A2(S->DU_avg1, i, j) = river_flux;
        }
    for (int j = jstrV; j <= jend; j++)
      for (int i = istr; i <= iend; i++)
        if (fabs(A2(S->riv_vflx, i, j)) > 1e-3) {
          const int iriver = (int)lround(A2(S->riv_vflx, i, j) / 10);
          const double river_flux = S->riv_vol[iriver - 1] * (A2(S->riv_vflx, i, j) - 10 * iriver);
          VBAR(i, j, knew) = river_flux * 2 / (A2(S->dm_v, i, j) * (A2(Dnew, i, j - 1) + A2(Dnew, i, j)));
          A2(S->DV_avg1, i, j) = river_flux;
        }
  }
  if (iif == S->nfast) {
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istrR; i <= S->iendR; i++) ZETA(i, j, knew) = A2(S->Zt_avg1, i, j);
    set_depth_tile(S);
  }
  or_exch2(S, S->zeta + (size_t)(knew - 1) * S->n2);
  or_exch2(S, S->ubar + (size_t)(knew - 1) * S->n2);
  or_exch2(S, S->vbar + (size_t)(knew - 1) * S->n2);
}

/* ---------------------------------------------------------------------- */
/* step3d_uv2_tile (step3d_uv2.F:18-786), IMPLICIT_BOTTOM_DRAG branch      */
/* ---------------------------------------------------------------------- */
void or_step3d_uv2(or_state *S) {
  const int N = S->N, nnew = S->nnew, nstp = S->nstp, knew = S->knew;
  double *FC = S->c1[1], *CF = S->c1[2], *DC = S->c1[3];
  for (int j = S->jstr; j <= S->jend; j++) {
    for (int i = S->istrU; i <= S->iend; i++) {
      C1(CF, i, 0) = 0.5 * (HZ(i, j, N) + HZ(i - 1, j, N));
      C1(DC, i, 0) = U(i, j, N, nnew);
      U(i, j, N, nnew) = U(i, j, N, nnew) / C1(CF, i, 0);
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = S->istrU; i <= S->iend; i++) {
        const double cff = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k));
        C1(CF, i, 0) = C1(CF, i, 0) + cff;
        C1(DC, i, 0) = C1(DC, i, 0) + U(i, j, k, nnew);
        U(i, j, k, nnew) = U(i, j, k, nnew) / cff;
      }
    for (int i = S->istrU; i <= S->iend; i++)
      C1(DC, i, 0) = (C1(DC, i, 0) * A2(S->dn_u, i, j) - A2(S->DU_avg1, i, j)) / (C1(CF, i, 0) * A2(S->dn_u, i, j));
    for (int k = 1; k <= N; k++)
      for (int i = S->istrU; i <= S->iend; i++) U(i, j, k, nnew) = (U(i, j, k, nnew) - C1(DC, i, 0)) * A2(S->umask, i, j);
    if (j >= S->jstrV) {
      for (int i = S->istr; i <= S->iend; i++) {
        C1(CF, i, 0) = 0.5 * (HZ(i, j, N) + HZ(i, j - 1, N));
        C1(DC, i, 0) = V(i, j, N, nnew);
        V(i, j, N, nnew) = V(i, j, N, nnew) / C1(CF, i, 0);
      }
      for (int k = N - 1; k >= 1; k--)
        for (int i = S->istr; i <= S->iend; i++) {
          const double cff = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k));
          C1(CF, i, 0) = C1(CF, i, 0) + cff;
          C1(DC, i, 0) = C1(DC, i, 0) + V(i, j, k, nnew);
          V(i, j, k, nnew) = V(i, j, k, nnew) / cff;
        }
      for (int i = S->istr; i <= S->iend; i++)
        C1(DC, i, 0) = (C1(DC, i, 0) * A2(S->dm_v, i, j) - A2(S->DV_avg1, i, j)) / (C1(CF, i, 0) * A2(S->dm_v, i, j));
      for (int k = 1; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++) V(i, j, k, nnew) = (V(i, j, k, nnew) - C1(DC, i, 0)) * A2(S->vmask, i, j);
    }
  }
  or_u3dbc(S);
  or_v3dbc(S);
  const int iu0 = S->istr, iu1 = S->c.ew_periodic ? S->iend : S->iendR;
  const int iv0 = S->c.ew_periodic ? S->istr : S->istrR, iv1 = S->c.ew_periodic ? S->iend : S->iendR;
  const int j0 = S->c.ns_periodic ? S->jstr : S->jstrR, j1 = S->c.ns_periodic ? S->jend : S->jendR;
  const double DELTA = 0.28, EPSIL = 0.36;
  for (int j = j0; j <= j1; j++) {
    for (int i = iu0; i <= iu1; i++) {
      C1(DC, i, N) = 0.5 * (HZ(i, j, N) + HZ(i - 1, j, N)) * A2(S->dn_u, i, j);
      C1(DC, i, 0) = C1(DC, i, N);
      C1(FC, i, 0) = C1(DC, i, N) * U(i, j, N, nnew);
    }
    for (int k = N - 1; k >= 1; k--)
      for (int i = iu0; i <= iu1; i++) {
        C1(DC, i, k) = 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j);
        C1(DC, i, 0) = C1(DC, i, 0) + C1(DC, i, k);
        C1(FC, i, 0) = C1(FC, i, 0) + C1(DC, i, k) * U(i, j, k, nnew);
      }
    for (int i = iu0; i <= iu1; i++) {
      C1(DC, i, 0) = 1.0 / C1(DC, i, 0);
      UBAR(i, j, knew) = C1(DC, i, 0) * A2(S->DU_avg1, i, j);
      C1(FC, i, 0) = C1(DC, i, 0) * (C1(FC, i, 0) - A2(S->DU_avg1, i, j));
      C1(CF, i, 0) = 0.0;
    }
    for (int k = N; k >= 1; k--)
      for (int i = iu0; i <= iu1; i++) {
        U(i, j, k, nnew) = (U(i, j, k, nnew) - C1(FC, i, 0)) * A2(S->umask, i, j);
        C1(CF, i, k) = DELTA * FLXU(i, j, k) + EPSIL * C1(DC, i, k) * (U(i, j, k, nstp) + U(i, j, k, nnew));
        C1(CF, i, 0) = C1(CF, i, 0) + C1(CF, i, k);
      }
    for (int i = iu0; i <= iu1; i++) C1(CF, i, 0) = C1(DC, i, 0) * (C1(CF, i, 0) - A2(S->DU_avg2, i, j));
    for (int k = 1; k <= N; k++)
      for (int i = iu0; i <= iu1; i++) FLXU(i, j, k) = C1(CF, i, k) - C1(DC, i, k) * C1(CF, i, 0);
    if (j >= S->jstr) {
      for (int i = iv0; i <= iv1; i++) {
        C1(DC, i, N) = 0.5 * (HZ(i, j, N) + HZ(i, j - 1, N)) * A2(S->dm_v, i, j);
        C1(DC, i, 0) = C1(DC, i, N);
        C1(FC, i, 0) = C1(DC, i, N) * V(i, j, N, nnew);
      }
      for (int k = N - 1; k >= 1; k--)
        for (int i = iv0; i <= iv1; i++) {
          C1(DC, i, k) = 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j);
          C1(DC, i, 0) = C1(DC, i, 0) + C1(DC, i, k);
          C1(FC, i, 0) = C1(FC, i, 0) + C1(DC, i, k) * V(i, j, k, nnew);
        }
      for (int i = iv0; i <= iv1; i++) {
        C1(DC, i, 0) = 1.0 / C1(DC, i, 0);
        VBAR(i, j, knew) = C1(DC, i, 0) * A2(S->DV_avg1, i, j);
        C1(FC, i, 0) = C1(DC, i, 0) * (C1(FC, i, 0) - A2(S->DV_avg1, i, j));
        C1(CF, i, 0) = 0.0;
      }
      for (int k = N; k >= 1; k--)
        for (int i = iv0; i <= iv1; i++) {
          V(i, j, k, nnew) = (V(i, j, k, nnew) - C1(FC, i, 0)) * A2(S->vmask, i, j);
          C1(CF, i, k) = DELTA * FLXV(i, j, k) + EPSIL * C1(DC, i, k) * (V(i, j, k, nstp) + V(i, j, k, nnew));
          C1(CF, i, 0) = C1(CF, i, 0) + C1(CF, i, k);
        }
      for (int i = iv0; i <= iv1; i++) C1(CF, i, 0) = C1(DC, i, 0) * (C1(CF, i, 0) - A2(S->DV_avg2, i, j));
      for (int k = 1; k <= N; k++)
        for (int i = iv0; i <= iv1; i++) FLXV(i, j, k) = C1(CF, i, k) - C1(DC, i, k) * C1(CF, i, 0);
    }
  }
  if (S->c.adv_isoneutral) or_iso_diff3(S, iu0, iu1, iv0, iv1, j0, j1);   /* before the river faces */
  if (S->river_source) river_uv(S, nnew, S->istr);
  if (S->c.adv_isoneutral) or_iso_exch_diff3(S);   /* step3d_uv2.F:730-732 */
  or_exch3(S, S->FlxU, N);
  or_exch3(S, S->u + (size_t)(nnew - 1) * S->n3, N);
  or_exch2(S, S->ubar + (size_t)(knew - 1) * S->n2);
  or_exch3(S, S->FlxV, N);
  or_exch3(S, S->v + (size_t)(nnew - 1) * S->n3, N);
  or_exch2(S, S->vbar + (size_t)(knew - 1) * S->n2);
}

/* ---------------------------------------------------------------------- */
/* step3d_t_iso_tile (step3d_t_ISO.F:45-1178), non-isoneutral branch       */
/* ---------------------------------------------------------------------- */
void or_step3d_t(or_state *S) {
  const int N = S->N, NT = S->NT, nnew = S->nnew, nrhs = S->nrhs;
  const double dt = S->dt;
  double *FX = S->s2[4], *FE = S->s2[5], *wrk1 = S->s2[6];
  double *WC = S->c1[0], *FC = S->c1[1], *CF = S->c1[2], *DC = S->c1[3];
  const int iso = S->c.adv_isoneutral;   /* ADV_ISONEUTRAL: centred fluxes (no UPSTREAM_TS, step3d_t_ISO.F:4-6) */
  for (int itrc = 1; itrc <= NT; itrc++) {
    for (int k = 1; k <= N; k++) {
      horiz_tracer_fluxes(S, k, itrc, nrhs, !iso, FX, FE, wrk1);
      for (int j = S->jstr; j <= S->jend; j++)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, k, nnew, itrc) = TT(i, j, k, nnew, itrc) - dt * A2(S->pm, i, j) * A2(S->pn, i, j) *
                                                                  (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j));
    }
    if (iso) or_iso_tracer(S, itrc);   /* step3d_t_ISO.F:253-846 */
    for (int j = S->jstr; j <= S->jend; j++) {
      vert_tracer_fluxes(S, j, itrc, nrhs, FC, CF, S->Hz);
      for (int k = 1; k <= N; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          TT(i, j, k, nnew, itrc) =
              TT(i, j, k, nnew, itrc) - dt * A2(S->pm, i, j) * A2(S->pn, i, j) * (C1(FC, i, k) - C1(FC, i, k - 1));
          if (S->pipe_source && A2(S->pipe_idx, i, j) > 0.) {  /* step3d_t_ISO.F:927-934 */
            const int pidx = (int)A2(S->pipe_idx, i, j);
            TT(i, j, k, nnew, itrc) = TT(i, j, k, nnew, itrc) + dt * A2(S->pm, i, j) * A2(S->pn, i, j) *
                                                                    A2(S->pipe_flx, i, j) *
                                                                    S->pipe_prf[(pidx - 1) + (size_t)S->npip * (k - 1)] *
                                                                    S->pipe_trc[(pidx - 1) + (size_t)S->npip * (itrc - 1)];
          }
        }
      /* heat of rain (step3d_t_ISO.F:939-951): BULK_FRC uses the 2 m air
       * temperature tair, otherwise the water's own t(N)/Hz(N) */
      if (itrc == 1)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, N, nnew, itrc) = TT(i, j, N, nnew, itrc) +
                                    dt * A2(S->swflx, i, j) *
                                        (S->c.bulk_frc ? A2(S->tair, i, j) : TT(i, j, N, nnew, itrc) / HZ(i, j, N));
      for (int i = S->istr; i <= S->iend; i++)
        TT(i, j, N, nnew, itrc) = TT(i, j, N, nnew, itrc) + dt * S->stflx[O2(i, j) + (size_t)(itrc - 1) * S->n2];
      if (S->c.lmd) {
        /* LMD_KPP solar heating + LMD_NONLOCAL (step3d_t_ISO.F, itemp/isalt branches) */
        const double *stf = S->stflx;
        if (itrc == 1) {
          for (int k = N - 1; k >= 1; k--)
            for (int i = S->istr; i <= S->iend; i++) {
              double cff = A2(S->srflx, i, j) * W3(S->swr_frac, i, j, k);
              if (S->c.lmd & OR_LMD_NONLOCAL) cff = cff - W3(S->ghat, i, j, k) * (stf[O2(i, j)] - A2(S->srflx, i, j));
              TT(i, j, k + 1, nnew, 1) = TT(i, j, k + 1, nnew, 1) - dt * cff;
              TT(i, j, k, nnew, 1) = TT(i, j, k, nnew, 1) + dt * cff;
            }
        } else if (itrc == 2 && S->c.salinity && (S->c.lmd & OR_LMD_NONLOCAL)) {
          for (int k = N - 1; k >= 1; k--)
            for (int i = S->istr; i <= S->iend; i++) {
              const double cff = -dt * W3(S->ghat, i, j, k) * stf[O2(i, j) + S->n2];
              TT(i, j, k + 1, nnew, 2) = TT(i, j, k + 1, nnew, 2) - cff;
              TT(i, j, k, nnew, 2) = TT(i, j, k, nnew, 2) + cff;
            }
        }
      }
      const int iAkt = itrc < S->nTS ? itrc : S->nTS;
      for (int i = S->istr; i <= S->iend; i++) {
        C1(DC, i, 0) = dt * A2(S->pm, i, j) * A2(S->pn, i, j);
        /* ADV_ISONEUTRAL && STABILIZE: Akt + Akz (step3d_t_ISO.F:1049-1053) */
        C1(FC, i, 1) = 2.0 * dt * (iso ? AKT(i, j, 1, iAkt) + W3(S->Akz, i, j, 1) : AKT(i, j, 1, iAkt)) /
                       (HZ(i, j, 1) + HZ(i, j, 2));
        C1(WC, i, 1) = C1(DC, i, 0) * WI(i, j, 1);
        const double cff = 1.0 / (HZ(i, j, 1) + C1(FC, i, 1) + fmax0(C1(WC, i, 1)));
        C1(CF, i, 1) = cff * (C1(FC, i, 1) - fmin0(C1(WC, i, 1)));
        C1(DC, i, 1) = cff * TT(i, j, 1, nnew, itrc);
      }
      for (int k = 2; k <= N - 1; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          C1(FC, i, k) = 2.0 * dt * (iso ? AKT(i, j, k, iAkt) + W3(S->Akz, i, j, k) : AKT(i, j, k, iAkt)) /
                         (HZ(i, j, k) + HZ(i, j, k + 1));
          C1(WC, i, k) = WI(i, j, k) * C1(DC, i, 0);
          const double cff = 1.0 / (HZ(i, j, k) + C1(FC, i, k) + fmax0(C1(WC, i, k)) + C1(FC, i, k - 1) - fmin0(C1(WC, i, k - 1)) -
                                    C1(CF, i, k - 1) * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1))));
          C1(CF, i, k) = cff * (C1(FC, i, k) - fmin0(C1(WC, i, k)));
          C1(DC, i, k) = cff * (TT(i, j, k, nnew, itrc) + C1(DC, i, k - 1) * (C1(FC, i, k - 1) + fmax0(C1(WC, i, k - 1))));
        }
      for (int i = S->istr; i <= S->iend; i++)
        TT(i, j, N, nnew, itrc) =
            (TT(i, j, N, nnew, itrc) + C1(DC, i, N - 1) * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)))) /
            (HZ(i, j, N) + C1(FC, i, N - 1) - fmin0(C1(WC, i, N - 1)) - C1(CF, i, N - 1) * (C1(FC, i, N - 1) + fmax0(C1(WC, i, N - 1)))) *
            A2(S->rmask, i, j);
      for (int k = N - 1; k >= 1; k--)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, k, nnew, itrc) = (C1(DC, i, k) + C1(CF, i, k) * TT(i, j, k + 1, nnew, itrc)) * A2(S->rmask, i, j);
    }
  }
  for (int itrc = 1; itrc <= NT; itrc++) or_t3dbc(S, itrc);
  for (int itrc = 1; itrc <= NT; itrc++)
    or_exch3(S, S->t + (size_t)(nnew - 1) * S->n3 + (size_t)(itrc - 1) * 3 * S->n3, N);
}

/* ---------------------------------------------------------------------- */
/* t3dmix_tile (t3dmix_S.F): Laplacian tracer diffusion along S            */
/* ---------------------------------------------------------------------- */
void or_t3dmix(or_state *S) {
  const int N = S->N, NT = S->NT, nnew = S->nnew, nrhs = S->nrhs;
  double *FX = S->s2[4], *FE = S->s2[5];
  for (int itrc = 1; itrc <= NT; itrc++) {
    const double *d2 = S->diff2 + (size_t)(itrc - 1) * S->n2;
    for (int k = 1; k <= N; k++) {
      for (int j = S->jstr; j <= S->jend; j++)
        for (int i = S->istr; i <= S->iend + 1; i++)
          A2(FX, i, j) = 0.25 * (A2(d2, i, j) + A2(d2, i - 1, j)) * A2(S->pmon_u, i, j) * (HZ(i, j, k) + HZ(i - 1, j, k)) *
                         (TT(i, j, k, nrhs, itrc) - TT(i - 1, j, k, nrhs, itrc)) * A2(S->umask, i, j);
      for (int j = S->jstr; j <= S->jend + 1; j++)
        for (int i = S->istr; i <= S->iend; i++)
          A2(FE, i, j) = 0.25 * (A2(d2, i, j) + A2(d2, i, j - 1)) * A2(S->pnom_v, i, j) * (HZ(i, j, k) + HZ(i, j - 1, k)) *
                         (TT(i, j, k, nrhs, itrc) - TT(i, j - 1, k, nrhs, itrc)) * A2(S->vmask, i, j);
      for (int j = S->jstr; j <= S->jend; j++)
        for (int i = S->istr; i <= S->iend; i++)
          TT(i, j, k, nnew, itrc) = TT(i, j, k, nnew, itrc) + S->dt * A2(S->pm, i, j) * A2(S->pn, i, j) *
                                                                  (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j)) /
                                                                  HZ(i, j, k);
    }
    or_exch3(S, S->t + (size_t)(nnew - 1) * S->n3 + (size_t)(itrc - 1) * 3 * S->n3, N);
  }
}
