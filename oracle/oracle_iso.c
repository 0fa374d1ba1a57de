/*
 * oracle_iso.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 *
 * ADV_ISONEUTRAL: the rotated (isoneutral) biharmonic tracer operator with
 * SW_TRIADS and STABILIZE, which step3d_t_ISO.F:15-18 always defines with it,
 * restated in the reference's own loop structure: the recursive k-loop over
 * two vertical slices k1/k2 of FSC, dTdz, dTdx, dTde (step3d_t_ISO.F:165-173),
 * so that this restatement and the full-3-D HIP form (k_iso.hip) share no
 * code.  Its inputs:
 *   dRdx, dRde   prsgrd.F:307-338, 423-453 (corrector stage only)
 *   diff3u/v     step3d_uv2.F:572-575, 616-619 (square roots of the
 *                hyperdiffusivities, from the corrected u,v(nnew))
 *   idRz         step3d_uv2.F:622-697 (limited inverse vertical density
 *                gradient, w-levels 1..N-1)
 * exchanged like the reference (step3d_uv1.F:529-532, step3d_uv2.F:730-732).
 *
 * Parity: no reference case with input data in /root/reference enables
 * ADV_ISONEUTRAL (tests/Flux_frc needs input_data that is not checked in),
 * so this restatement is parity unpinned to reference output; it is the
 * checker for the HIP path (tests/test_iso.py).
 *
 * One deviation, forced by the reference reading unset scratch: at a
 * physical (non-periodic) edge prsgrd's dRdx(istr) reads rx(istr-1) and
 * dRdx(iend+1) reads rx(iend+2), two cells its extrapolation never writes
 * (prsgrd.F:256-268 sets only rx(imin-1), rx(imax+1)); the same for dRde at
 * the south/north edges.  The restatement continues the extrapolation
 * (rx(imin-2) = rx(imin), rx(imax+2) = rx(imax)), like k_iso.hip.
 */
#include "oracle_core.h"

#define ISO_GAMMA 0.0833333333333   /* step3d_uv2.F:76 */
#define ALPHA_MAX 2.                /* step3d_uv2.F:75 */

/* prsgrd.F:307-338: dRdx(:,:,k) from the XI elementary differences rx
 * (i = imin..imax, extrapolated at physical edges) of the same k */
void or_iso_dRdx(or_state *S, int k, double *rx, int imin, int imax) {
  const double r0g = S->rho0 / S->g;
  if (!S->c.ew_periodic) {
    if (S->west_edge) for (int j = S->jstr; j <= S->jend; j++) A2(rx, imin - 2, j) = A2(rx, imin, j);
    if (S->east_edge) for (int j = S->jstr; j <= S->jend; j++) A2(rx, imax + 2, j) = A2(rx, imax, j);
  }
  for (int j = S->jstr; j <= S->jend; j++)
    for (int i = S->istr; i <= S->iendR; i++) {
      const double fs = A2(S->f, i, j) + A2(S->f, i - 1, j);
      R3(S->dRdx, i, j, k) = 0.5 * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) *
                             (r0g * 0.25 * (fs * fs) * (ZR(i, j, k) - ZR(i - 1, j, k)) - 0.5 * A2(rx, i, j) -
                              0.25 * (A2(rx, i - 1, j) + A2(rx, i + 1, j)));
    }
}

/* prsgrd.F:423-453 */
void or_iso_dRde(or_state *S, int k, double *rx, int jmin, int jmax) {
  const double r0g = S->rho0 / S->g;
  if (!S->c.ns_periodic) {
    if (S->south_edge) for (int i = S->istr; i <= S->iend; i++) A2(rx, i, jmin - 2) = A2(rx, i, jmin);
    if (S->north_edge) for (int i = S->istr; i <= S->iend; i++) A2(rx, i, jmax + 2) = A2(rx, i, jmax);
  }
  for (int j = S->jstr; j <= S->jendR; j++)
    for (int i = S->istr; i <= S->iend; i++) {
      const double fs = A2(S->f, i, j) + A2(S->f, i, j - 1);
      R3(S->dRde, i, j, k) = 0.5 * (A2(S->pn, i, j) + A2(S->pn, i, j - 1)) *
                             (r0g * 0.25 * (fs * fs) * (ZR(i, j, k) - ZR(i, j - 1, k)) - 0.5 * A2(rx, i, j) -
                              0.25 * (A2(rx, i, j - 1) + A2(rx, i, j + 1)));
    }
}

/* prsgrd's exchange of the slopes (step3d_uv1.F:529-532) */
void or_iso_exch_slopes(or_state *S) {
  or_exch3(S, S->dRdx, S->N);
  or_exch3(S, S->dRde, S->N);
}

/* step3d_uv2.F:572-575, 616-619, 622-697, 730-732: diff3u over IU_RANGE x
 * J_RANGE, diff3v over IV_RANGE x (J_RANGE, j >= jstr), idRz over the
 * interior at w-levels 1..N-1; (iu0,iu1), (iv0,iv1), (j0,j1) are the
 * ranges of the flux correction loop of or_step3d_uv2 */
void or_iso_diff3(or_state *S, int iu0, int iu1, int iv0, int iv1, int j0, int j1) {
  const int N = S->N, nnew = S->nnew;
  const double r0g = S->rho0 / S->g, qp2 = S->qp2, epsil = 1.E-33;
  for (int j = j0; j <= j1; j++) {
    for (int k = 1; k <= N; k++)
      for (int i = iu0; i <= iu1; i++)
        R3(S->diff3u, i, j, k) = sqrt(ISO_GAMMA * fabs(U(i, j, k, nnew)) * A2(S->dm_u, i, j)) * A2(S->dm_u, i, j);
    if (j >= S->jstr)
      for (int k = 1; k <= N; k++)
        for (int i = iv0; i <= iv1; i++)
          R3(S->diff3v, i, j, k) = sqrt(ISO_GAMMA * fabs(V(i, j, k, nnew)) * A2(S->dn_v, i, j)) * A2(S->dn_v, i, j);
    if (j >= S->jstr && j <= S->jend)
      for (int k = 1; k <= N - 1; k++)
        for (int i = S->istr; i <= S->iend; i++) {
          double dRz;
          if (S->c.nonlin_eos) {
            const double dpth = -0.5 * (ZR(i, j, k + 1) + ZR(i, j, k));
            dRz = R3(S->rho1, i, j, k) - R3(S->rho1, i, j, k + 1) +
                  (R3(S->qp1, i, j, k) - R3(S->qp1, i, j, k + 1)) * dpth * (1. - 2. * qp2 * dpth);
          } else {
            dRz = R3(S->rho, i, j, k) - R3(S->rho, i, j, k + 1);
          }
          const double fc = A2(S->f, i, j);
          dRz = dmax(dRz, 0.) + r0g * (fc * fc) * (ZR(i, j, k + 1) - ZR(i, j, k));
          const double dRx_max =
              dmax(dmax(A2(S->dm_u, i, j) * dmax(fabs(R3(S->dRdx, i, j, k)), fabs(R3(S->dRdx, i, j, k + 1))),
                        A2(S->dm_u, i + 1, j) * dmax(fabs(R3(S->dRdx, i + 1, j, k)), fabs(R3(S->dRdx, i + 1, j, k + 1)))),
                   dmax(A2(S->dn_v, i, j) * dmax(fabs(R3(S->dRde, i, j, k)), fabs(R3(S->dRde, i, j, k + 1))),
                        A2(S->dn_v, i, j + 1) * dmax(fabs(R3(S->dRde, i, j + 1, k)), fabs(R3(S->dRde, i, j + 1, k + 1)))));
          double cfs, cfb;
          if (S->c.lmd) {   /* LMD_KPP / LMD_BKPP */
            cfs = dmin(1., (ZW(i, j, N) - ZW(i, j, k)) / dmax(50., A2(S->hbls, i, j)));
            cfb = dmin(1., (ZW(i, j, k) - ZW(i, j, 0)) / dmax(50., A2(S->hbbl, i, j)));
          } else {
            cfs = dmin(1., (ZW(i, j, N) - ZW(i, j, k)) / 50.);
            cfb = dmin(1., (ZW(i, j, k) - ZW(i, j, 0)) / 50.);
          }
          const double cff = ALPHA_MAX * cfs * (2. - cfs) * cfb * (2. - cfb);
          W3(S->idRz, i, j, k) = cff / dmax(dmax(cff * dRz, dRx_max), epsil);
        }
  }
}

void or_iso_exch_diff3(or_state *S) {
  or_exch3(S, S->idRz, S->N + 1);
  or_exch3(S, S->diff3u, S->N);
  or_exch3(S, S->diff3v, S->N);
}

static const double wgt[5] = {0., 1., 0.5, 0.3333333333333333, 0.25};   /* step3d_t_ISO.F:121-122 */

/* the SW_TRIADS vertical components (step3d_t_ISO.F:411-485, 722-805):
 * sumX*wgt(idx) + sumE*wgt(ide) at (i,j) between levels k and k+1 */
static double triads(or_state *S, int i, int j, int k, const double *dTdz2, const double *dTdx1,
                     const double *dTdx2, const double *dTde1, const double *dTde2) {
  const double *dRdx = S->dRdx, *dRde = S->dRde, *d3u = S->diff3u, *d3v = S->diff3v;
  const double tz = A2(dTdz2, i, j);
  double sumX = 0., sumE = 0.;
  int idx = 0, ide = 0;
  if (R3(dRdx, i, j, k) < 0.) {
    sumX = R3(d3u, i, j, k) * R3(dRdx, i, j, k) * (R3(dRdx, i, j, k) * tz - A2(dTdx1, i, j));
    idx = 1;
  }
  if (R3(dRdx, i, j, k + 1) > 0.) {
    sumX = sumX + R3(d3u, i, j, k + 1) * R3(dRdx, i, j, k + 1) * (R3(dRdx, i, j, k + 1) * tz - A2(dTdx2, i, j));
    idx = idx + 1;
  }
  if (R3(dRdx, i + 1, j, k + 1) < 0.) {
    sumX = sumX + R3(d3u, i + 1, j, k + 1) * R3(dRdx, i + 1, j, k + 1) *
                      (R3(dRdx, i + 1, j, k + 1) * tz - A2(dTdx2, i + 1, j));
    idx = idx + 1;
  }
  if (R3(dRdx, i + 1, j, k) > 0.) {
    sumX = sumX + R3(d3u, i + 1, j, k) * R3(dRdx, i + 1, j, k) * (R3(dRdx, i + 1, j, k) * tz - A2(dTdx1, i + 1, j));
    idx = idx + 1;
  }
  if (R3(dRde, i, j, k) < 0.) {
    sumE = R3(d3v, i, j, k) * R3(dRde, i, j, k) * (R3(dRde, i, j, k) * tz - A2(dTde1, i, j));
    ide = 1;
  }
  if (R3(dRde, i, j, k + 1) > 0.) {
    sumE = sumE + R3(d3v, i, j, k + 1) * R3(dRde, i, j, k + 1) * (R3(dRde, i, j, k + 1) * tz - A2(dTde2, i, j));
    ide = ide + 1;
  }
  if (R3(dRde, i, j + 1, k + 1) < 0.) {
    sumE = sumE + R3(d3v, i, j + 1, k + 1) * R3(dRde, i, j + 1, k + 1) *
                      (R3(dRde, i, j + 1, k + 1) * tz - A2(dTde2, i, j + 1));
    ide = ide + 1;
  }
  if (R3(dRde, i, j + 1, k) > 0.) {
    sumE = sumE + R3(d3v, i, j + 1, k) * R3(dRde, i, j + 1, k) * (R3(dRde, i, j + 1, k) * tz - A2(dTde1, i, j + 1));
    ide = ide + 1;
  }
  return sumX * wgt[idx] + sumE * wgt[ide];
}

static double max4(double a, double b, double c, double d) { return dmax(dmax(a, b), dmax(c, d)); }

/* STABILIZE with SW_TRIADS (step3d_t_ISO.F:656-695): Akz(i,j,k) from the
 * metric FSC = idRz*dz (k2 slice before it is turned into the flux) */
static double akz_of(or_state *S, int i, int j, int k, double fsc) {
  const double *dRdx = S->dRdx, *dRde = S->dRde, *d3u = S->diff3u, *d3v = S->diff3v;
  double a;
  a = fsc * R3(dRdx, i, j, k);         const double s2_XLL = a * a;
  a = fsc * R3(dRdx, i, j, k + 1);     const double s2_XLU = a * a;
  a = fsc * R3(dRdx, i + 1, j, k + 1); const double s2_XRU = a * a;
  a = fsc * R3(dRdx, i + 1, j, k);     const double s2_XRL = a * a;
  a = fsc * R3(dRde, i, j, k);         const double s2_ELL = a * a;
  a = fsc * R3(dRde, i, j, k + 1);     const double s2_ELU = a * a;
  a = fsc * R3(dRde, i, j + 1, k + 1); const double s2_ERU = a * a;
  a = fsc * R3(dRde, i, j + 1, k);     const double s2_ERL = a * a;
  const double cff = 2. / (HZ(i, j, k + 1) + HZ(i, j, k));
  const double cff2 = cff * cff, cffX = A2(S->pm, i, j) * A2(S->pm, i, j), cffE = A2(S->pn, i, j) * A2(S->pn, i, j);
  return 15. *
         (max4(R3(d3u, i, j, k) * s2_XLL, R3(d3u, i + 1, j, k) * s2_XRL, R3(d3u, i, j, k + 1) * s2_XLU,
               R3(d3u, i + 1, j, k + 1) * s2_XRU) +
          max4(R3(d3v, i, j, k) * s2_ELL, R3(d3v, i, j + 1, k) * s2_ERL, R3(d3v, i, j, k + 1) * s2_ELU,
               R3(d3v, i, j + 1, k + 1) * s2_ERU)) *
         (max4(R3(d3u, i, j, k) * (cffX + cff2 * s2_XLL), R3(d3u, i, j, k + 1) * (cffX + cff2 * s2_XLU),
               R3(d3u, i + 1, j, k + 1) * (cffX + cff2 * s2_XRU), R3(d3u, i + 1, j, k) * (cffX + cff2 * s2_XRL)) +
          max4(R3(d3v, i, j, k) * (cffE + cff2 * s2_ELL), R3(d3v, i, j, k + 1) * (cffE + cff2 * s2_ELU),
               R3(d3v, i, j + 1, k + 1) * (cffE + cff2 * s2_ERU), R3(d3v, i, j + 1, k) * (cffE + cff2 * s2_ERL)));
}

/* step3d_t_ISO.F:253-846 for tracer itrc: the first rotated Laplacian of
 * t(nstp) into LapT, its lateral boundary values, and the second one added
 * to t(nnew) (which holds Hz*t after the horizontal advection); Akz(:,:,1:N-1)
 * is left for the implicit vertical diffusion (step3d_t_ISO.F:1049-1065) */
void or_iso_tracer(or_state *S, int itrc) {
  const int N = S->N, nstp = S->nstp, nnew = S->nnew;
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const double dt = S->dt;
  int imin, imax, jmin, jmax;   /* step3d_t_ISO.F:132-161 */
  if (!S->c.ew_periodic) {
    imin = S->west_edge ? istr : istr - 1;
    imax = S->east_edge ? iend : iend + 1;
  } else { imin = istr - 1; imax = iend + 1; }
  if (!S->c.ns_periodic) {
    jmin = S->south_edge ? jstr : jstr - 1;
    jmax = S->north_edge ? jend : jend + 1;
  } else { jmin = jstr - 1; jmax = jend + 1; }
  double *FSC[3] = {NULL, S->iso_FSC, S->iso_FSC + S->n2}, *dTdz[3] = {NULL, S->iso_dTdz, S->iso_dTdz + S->n2};
  double *dTdx[3] = {NULL, S->iso_dTdx, S->iso_dTdx + S->n2}, *dTde[3] = {NULL, S->iso_dTde, S->iso_dTde + S->n2};
  double *FX = S->s2[10], *FE = S->s2[11], *LapT = S->iso_LapT;
#define TS(i, j, k) TT(i, j, k, nstp, itrc)
  /* ---- the first rotated Laplacian (step3d_t_ISO.F:308-512) ---- */
  int k1, k2 = 1;
  for (int k = 0; k <= N; k++) {
    k1 = k2;
    k2 = 3 - k1;
    if (k == 0) {
      for (int j = jmin - 1; j <= jmax + 1; j++)
        for (int i = imin - 1; i <= imax + 1; i++) {
          A2(FSC[k2], i, j) = 0.;
          A2(dTdz[k2], i, j) = W3(S->idRz, i, j, 1) * (TS(i, j, 2) - TS(i, j, 1));
        }
    } else if (k < N) {
      for (int j = jmin - 1; j <= jmax + 1; j++)
        for (int i = imin - 1; i <= imax + 1; i++) {
          A2(FSC[k2], i, j) = W3(S->idRz, i, j, k) * (ZR(i, j, k + 1) - ZR(i, j, k));
          A2(dTdz[k2], i, j) = W3(S->idRz, i, j, k) * (TS(i, j, k + 1) - TS(i, j, k));
        }
    } else {
      for (int j = jmin - 1; j <= jmax + 1; j++)
        for (int i = imin - 1; i <= imax + 1; i++) {
          A2(FSC[k2], i, j) = 0.;
          A2(dTdz[k2], i, j) = A2(dTdz[k1], i, j);
        }
    }
    if (k < N) {
      for (int j = jmin; j <= jmax; j++)
        for (int i = imin; i <= imax + 1; i++)
          A2(dTdx[k2], i, j) = 0.5 * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) * (TS(i, j, k + 1) - TS(i - 1, j, k + 1)) *
                               A2(S->umask, i, j);
      for (int j = jmin; j <= jmax + 1; j++)
        for (int i = imin; i <= imax; i++)
          A2(dTde[k2], i, j) = 0.5 * (A2(S->pn, i, j) + A2(S->pn, i, j - 1)) * (TS(i, j, k + 1) - TS(i, j - 1, k + 1)) *
                               A2(S->vmask, i, j);
    }
    if (k > 0) {
      for (int j = jmin; j <= jmax; j++)
        for (int i = imin; i <= imax + 1; i++) {
          const double r = R3(S->dRdx, i, j, k);
          A2(FX, i, j) = R3(S->diff3u, i, j, k) * 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j) *
                         (A2(dTdx[k1], i, j) - 0.5 * (dmin(r, 0.) * (A2(dTdz[k1], i - 1, j) + A2(dTdz[k2], i, j)) +
                                                      dmax(r, 0.) * (A2(dTdz[k2], i - 1, j) + A2(dTdz[k1], i, j))));
        }
      for (int j = jmin; j <= jmax + 1; j++)
        for (int i = imin; i <= imax; i++) {
          const double r = R3(S->dRde, i, j, k);
          A2(FE, i, j) = R3(S->diff3v, i, j, k) * 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j) *
                         (A2(dTde[k1], i, j) - 0.5 * (dmin(r, 0.) * (A2(dTdz[k1], i, j - 1) + A2(dTdz[k2], i, j)) +
                                                      dmax(r, 0.) * (A2(dTdz[k2], i, j - 1) + A2(dTdz[k1], i, j))));
        }
      if (k < N)
        for (int j = jmin; j <= jmax; j++)
          for (int i = imin; i <= imax; i++)
            A2(FSC[k2], i, j) = A2(FSC[k2], i, j) *
                                triads(S, i, j, k, dTdz[k2], dTdx[k1], dTdx[k2], dTde[k1], dTde[k2]);
      for (int j = jmin; j <= jmax; j++)
        for (int i = imin; i <= imax; i++)
          R3(LapT, i, j, k) = (A2(S->pm, i, j) * A2(S->pn, i, j) *
                                   (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j)) +
                               A2(FSC[k2], i, j) - A2(FSC[k1], i, j)) /
                              HZ(i, j, k);
    }
  }
  /* lateral boundary values of LapT (step3d_t_ISO.F:515-565) */
  if (!S->c.ew_periodic) {
    if (S->west_edge)
      for (int k = 1; k <= N; k++)
        for (int j = jmin; j <= jmax; j++) R3(LapT, istr - 1, j, k) = (S->c.obc & 1) ? R3(LapT, istr, j, k) : 0.;
    if (S->east_edge)
      for (int k = 1; k <= N; k++)
        for (int j = jmin; j <= jmax; j++) R3(LapT, iend + 1, j, k) = (S->c.obc & 2) ? R3(LapT, iend, j, k) : 0.;
  }
  if (!S->c.ns_periodic) {
    if (S->south_edge)
      for (int k = 1; k <= N; k++)
        for (int i = imin; i <= imax; i++) R3(LapT, i, jstr - 1, k) = (S->c.obc & 4) ? R3(LapT, i, jstr, k) : 0.;
    if (S->north_edge)
      for (int k = 1; k <= N; k++)
        for (int i = imin; i <= imax; i++) R3(LapT, i, jend + 1, k) = (S->c.obc & 8) ? R3(LapT, i, jend, k) : 0.;
  }
  /* ---- the second rotated Laplacian, added to t(nnew) (step3d_t_ISO.F:567-846) ---- */
  k2 = 1;
  for (int k = 0; k <= N; k++) {
    k1 = k2;
    k2 = 3 - k1;
    if (k == 0) {
      for (int j = jstr - 1; j <= jend + 1; j++)
        for (int i = istr - 1; i <= iend + 1; i++) {
          A2(FSC[k2], i, j) = 0.;
          A2(dTdz[k2], i, j) = W3(S->idRz, i, j, 1) * (R3(LapT, i, j, 2) - R3(LapT, i, j, 1));
        }
    } else if (k < N) {
      for (int j = jstr - 1; j <= jend + 1; j++)
        for (int i = istr - 1; i <= iend + 1; i++) {
          A2(FSC[k2], i, j) = W3(S->idRz, i, j, k) * (ZR(i, j, k + 1) - ZR(i, j, k));
          A2(dTdz[k2], i, j) = W3(S->idRz, i, j, k) * (R3(LapT, i, j, k + 1) - R3(LapT, i, j, k));
        }
    } else {
      for (int j = jmin - 1; j <= jmax + 1; j++)
        for (int i = imin - 1; i <= imax + 1; i++) {
          A2(FSC[k2], i, j) = 0.;
          A2(dTdz[k2], i, j) = A2(dTdz[k1], i, j);
        }
    }
    if (k < N) {
      for (int j = jstr; j <= jend; j++)
        for (int i = istr; i <= iend + 1; i++)
          A2(dTdx[k2], i, j) = 0.5 * (A2(S->pm, i, j) + A2(S->pm, i - 1, j)) *
                               (R3(LapT, i, j, k + 1) - R3(LapT, i - 1, j, k + 1)) * A2(S->umask, i, j);
      for (int j = jstr; j <= jend + 1; j++)
        for (int i = istr; i <= iend; i++)
          A2(dTde[k2], i, j) = 0.5 * (A2(S->pn, i, j) + A2(S->pn, i, j - 1)) *
                               (R3(LapT, i, j, k + 1) - R3(LapT, i, j - 1, k + 1)) * A2(S->vmask, i, j);
    }
    if (k > 0) {
      for (int j = jstr; j <= jend; j++)
        for (int i = istr; i <= iend + 1; i++) {
          const double r = R3(S->dRdx, i, j, k);
          A2(FX, i, j) = -R3(S->diff3u, i, j, k) * 0.5 * (HZ(i, j, k) + HZ(i - 1, j, k)) * A2(S->dn_u, i, j) *
                         (A2(dTdx[k1], i, j) - 0.5 * (dmin(r, 0.) * (A2(dTdz[k1], i - 1, j) + A2(dTdz[k2], i, j)) +
                                                      dmax(r, 0.) * (A2(dTdz[k2], i - 1, j) + A2(dTdz[k1], i, j))));
        }
      for (int j = jstr; j <= jend + 1; j++)
        for (int i = istr; i <= iend; i++) {
          const double r = R3(S->dRde, i, j, k);
          A2(FE, i, j) = -R3(S->diff3v, i, j, k) * 0.5 * (HZ(i, j, k) + HZ(i, j - 1, k)) * A2(S->dm_v, i, j) *
                         (A2(dTde[k1], i, j) - 0.5 * (dmin(r, 0.) * (A2(dTdz[k1], i, j - 1) + A2(dTdz[k2], i, j)) +
                                                      dmax(r, 0.) * (A2(dTdz[k2], i, j - 1) + A2(dTdz[k1], i, j))));
        }
      if (k < N)
        for (int j = jstr; j <= jend; j++)
          for (int i = istr; i <= iend; i++) {
            const double akz = akz_of(S, i, j, k, A2(FSC[k2], i, j));
            W3(S->Akz, i, j, k) = akz;
            const double cff = 2. / (HZ(i, j, k + 1) + HZ(i, j, k));
            A2(FSC[k2], i, j) = -A2(FSC[k2], i, j) *
                                    triads(S, i, j, k, dTdz[k2], dTdx[k1], dTdx[k2], dTde[k1], dTde[k2]) -
                                cff * akz * (TS(i, j, k + 1) - TS(i, j, k));
          }
      for (int j = jstr; j <= jend; j++)
        for (int i = istr; i <= iend; i++)
          TT(i, j, k, nnew, itrc) =
              TT(i, j, k, nnew, itrc) +
              dt * (A2(S->pm, i, j) * A2(S->pn, i, j) * (A2(FX, i + 1, j) - A2(FX, i, j) + A2(FE, i, j + 1) - A2(FE, i, j)) +
                    A2(FSC[k2], i, j) - A2(FSC[k1], i, j));
    }
  }
#undef TS
}
