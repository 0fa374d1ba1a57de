/*
 * oracle_main.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 *
 * State allocation, initialisation sequence (main.F:85-321), the step
 * driver (main.F:333-520), global diagnostics (diag.F:58-659) and the
 * analytic cases (tests/Filament/ana_grid.h, ana_init.h; synthetic basin).
 */
#include <stdio.h>
#include "oracle_core.h"

static double *zalloc(size_t n) { return (double *)calloc(n ? n : 1, sizeof(double)); }

or_state *or_create(const or_cfg *cfg) {
  or_state *S = (or_state *)calloc(1, sizeof(or_state));
  S->c = *cfg;
  S->Lm = cfg->LLm; S->Mm = cfg->MMm; S->N = cfg->N; S->NT = cfg->NT;
  S->nTS = cfg->salinity ? 2 : 1;
  S->nx2 = S->Lm + 4; S->ny2 = S->Mm + 4;
  S->n2 = (size_t)S->nx2 * S->ny2;
  S->n3 = S->n2 * S->N;
  S->n3w = S->n2 * (S->N + 1);
  /* tile 0 covers the whole (single-rank) subdomain: compute_tile_bounds.h */
  S->istr = 1; S->iend = S->Lm; S->jstr = 1; S->jend = S->Mm;
  /* physical edges: WESTERN_EDGE etc. (set_global_definitions.h:174-262) */
  S->west_edge = S->east_edge = !cfg->ew_periodic;
  S->south_edge = S->north_edge = !cfg->ns_periodic;
  /* compute_auxiliary_bounds.h */
  S->istrR = S->west_edge ? S->istr - 1 : S->istr;
  S->istrU = S->west_edge ? S->istr + 1 : S->istr;
  S->iendR = S->east_edge ? S->iend + 1 : S->iend;
  S->jstrR = S->south_edge ? S->jstr - 1 : S->jstr;
  S->jstrV = S->south_edge ? S->jstr + 1 : S->jstr;
  S->jendR = S->north_edge ? S->jend + 1 : S->jend;
  /* compute_extended_bounds.h */
  S->istrE = cfg->ew_periodic ? S->istr - 2 : S->istr - 1;
  S->iendE = cfg->ew_periodic ? S->iend + 2 : S->iend + 1;
  S->jstrE = cfg->ns_periodic ? S->jstr - 2 : S->jstr - 1;
  S->jendE = cfg->ns_periodic ? S->jend + 2 : S->jend + 1;
  /* scalars (scalars.F:126-130, eos_vars.F:24, init_scalars.F) */
  S->g = 9.81; S->vonKar = 0.41; S->qp2 = 0.0000172; S->gamma2 = 1.0;
  S->rho0 = cfg->rho0; S->dt = cfg->dt; S->dtfast = cfg->dt / (double)cfg->ndtfast;
  S->Cs_w = zalloc(S->N + 1); S->Cs_r = zalloc(S->N + 1);
  const size_t n2 = S->n2, n3 = S->n3, n3w = S->n3w;
  double **g2[] = {&S->h, &S->hinv, &S->f, &S->fomn, &S->xr, &S->yr, &S->pm, &S->pn, &S->dm_r, &S->dn_r,
                   &S->pn_u, &S->dm_u, &S->dn_u, &S->dm_v, &S->pm_v, &S->dn_v, &S->dm_p, &S->dn_p, &S->iA_u,
                   &S->iA_v, &S->pmon_u, &S->pnom_v, &S->rmask, &S->pmask, &S->umask, &S->vmask, &S->rufrc,
                   &S->rvfrc, &S->rhoA, &S->rhoS, &S->r_D, &S->Zt_avg1, &S->DU_avg1, &S->DV_avg1, &S->DU_avg2,
                   &S->DV_avg2, &S->DU_avg_bak, &S->DV_avg_bak, &S->visc2_r, &S->visc2_p, &S->sustr, &S->svstr,
                   &S->srflx, &S->swflx, &S->hbls, &S->hbbl};
  for (size_t q = 0; q < sizeof(g2) / sizeof(g2[0]); q++) *g2[q] = zalloc(n2);
  S->zeta = zalloc(4 * n2); S->ubar = zalloc(4 * n2); S->vbar = zalloc(4 * n2);
  S->u = zalloc(3 * n3); S->v = zalloc(3 * n3);
  S->t = zalloc(3 * n3 * S->NT);
  S->FlxU = zalloc(n3); S->FlxV = zalloc(n3); S->Hz = zalloc(n3); S->Hz_u = zalloc(n3); S->Hz_v = zalloc(n3);
  S->z_r = zalloc(n3); S->z_w = zalloc(n3w); S->We = zalloc(n3w); S->Wi = zalloc(n3w);
  S->rho = zalloc(n3); S->rho1 = zalloc(n3); S->qp1 = zalloc(n3); S->bvf = zalloc(n3w);
  S->Akv = zalloc(n3w); S->Akt = zalloc(n3w * S->nTS);
  S->ghat = zalloc(n3w); S->swr_frac = zalloc(n3w);
  S->diff2 = zalloc(n2 * S->NT); S->stflx = zalloc(n2 * S->NT);
  S->ru = zalloc(n3); S->rv = zalloc(n3); S->P = zalloc(n3); S->rhos3 = zalloc(n3);
  for (int q = 0; q < 14; q++) S->s2[q] = zalloc(n2);
  for (int q = 0; q < 6; q++) S->c1[q] = zalloc((size_t)S->nx2 * (S->N + 1));
  if (cfg->lmd) or_lmd_alloc(S);
  if (cfg->adv_isoneutral) {
    S->dRdx = zalloc(n3); S->dRde = zalloc(n3); S->idRz = zalloc(n3w);
    S->diff3u = zalloc(n3); S->diff3v = zalloc(n3); S->Akz = zalloc(n3w);
    S->iso_FSC = zalloc(2 * n2); S->iso_dTdz = zalloc(2 * n2); S->iso_dTdx = zalloc(2 * n2);
    S->iso_dTde = zalloc(2 * n2); S->iso_LapT = zalloc(n3);
  }
  S->pipe_flx = zalloc(n2); S->pipe_idx = zalloc(n2);
  S->npip = 1;
  S->pipe_prf = zalloc((size_t)S->N); S->pipe_trc = zalloc((size_t)S->NT);
  S->riv_uflx = zalloc(n2); S->riv_vflx = zalloc(n2);
  S->uwnd = zalloc(n2); S->vwnd = zalloc(n2); S->tair = zalloc(n2); S->qair = zalloc(n2); S->prate = zalloc(n2);
  S->swrad = zalloc(n2); S->lwrad = zalloc(n2); S->sustr_r = zalloc(n2); S->svstr_r = zalloc(n2);
  S->dndx = zalloc(n2); S->dmde = zalloc(n2); S->ptide = zalloc(n2);
  /* boundary.F:111-129: zeta_west(0:Mm+1), u_west(0:Mm+1,N), t_west(0:Mm+1,N,NT), ... */
  S->nbry[0] = S->nbry[1] = S->Mm + 2;
  S->nbry[2] = S->nbry[3] = S->Lm + 2;
  for (int q = 0; q < 4; q++) {
    const size_t nb = (size_t)S->nbry[q];
    S->bry_zeta[q] = zalloc(nb); S->bry_ubar[q] = zalloc(nb); S->bry_vbar[q] = zalloc(nb);
    S->bry_u[q] = zalloc(nb * S->N); S->bry_v[q] = zalloc(nb * S->N); S->bry_t[q] = zalloc(nb * S->N * S->NT);
  }
  if (cfg->obc && (S->Lm + 4 > 4200 || S->Mm + 4 > 4200)) { fprintf(stderr, "oracle: OBC strips limited to 4196 points\n"); return NULL; }
  return S;
}

void or_destroy(or_state *S) {
  if (!S) return;
  /* process exit reclaims memory in tests; free the big ones */
  free(S->u); free(S->v); free(S->t); free(S->zeta); free(S->ubar); free(S->vbar);
  for (int q = 0; q < S->nfrc; q++) { free(S->frc[q].rec[0]); free(S->frc[q].rec[1]); free(S->frc[q].rec[2]); }
  free(S);
}

/* ---------------------------------------------------------------------- */
/* set_scoord (set_scoord.F:4-66): SM09 stretching functions               */
/* ---------------------------------------------------------------------- */
static double CSF(double sc, double theta_s, double theta_b) {
  double csrf, r;
  if (theta_s > 0.0) csrf = (1.0 - cosh(theta_s * sc)) / (cosh(theta_s) - 1.0);
  else csrf = -(sc * sc);
  if (theta_b > 0.0) r = (exp(theta_b * csrf) - 1.0) / (1.0 - exp(-theta_b));
  else r = csrf;
  return r;
}
static void set_scoord(or_state *S) {
  const int N = S->N;
  const double ds = 1.0 / (double)N;
  S->Cs_w[N] = 0.0;
  for (int k = N - 1; k >= 1; k--) S->Cs_w[k] = CSF(ds * (double)(k - N), S->c.theta_s, S->c.theta_b);
  S->Cs_w[0] = -1.0;
  for (int k = 1; k <= N; k++) S->Cs_r[k] = CSF(ds * ((double)(k - N) - 0.5), S->c.theta_s, S->c.theta_b);
}

/* ---------------------------------------------------------------------- */
/* set_weights (set_weights.F:7-235): p=2,q=4,r=0.25 power-law filter      */
/* ---------------------------------------------------------------------- */
static void set_weights(or_state *S) {
  const int ndtfast = S->c.ndtfast;
  double (*w)[288] = S->weight;
  int nfast = 0;
  for (int i = 1; i <= 2 * ndtfast; i++) { w[0][i - 1] = 0.0; w[1][i - 1] = 0.0; }
  const double p = 2.0, q = 4.0, r = 0.25;
  double scale = (p + 1.0) * (p + q + 1.0) / ((p + 2.0) * (p + q + 2.0) * (double)ndtfast);
  double sum, shft, cff;
  for (int iter = 1; iter <= 16; iter++) {
    nfast = 0;
    for (int i = 1; i <= 2 * ndtfast; i++) {
      cff = scale * (double)i;
      w[0][i - 1] = pow(cff, p) - pow(cff, p + q) - r * cff;
      if (w[0][i - 1] > 0.0) nfast = i;
      if (nfast > 0 && w[0][i - 1] < 0.0) w[0][i - 1] = 0.0;
    }
    sum = 0.0; shft = 0.0;
    for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; shft = shft + w[0][i - 1] * (double)i; }
    scale = scale * shft / (sum * (double)ndtfast);
  }
  for (int iter = 1; iter <= ndtfast; iter++) {
    sum = 0.0; shft = 0.0;
    for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; shft = shft + (double)i * w[0][i - 1]; }
    shft = shft / sum;
    cff = (double)ndtfast - shft;
    if (cff > 1.0) {
      nfast = nfast + 1;
      for (int i = nfast; i >= 2; i--) w[0][i - 1] = w[0][i - 2];
      w[0][0] = 0.0;
    } else if (cff > 0.0) {
      sum = 1.0 - cff;
      for (int i = nfast; i >= 2; i--) w[0][i - 1] = sum * w[0][i - 1] + cff * w[0][i - 2];
      w[0][0] = sum * w[0][0];
    } else if (cff < -1.0) {
      nfast = nfast - 1;
      for (int i = 1; i <= nfast; i++) w[0][i - 1] = w[0][i];
      w[0][nfast] = 0.0;
    } else if (cff < 0.0) {
      sum = 1.0 + cff;
      for (int i = 1; i <= nfast - 1; i++) w[0][i - 1] = sum * w[0][i - 1] - cff * w[0][i];
      w[0][nfast - 1] = sum * w[0][nfast - 1];
    }
  }
  for (int j = 1; j <= nfast; j++) {
    cff = w[0][j - 1];
    for (int i = 1; i <= j; i++) w[1][i - 1] = w[1][i - 1] + cff;
  }
  sum = 0.0; cff = 0.0;
  for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; cff = cff + w[1][i - 1]; }
  sum = 1.0 / sum; cff = 1.0 / cff;
  for (int i = 1; i <= nfast; i++) { w[0][i - 1] = sum * w[0][i - 1]; w[1][i - 1] = cff * w[1][i - 1]; }
  S->nfast = nfast;
}

/* ---------------------------------------------------------------------- */
/* setup_grid1 (setup_grid1.F): metric combinations, masks                 */
/* ---------------------------------------------------------------------- */
static void setup_grid1(or_state *S) {
  for (int j = S->jstrE; j <= S->jendE; j++)
    for (int i = S->istrE; i <= S->iendE; i++)
      A2(S->fomn, i, j) = A2(S->f, i, j) / (A2(S->pm, i, j) * A2(S->pn, i, j));
  const double *pm = S->pm, *pn = S->pn, *rm = S->rmask;
  for (int j = S->jstrR; j <= S->jendR; j++)
    for (int i = S->istrR; i <= S->iendR; i++) {
      A2(S->dm_r, i, j) = 1.0 / A2(pm, i, j);
      A2(S->dn_r, i, j) = 1.0 / A2(pn, i, j);
    }
  for (int j = S->jstrR; j <= S->jendR; j++)
    for (int i = S->istr; i <= S->iendR; i++) {
      A2(S->pmon_u, i, j) = (A2(pm, i, j) + A2(pm, i - 1, j)) / (A2(pn, i, j) + A2(pn, i - 1, j));
      A2(S->dm_u, i, j) = 2.0 / (A2(pm, i, j) + A2(pm, i - 1, j));
      A2(S->dn_u, i, j) = 2.0 / (A2(pn, i, j) + A2(pn, i - 1, j));
      A2(S->pn_u, i, j) = 0.5 * (A2(pn, i, j) + A2(pn, i - 1, j));
      A2(S->umask, i, j) = A2(rm, i, j) * A2(rm, i - 1, j);
      A2(S->iA_u, i, j) = 0.25 * (A2(pm, i, j) + A2(pm, i - 1, j)) * (A2(pn, i, j) + A2(pn, i - 1, j));
    }
  for (int j = S->jstr; j <= S->jendR; j++)
    for (int i = S->istrR; i <= S->iendR; i++) {
      A2(S->pnom_v, i, j) = (A2(pn, i, j) + A2(pn, i, j - 1)) / (A2(pm, i, j) + A2(pm, i, j - 1));
      A2(S->dm_v, i, j) = 2.0 / (A2(pm, i, j) + A2(pm, i, j - 1));
      A2(S->dn_v, i, j) = 2.0 / (A2(pn, i, j) + A2(pn, i, j - 1));
      A2(S->pm_v, i, j) = 0.5 * (A2(pm, i, j) + A2(pm, i, j - 1));
      A2(S->vmask, i, j) = A2(rm, i, j) * A2(rm, i, j - 1);
      A2(S->iA_v, i, j) = 0.25 * (A2(pm, i, j) + A2(pm, i, j - 1)) * (A2(pn, i, j) + A2(pn, i, j - 1));
    }
  for (int j = S->jstr; j <= S->jendR; j++)
    for (int i = S->istr; i <= S->iendR; i++) {
      A2(S->dm_p, i, j) = 4.0 / (A2(pm, i, j) + A2(pm, i, j - 1) + A2(pm, i - 1, j) + A2(pm, i - 1, j - 1));
      A2(S->dn_p, i, j) = 4.0 / (A2(pn, i, j) + A2(pn, i, j - 1) + A2(pn, i - 1, j) + A2(pn, i - 1, j - 1));
      const int a = A2(rm, i - 1, j) > 0.5, b = A2(rm, i, j) > 0.5, c = A2(rm, i - 1, j - 1) > 0.5, d = A2(rm, i, j - 1) > 0.5;
      const int n = a + b + c + d;
      double pmk;
      if (n == 4) pmk = 1.0;
      else if (n == 3) pmk = 1.0;                      /* cff1 */
      else if (n == 2 && ((a && c) || (b && d) || (a && b) || (c && d))) pmk = 2.0; /* cff2: straight wall */
      else pmk = 0.0;
      A2(S->pmask, i, j) = pmk;
    }
  double *ex[] = {S->dm_r, S->dn_r, S->dm_p, S->dn_p, S->dm_u, S->dn_u, S->iA_u, S->dm_v, S->dn_v,
                  S->iA_v, S->pmon_u, S->pnom_v, S->rmask, S->umask, S->vmask, S->pmask};
  for (size_t q = 0; q < sizeof(ex) / sizeof(ex[0]); q++) or_exch2(S, ex[q]);
  if (S->c.curvgrid) {  /* setup_grid1.F:89-103, exchanged at :203 */
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istr; i <= S->iend; i++) A2(S->dndx, i, j) = 0.5 / A2(pn, i + 1, j) - 0.5 / A2(pn, i - 1, j);
    for (int j = S->jstr; j <= S->jend; j++)
      for (int i = S->istrR; i <= S->iendR; i++) A2(S->dmde, i, j) = 0.5 / A2(pm, i, j + 1) - 0.5 / A2(pm, i, j - 1);
    or_exch2(S, S->dndx);
    or_exch2(S, S->dmde);
  }
}

/* ---------------------------------------------------------------------- */
/* reduction-by-pairs within a rank (diag.F:409-471, setup_grid2.F)       */
/* ---------------------------------------------------------------------- */
static double pair_reduce(or_state *S, double *A, int istr, int iend, int jstr, int jend) {
  int isize = iend - istr, jsize = jend - jstr;
  while (isize > 0 || jsize > 0) {
    if (jsize > 0) {
      int js = (jsize + 1) / 2 - 1;
      for (int j = 0; j <= js; j++) {
        int jtg = jstr + j;
        for (int i = istr; i <= istr + isize; i++) A2(A, i, jtg) = A2(A, i, jtg + j) + A2(A, i, jtg + j + 1);
      }
      if (2 * js + 1 < jsize) {
        js = js + 1;
        int jtg = jstr + js;
        for (int i = istr; i <= istr + isize; i++) A2(A, i, jtg) = A2(A, i, jtg + js);
      }
      jsize = js;
    }
    if (isize > 0) {
      int is = (isize + 1) / 2 - 1;
      for (int j = jstr; j <= jstr + jsize; j++)
        for (int i = 0; i <= is; i++) {
          int itg = istr + i;
          A2(A, itg, j) = A2(A, itg + i, j) + A2(A, itg + i + 1, j);
        }
      if (2 * is + 1 < isize) {
        is = is + 1;
        int itg = istr + is;
        for (int j = jstr; j <= jstr + jsize; j++) A2(A, itg, j) = A2(A, itg + is, j);
      }
      isize = is;
    }
  }
  return A2(A, istr, jstr);
}

/* rank sub-domain bounds of an NP_XI x NP_ETA decomposition (mpi_setup.F:115-155) */
static void rank_bounds(int LLm, int np, int node, int *i0, int *i1) {
  int Lm = (LLm + np - 1) / np, off = np * Lm - LLm, sw, lm = Lm;
  if (node == 0) sw = 0; else sw = node * Lm - off / 2;
  if (node == 0) lm = lm - off / 2;
  if (node == np - 1) lm = lm - (off + 1) / 2;
  *i0 = sw + 1; *i1 = sw + lm;
}

/* tree summation over ranks (diag.F:488-535): receiver r adds r+step */
static double tree_sum(double *v, int n) {
  int size = n;
  while (size > 1) {
    int step = (size + 1) / 2;
    for (int r = 0; r < size - step; r++) v[r] = v[r] + v[r + step];
    size = step;
  }
  return v[0];
}

static void rank_sums(or_state *S, double **fields, int nf, double *out) {
  const int npx = S->c.diag_np_xi > 0 ? S->c.diag_np_xi : 1, npe = S->c.diag_np_eta > 0 ? S->c.diag_np_eta : 1;
  const int nr = npx * npe;
  double vals[64][8];
  for (int jn = 0; jn < npe; jn++)
    for (int in = 0; in < npx; in++) {
      int i0, i1, j0, j1;
      rank_bounds(S->Lm, npx, in, &i0, &i1);
      rank_bounds(S->Mm, npe, jn, &j0, &j1);
      for (int f = 0; f < nf; f++) vals[in + jn * npx][f] = pair_reduce(S, fields[f], i0, i1, j0, j1);
    }
  for (int f = 0; f < nf; f++) {
    double v[64];
    for (int r = 0; r < nr; r++) v[r] = vals[r][f];
    out[f] = tree_sum(v, nr);
  }
}

static void setup_grid2(or_state *S) {
  double *dA = S->s2[0], *dV = S->s2[1];
  for (int j = 1; j <= S->Mm; j++)
    for (int i = 1; i <= S->Lm; i++) {
      A2(dA, i, j) = A2(S->rmask, i, j) / (A2(S->pm, i, j) * A2(S->pn, i, j));
      A2(dV, i, j) = A2(dA, i, j) * A2(S->h, i, j);
    }
  double *fl[2] = {dA, dV};
  double out[2];
  rank_sums(S, fl, 2, out);
  S->area = out[0];
  S->volume = out[1];
}

/* ---------------------------------------------------------------------- */
/* diag_tile (diag.F:58-659), code_check line: KE, BAROTR_KE, CFLs         */
/* ---------------------------------------------------------------------- */
void or_diag(or_state *S) {
  const int N = S->N, nstp = S->nstp;
  double *ub = S->s2[6], *vb = S->s2[7], *ke = S->s2[0], *ke2b = S->s2[1], *dVol = S->s2[2];
  for (int j = 1; j <= S->Mm + 1; j++) {
    for (int i = 1; i <= S->Lm + 1; i++) {
      A2(ub, i, j) = (HZ(i, j, N) + HZ(i - 1, j, N)) * U(i, j, N, nstp);
      A2(vb, i, j) = (HZ(i, j, N) + HZ(i, j - 1, N)) * V(i, j, N, nstp);
    }
    for (int k = N - 1; k >= 2; k--)
      for (int i = 1; i <= S->Lm + 1; i++) {
        A2(ub, i, j) = A2(ub, i, j) + (HZ(i, j, k) + HZ(i - 1, j, k)) * U(i, j, k, nstp);
        A2(vb, i, j) = A2(vb, i, j) + (HZ(i, j, k) + HZ(i, j - 1, k)) * V(i, j, k, nstp);
      }
    for (int i = 1; i <= S->Lm + 1; i++) {
      A2(ub, i, j) = (A2(ub, i, j) + (HZ(i, j, 1) + HZ(i - 1, j, 1)) * U(i, j, 1, nstp)) /
                     (ZW(i, j, N) + ZW(i - 1, j, N) - ZW(i, j, 0) - ZW(i - 1, j, 0));
      A2(vb, i, j) = (A2(vb, i, j) + (HZ(i, j, 1) + HZ(i, j - 1, 1)) * V(i, j, 1, nstp)) /
                     (ZW(i, j, N) + ZW(i, j - 1, N) - ZW(i, j, 0) - ZW(i, j - 1, 0));
    }
  }
  /* per-rank Cu maxima scanned in the reference loop order, then tree-max */
  const int npx = S->c.diag_np_xi > 0 ? S->c.diag_np_xi : 1, npe = S->c.diag_np_eta > 0 ? S->c.diag_np_eta : 1;
  double rCu[64], rCw[64];
  for (int r = 0; r < npx * npe; r++) { rCu[r] = 0.0; rCw[r] = 0.0; }
  for (int j = 1; j <= S->Mm; j++)
    for (int i = 1; i <= S->Lm; i++) {
      const double v2b = 0.5 * (A2(ub, i, j) * A2(ub, i, j) + A2(ub, i + 1, j) * A2(ub, i + 1, j) +
                                A2(vb, i, j) * A2(vb, i, j) + A2(vb, i, j + 1) * A2(vb, i, j + 1));
      A2(ke, i, j) = 0.0;
      A2(ke2b, i, j) = 0.5 * (ZW(i, j, N) - ZW(i, j, 0)) * v2b;
    }
  for (int jn = 0; jn < npe; jn++)
    for (int in = 0; in < npx; in++) {
      int i0, i1, j0, j1, r = in + jn * npx;
      rank_bounds(S->Lm, npx, in, &i0, &i1);
      rank_bounds(S->Mm, npe, jn, &j0, &j1);
      for (int j = j0; j <= j1; j++)
        for (int k = N; k >= 1; k--)
          for (int i = i0; i <= i1; i++) {
            const double u0 = U(i, j, k, nstp), u1 = U(i + 1, j, k, nstp), v0 = V(i, j, k, nstp), v1 = V(i, j + 1, k, nstp);
            const double v2 = 0.5 * (u0 * u0 + u1 * u1 + v0 * v0 + v1 * v1);
            const double ciV = S->dt * A2(S->rmask, i, j) * A2(S->pm, i, j) * A2(S->pn, i, j) / HZ(i, j, k);
            const double cw = ciV * (fmax0(WE(i, j, k) + WI(i, j, k)) - fmin0(WE(i, j, k - 1) + WI(i, j, k - 1)));
            const double cx = cw + ciV * (fmax0(FLXU(i + 1, j, k)) - fmin0(FLXU(i, j, k)) + fmax0(FLXV(i, j + 1, k)) -
                                          fmin0(FLXV(i, j, k)));
            if (cx > rCu[r]) { rCu[r] = cx; rCw[r] = cw; }
            A2(ke, i, j) = A2(ke, i, j) + 0.5 * v2 * HZ(i, j, k);
          }
    }
  for (int j = 1; j <= S->Mm; j++)
    for (int i = 1; i <= S->Lm; i++) {
      const double dA = A2(S->rmask, i, j) / (A2(S->pm, i, j) * A2(S->pn, i, j));
      A2(dVol, i, j) = dA * ZW(i, j, N);
      A2(ke, i, j) = dA * A2(ke, i, j);
      A2(ke2b, i, j) = dA * A2(ke2b, i, j);
    }
  double *fl[3] = {dVol, ke, ke2b};
  double out[3];
  rank_sums(S, fl, 3, out);
  /* tree max for Cu_Adv (strict '>' as diag.F:526) */
  int size = npx * npe;
  while (size > 1) {
    int step = (size + 1) / 2;
    for (int r = 0; r < size - step; r++)
      if (rCu[r + step] > rCu[r]) { rCu[r] = rCu[r + step]; rCw[r] = rCw[r + step]; }
    size = step;
  }
  const double avzeta = out[0];
  S->avke = out[1] / (S->volume + avzeta);
  S->avke2b = out[2] / (S->volume + avzeta);
  S->Cu_Adv = rCu[0];
  S->Cu_W = rCw[0];
  S->norms[0] = S->avke; S->norms[1] = S->avke2b; S->norms[2] = S->Cu_Adv; S->norms[3] = S->Cu_W;
}

/* ---------------------------------------------------------------------- */
/* analytic cases                                                          */
/* ---------------------------------------------------------------------- */
void or_ana_grid(or_state *S) {
  const int nx = S->Lm, ny = S->Mm;
  if (S->c.case_id == OR_CASE_FILAMENT) {
    /* tests/Filament/ana_grid.h:11-56 */
    const double SizeX = S->c.sizex, SizeY = S->c.sizey;
    const double f0 = 2 * 7.81e-5, beta = 0;
    const double dx = SizeX / S->c.LLm, dy = SizeY / S->c.MMm;
    const double x_mid = SizeX / 2.0;
    double x0 = dx * 0.0, y0 = dy * 0.0;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        A2(S->xr, i, j) = x0 + dx * ((double)i - 0.5) - x_mid;
        A2(S->yr, i, j) = y0 + dy * ((double)j - 0.5);
        A2(S->pm, i, j) = 1.0 / dx;
        A2(S->pn, i, j) = 1.0 / dy;
      }
    x0 = SizeX / 2.0; y0 = SizeY / 2.0;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) A2(S->f, i, j) = f0 + beta * (A2(S->yr, i, j) - y0);
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) { A2(S->h, i, j) = 1000; A2(S->rmask, i, j) = 1; }
  } else if (S->c.case_id == OR_CASE_PIPES) {
    /* tests/Pipes_ana/ana_grid.h:19-131 (single rank: iSW_corn = jSW_corn = 0) */
    const double SizeX = S->c.sizex, SizeY = S->c.sizey, f0 = 1.0e-4, beta = 0;
    const double dx = SizeX / S->c.LLm, dy = SizeY / S->c.MMm;
    double x0 = 0., y0 = 0.;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        A2(S->xr, i, j) = x0 + dx * ((double)i - 0.5);
        A2(S->yr, i, j) = y0 + dy * ((double)j - 0.5);
        A2(S->pm, i, j) = 1. / dx;
        A2(S->pn, i, j) = 1. / dy;
      }
    x0 = SizeX / 2.; y0 = SizeY / 2.;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) A2(S->f, i, j) = f0 + beta * (A2(S->yr, i, j) - y0);
    const double depth = 10, max_depth = 100;
    const double shelf = SizeY / 5, slope = (max_depth - depth) / (SizeY * 4 / 5);
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        if (A2(S->yr, i, j) < shelf) A2(S->h, i, j) = depth;
        else A2(S->h, i, j) = depth + (A2(S->yr, i, j) - shelf) * slope;
      }
    const double land = SizeY * 0.1, coast = SizeY * 0.02, riv_west = SizeX * 0.4, riv_east = SizeX * 0.6;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        A2(S->rmask, i, j) = 1;
        if (A2(S->yr, i, j) < land)
          if (A2(S->xr, i, j) < riv_west || A2(S->xr, i, j) > riv_east) A2(S->rmask, i, j) = 0.0;
        if (A2(S->yr, i, j) < coast) A2(S->rmask, i, j) = 0.0;
      }
    /* pipe location; ana_pipe_frc.h: pipe_vol = 5e2, pipe_trc = (24, 1), pipe_prf(1:2) = 0.5 */
    const double psz = SizeX * 0.02, px = SizeX * .5, py = SizeY * .5;
    const double pipe_cells = (double)(lround(psz / dx) * lround(psz / dx));
    S->pipe_source = 1;
    S->npip = 1;
    for (int k = 0; k < S->N; k++) S->pipe_prf[k] = 0.0;
    S->pipe_prf[0] = 0.5; S->pipe_prf[1] = 0.5;
    S->pipe_trc[0] = 24.0; S->pipe_trc[1] = 1.0;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        double frac = 0.0, idx = 0.0;
        if (A2(S->xr, i, j) > px - 0.5 * psz && A2(S->xr, i, j) < px + 0.5 * psz)
          if (A2(S->yr, i, j) > py - 0.5 * psz && A2(S->yr, i, j) < py + 0.5 * psz) { frac = 1.0 / pipe_cells; idx = 1; }
        A2(S->pipe_idx, i, j) = idx;
        A2(S->pipe_flx, i, j) = frac * 5e2;
      }
  } else if (S->c.case_id == OR_CASE_RIVERS) {
    /* tests/Rivers_ana/ana_grid.h:1-101 (single rank: iSW_corn = jSW_corn = 0),
       loops over 0..ny+1, 0..nx+1 as written */
    const double Size_XI = 1.0e4, Size_ETA = 1.0e4, depth = 5., max_depth = 100.0, f0 = 0.0e-4, beta = 0.;
    const double xl = Size_XI, el = Size_ETA;
    const double dx = Size_XI / (double)S->c.LLm, dy = Size_ETA / (double)S->c.MMm;
    double x0 = 0., y0 = 0.;
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) {
        A2(S->xr, i, j) = x0 + dx * ((double)i - 0.5);
        A2(S->yr, i, j) = y0 + dy * ((double)j - 0.5);
        A2(S->pm, i, j) = 1. / dx;
        A2(S->pn, i, j) = 1. / dy;
      }
    x0 = Size_XI / 2.; y0 = Size_ETA / 2.;
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) A2(S->f, i, j) = f0 + beta * (A2(S->yr, i, j) - y0);
    const double shelf = Size_ETA / 5, slope = (max_depth - depth) / (Size_ETA * 4 / 5);
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) {
        if (A2(S->yr, i, j) < shelf) A2(S->h, i, j) = depth;
        else A2(S->h, i, j) = depth + (A2(S->yr, i, j) - shelf) * slope;
      }
    const double land = el * 0.1, coast = el * 0.02, riv_west = xl * 0.4, riv_east = xl * 0.6;
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) {
        A2(S->rmask, i, j) = 1;
        if (A2(S->yr, i, j) < land)
          if (A2(S->xr, i, j) < riv_west || A2(S->xr, i, j) > riv_east) A2(S->rmask, i, j) = 0.0;
        if (A2(S->yr, i, j) < coast) A2(S->rmask, i, j) = 0.0;
      }
    /* river_frc.F init_river_frc (analytical, :118-135) + calc_river_flux
       (:228-282); one river, ana_frc_river.h: riv_vol = 5e2, riv_trc = (24, 1) */
    S->river_source = 1;
    S->nriv = 1;
    S->riv_vol[0] = 5e2;
    S->riv_trc[0] = 24.0;
    if (S->NT > 1) S->riv_trc[1] = 1.0;
    const double riv_cells = (double)lround((riv_east - riv_west) * A2(S->pm, 1, 1));
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) {
        if (!(A2(S->xr, i, j) > riv_west && A2(S->xr, i, j) < riv_east)) continue;
        if (!(A2(S->rmask, i, j) == 0 && A2(S->rmask, i, j + 1) == 1)) continue;
        const double rfrc = 1 / riv_cells;
        const int ridx = 1;
        /* faces is an integer in calc_river_flux (river_frc.F:233) */
        const int faces = (int)(A2(S->rmask, i - 1, j) + A2(S->rmask, i + 1, j) + A2(S->rmask, i, j - 1) + A2(S->rmask, i, j + 1));
        if (A2(S->rmask, i - 1, j) > 0) A2(S->riv_uflx, i, j) = -(rfrc) / faces + 10 * ridx;
        if (A2(S->rmask, i + 1, j) > 0) A2(S->riv_uflx, i + 1, j) = (rfrc) / faces + 10 * ridx;
        if (A2(S->rmask, i, j - 1) > 0) A2(S->riv_vflx, i, j) = -(rfrc) / faces + 10 * ridx;
        if (A2(S->rmask, i, j + 1) > 0) A2(S->riv_vflx, i, j + 1) = (rfrc) / faces + 10 * ridx;
      }
  } else {
    /* synthetic closed basin (C3 stand-in) */
    const double dx = S->c.sizex / S->c.LLm, dy = S->c.sizey / S->c.MMm;
    const double R = 0.5 * (S->c.sizex < S->c.sizey ? S->c.sizex : S->c.sizey);
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        const double x = dx * ((double)i - 0.5), y = dy * ((double)j - 0.5);
        A2(S->xr, i, j) = x; A2(S->yr, i, j) = y;
        A2(S->pm, i, j) = 1.0 / dx; A2(S->pn, i, j) = 1.0 / dy;
        if (S->c.curvgrid) {  /* non-uniform metrics: m varies along eta, n along xi */
          const double pi = 3.14159265358979323;
          A2(S->pm, i, j) = (1.0 + 0.1 * sin(2.0 * pi * ((double)j - 0.5) / (double)S->c.MMm)) / dx;
          A2(S->pn, i, j) = (1.0 + 0.1 * cos(2.0 * pi * ((double)i - 0.5) / (double)S->c.LLm)) / dy;
        }
        A2(S->f, i, j) = 1.0e-4;
        const double rx = x - 0.5 * S->c.sizex, ry = y - 0.5 * S->c.sizey;
        double s = 1.0 - (rx * rx + ry * ry) / (R * R);
        if (s < 0.0) s = 0.0;
        A2(S->h, i, j) = 200.0 + 3800.0 * s;
        A2(S->rmask, i, j) = 1.0;
        if (S->c.island) {  /* circular island of radius 0.1 min(Lx,Ly) at (0.35 Lx, 0.6 Ly) */
          const double ix = x - 0.35 * S->c.sizex, iy = y - 0.6 * S->c.sizey, ir = 0.2 * R;
          if (ix * ix + iy * iy < ir * ir) A2(S->rmask, i, j) = 0.0;
        }
      }
  }
}

void or_ana_init(or_state *S) {
  const int nx = S->Lm, ny = S->Mm, nz = S->N;
  S->forw_start = S->ntstart;
  if (S->c.case_id == OR_CASE_FILAMENT) {
    /* tests/Filament/ana_init.h:16-140 */
    const double b0 = 5.0e-2, B_cff = 0.025, lambda_inv = 8.0, Nb = 1.0e-7, N0 = 3.0e-5, h0 = 60.0, dh0 = 15.,
                 L = 2000.0, HD = 1000;
    const double g = S->g, alpha = S->c.Tcoef / S->rho0;
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) {
        const double xl = A2(S->xr, i, j) / L;
        const double h_sbl = h0 + dh0 * exp(-(xl * xl));
        for (int k = 1; k <= nz; k++) {
          const double zr = ZR(i, j, k);
          const double b = b0 + Nb * (zr + HD) +
                           0.5 * N0 * ((1 + B_cff) * zr - (1 - B_cff) * (h_sbl + lambda_inv * log(cosh((1. / lambda_inv) * (zr + h_sbl)))));
          TT(i, j, k, 1, 1) = b / (g * alpha);
        }
      }
    double bf_int = 0;
    for (int k = 1; k <= nz; k++) {
      const double zr = ZR(1, 1, k);
      bf_int = bf_int + HZ(1, 1, k) *
                            (b0 + Nb * (zr + HD) +
                             0.5 * N0 * ((1 + B_cff) * zr - (1 - B_cff) * (h0 + lambda_inv * log(cosh((1. / lambda_inv) * (zr + h0)))))) /
                            g;
    }
    for (int k = 1; k <= nz; k++)
      for (int j = -1; j <= ny + 2; j++)
        for (int i = -1; i <= nx + 2; i++) {
          TT(i, j, k, 2, 1) = TT(i, j, k, 1, 1);
          if (S->c.salinity) { TT(i, j, k, 1, 2) = 36.; TT(i, j, k, 2, 2) = TT(i, j, k, 1, 2); }
        }
    memset(S->zeta, 0, 4 * S->n2 * sizeof(double));
    for (int k = 1; k <= nz; k++)
      for (int j = -1; j <= ny + 2; j++)
        for (int i = -1; i <= nx + 2; i++) ZETA(i, j, 1) = ZETA(i, j, 1) + TT(i, j, k, 1, 1) * alpha * HZ(i, j, k);
    for (int j = -1; j <= ny + 2; j++)
      for (int i = -1; i <= nx + 2; i++) ZETA(i, j, 1) = (ZETA(i, j, 1) - bf_int);
    for (int j = 0; j <= ny + 1; j++)
      for (int i = 0; i <= nx + 1; i++) {
        const double dzdx = 0.5 * A2(S->pm, i, j) * (ZETA(i + 1, j, 1) - ZETA(i - 1, j, 1));
        V(i, j, nz, 1) = g * dzdx / A2(S->f, i, j);
      }
    for (int k = nz - 1; k >= 1; k--)
      for (int j = 0; j <= ny + 1; j++)
        for (int i = 0; i <= nx + 1; i++) {
          const double dbdx = 0.25 * A2(S->pm, i, j) * g * alpha *
                              (TT(i + 1, j, k, 1, 1) - TT(i - 1, j, k, 1, 1) + TT(i + 1, j, k + 1, 1, 1) - TT(i - 1, j, k + 1, 1, 1));
          V(i, j, k, 1) = V(i, j, k + 1, 1) - dbdx * (ZR(i, j, k + 1) - ZR(i, j, k)) / A2(S->f, i, j);
        }
    memset(S->vbar, 0, 4 * S->n2 * sizeof(double));
    for (int k = nz - 1; k >= 1; k--)
      for (int j = 0; j <= ny + 1; j++)
        for (int i = 0; i <= nx + 1; i++) VBAR(i, j, 1) = VBAR(i, j, 1) + V(i, j, k, 1) * HZ(i, j, k) / HD;
    for (int j = 1; j <= ny; j++)
      for (int i = 1; i <= nx; i++) {
        UBAR(i, j, 1) = 0.;
        VBAR(i, j, 2) = VBAR(i, j, 1);
        ZETA(i, j, 2) = ZETA(i, j, 1);
        for (int k = 1; k <= nz; k++) { U(i, j, k, 1) = 0.; U(i, j, k, 2) = U(i, j, k, 1); V(i, j, k, 2) = V(i, j, k, 1); }
      }
  } else if (S->c.case_id == OR_CASE_PIPES || S->c.case_id == OR_CASE_RIVERS) {
    /* tests/Pipes_ana/ana_init.h:14-52, tests/Rivers_ana/ana_init.h:10-40:
       rest state, T = 4 + 10 e^{z/50}, S = 36 */
    for (int k = 1; k <= nz; k++)
      for (int j = 0; j <= ny + 1; j++)
        for (int i = 0; i <= nx + 1; i++) {
          TT(i, j, k, 1, 1) = 4. + 10. * exp(ZR(i, j, k) / 50.);
          TT(i, j, k, 1, 2) = 36.;
          TT(i, j, k, 2, 1) = TT(i, j, k, 1, 1);
          TT(i, j, k, 2, 2) = TT(i, j, k, 1, 2);
        }
  } else {
    /* synthetic basin: stratified T, weak S gradient, at rest */
    const double Lx = S->c.sizex, Ly = S->c.sizey, pi = 3.14159265358979323;
    for (int k = 1; k <= nz; k++)
      for (int j = -1; j <= ny + 2; j++)
        for (int i = -1; i <= nx + 2; i++) {
          const double x = A2(S->xr, i, j), y = A2(S->yr, i, j), ez = exp(ZR(i, j, k) / 500.0);
          TT(i, j, k, 1, 1) = 4.0 + 10.0 * ez + 0.5 * sin(2.0 * pi * x / Lx) * sin(2.0 * pi * y / Ly) * ez;
          TT(i, j, k, 2, 1) = TT(i, j, k, 1, 1);
          if (S->c.salinity) {
            TT(i, j, k, 1, 2) = 35.0 + 0.25 * cos(2.0 * pi * x / Lx);
            TT(i, j, k, 2, 2) = TT(i, j, k, 1, 2);
          }
          for (int it = 3; it <= S->NT; it++) {
            const double rx = (x - 0.3 * Lx) / (0.1 * Lx), ry = (y - 0.5 * Ly) / (0.1 * Ly);
            TT(i, j, k, 1, it) = exp(-(rx * rx + ry * ry)) * ez * (double)(it - 2);
            TT(i, j, k, 2, it) = TT(i, j, k, 1, it);
          }
        }
  }
  /* ana_init_generic: exchanges */
  or_exch2(S, S->zeta); or_exch2(S, S->ubar); or_exch2(S, S->vbar);
  or_exch3(S, S->u, S->N); or_exch3(S, S->v, S->N);
  for (int it = 1; it <= S->NT; it++) or_exch3(S, S->t + (size_t)(it - 1) * 3 * S->n3, S->N);
}

/* set_forces: analytic surface fluxes (analytical.F ana_smflux/srflux/stflux) */
void or_ana_forces(or_state *S) {
  if (S->c.case_id == OR_CASE_BASIN && S->c.bulk_frc) {
    /* BULK_FRC with a synthetic analytic atmosphere (C4 stand-in):
       westerly jet, air 2-3 degC below the sea surface, humid, light rain;
       with the in-step clock on, the atmosphere comes from the records */
    const double pi = 3.14159265358979323;
    for (int j = -1; j <= S->Mm + 2 && !S->frc_clock; j++)
      for (int i = -1; i <= S->Lm + 2; i++) {
        const double x = A2(S->xr, i, j), y = A2(S->yr, i, j);
        A2(S->uwnd, i, j) = 8.0 * sin(pi * y / S->c.sizey);
        A2(S->vwnd, i, j) = 2.0 * cos(pi * x / S->c.sizex);
        A2(S->tair, i, j) = 10.0 + 3.0 * cos(2.0 * pi * x / S->c.sizex);
        A2(S->qair, i, j) = 0.007 + 0.001 * sin(2.0 * pi * y / S->c.sizey);
        A2(S->prate, i, j) = 0.3;
        A2(S->swrad, i, j) = 150.0 + 50.0 * sin(pi * y / S->c.sizey);
        A2(S->lwrad, i, j) = 320.0;
      }
    or_bulk_flux(S);
    return;
  }
  if (S->c.case_id == OR_CASE_BASIN) {
    const double pi = 3.14159265358979323;
    for (int j = -1; j <= S->Mm + 2; j++)
      for (int i = -1; i <= S->Lm + 2; i++) {
        A2(S->sustr, i, j) = 1.0e-4 * sin(pi * A2(S->yr, i, j) / S->c.sizey);
        A2(S->svstr, i, j) = 0.0;
        if (S->c.surf_flux) {  /* synthetic ana_stflux/ana_srflux: cooling, short-wave, evaporation */
          const double x = A2(S->xr, i, j), y = A2(S->yr, i, j);
          A2(S->stflx, i, j) = -1.0e-4 * (1.0 + 0.5 * cos(2.0 * pi * x / S->c.sizex));
          A2(S->srflx, i, j) = 4.0e-5 * (1.0 + 0.5 * sin(pi * y / S->c.sizey));
          if (S->c.salinity) S->stflx[O2(i, j) + S->n2] = 1.0e-7 * cos(pi * y / S->c.sizey);
        }
      }
  }
}

/* set_nudgcof_tile (set_nudgcof.F:17-111): sponge bands along the open
 * edges add v_sponge*wrk to visc2_r, visc2_p and diff2 on the tile's
 * own points (no exchange follows in the reference, main.F:299) */
void or_set_nudgcof(or_state *S) {
  const int isp = 15 + 1;
  double *wrk = S->s2[0];
  for (int j = (S->jstrR - 1 > -1 ? S->jstrR - 1 : -1); j <= S->jendR; j++)
    for (int i = (S->istrR - 1 > -1 ? S->istrR - 1 : -1); i <= S->iendR; i++) {
      int ibnd = isp;
      if (S->c.obc & 1) ibnd = ibnd < i ? ibnd : i;
      if (S->c.obc & 2) ibnd = ibnd < S->c.LLm + 1 - i ? ibnd : S->c.LLm + 1 - i;
      if (S->c.obc & 4) ibnd = ibnd < j ? ibnd : j;
      if (S->c.obc & 8) ibnd = ibnd < S->c.MMm + 1 - j ? ibnd : S->c.MMm + 1 - j;
      A2(wrk, i, j) = (double)(isp - ibnd) / (double)isp;
    }
  const double vs = S->c.v_sponge;
  for (int j = S->jstrR; j <= S->jendR; j++)
    for (int i = S->istrR; i <= S->iendR; i++) A2(S->visc2_r, i, j) = A2(S->visc2_r, i, j) + vs * A2(wrk, i, j);
  for (int j = S->jstr; j <= S->jendR; j++)
    for (int i = S->istr; i <= S->iendR; i++)
      A2(S->visc2_p, i, j) = A2(S->visc2_p, i, j) +
                             0.25 * vs * (A2(wrk, i, j) + A2(wrk, i - 1, j) + A2(wrk, i, j - 1) + A2(wrk, i - 1, j - 1));
  for (int it = 1; it <= S->NT; it++)
    for (int j = S->jstrR; j <= S->jendR; j++)
      for (int i = S->istrR; i <= S->iendR; i++) {
        double *d2 = S->diff2 + (size_t)(it - 1) * S->n2;
        A2(d2, i, j) = A2(d2, i, j) + vs * A2(wrk, i, j);
      }
  memset(wrk, 0, S->n2 * sizeof(double));
}

/* Analytic open-boundary data (stands in for set_bry_all / boundary.F:227,
 * which read netCDF): smooth along-edge profiles, time independent.
 * zeta/ubar/vbar/u/v from closed-form expressions, tracers = initial edge
 * state + 0.05.  sj = (j-0.5)/MMm, si = (i-0.5)/LLm (global indices). */
void or_ana_bry(or_state *S) {
  const double pi = 3.14159265358979323;
  const int N = S->N;
  for (int q = 0; q < 4; q++)
    for (int m = 0; m < S->nbry[q]; m++) {
      const double s = q < 2 ? ((double)m - 0.5) / (double)S->c.MMm : ((double)m - 0.5) / (double)S->c.LLm;
      const double sgn = (q == 0 || q == 2) ? 1.0 : -1.0;
      S->bry_zeta[q][m] = sgn * (q < 2 ? 0.05 : 0.03) * sin(pi * s);
      S->bry_ubar[q][m] = q < 2 ? 0.02 * sin(pi * s) : 0.01;
      S->bry_vbar[q][m] = q < 2 ? -0.01 : 0.015 * sin(pi * s);
      for (int k = 1; k <= N; k++) {
        const double fk = 1.0 + 0.2 * ((double)k - 0.5) / (double)N;
        S->bry_u[q][m + (size_t)S->nbry[q] * (k - 1)] = S->bry_ubar[q][m] * fk;
        S->bry_v[q][m + (size_t)S->nbry[q] * (k - 1)] = S->bry_vbar[q][m] * fk;
        for (int it = 1; it <= S->NT; it++) {
          const int i = q == 0 ? 0 : q == 1 ? S->Lm + 1 : m, j = q == 2 ? 0 : q == 3 ? S->Mm + 1 : m;
          S->bry_t[q][m + (size_t)S->nbry[q] * ((k - 1) + (size_t)N * (it - 1))] = TT(i, j, k, 1, it) + 0.05;
        }
      }
    }
}

/* ---------------------------------------------------------------------- */
/* roms_init (main.F:85-321)                                               */
/* ---------------------------------------------------------------------- */
int or_init(or_state *S) {
  S->iic = 0; S->kstp = 1; S->knew = 1; S->iif = 1; S->nstp = 1; S->nnew = 1; S->nrhs = 1;
  S->ntstart = 1; S->forw_start = 0;
  set_weights(S);
  set_scoord(S);
  or_ana_grid(S);
  setup_grid1(S);
  setup_grid2(S);
  /* mixing.F:156-162: visc2_r=visc2_p=visc2; diff2=tnu2 */
  for (size_t q = 0; q < S->n2; q++) { S->visc2_r[q] = S->c.visc2; S->visc2_p[q] = S->c.visc2; }
  for (size_t q = 0; q < S->n2 * S->NT; q++) S->diff2[q] = S->c.tnu2;
  or_set_depth(S);
  if (S->c.lmd) or_swr_frac(S);  /* main.F:217-220 */
  or_ana_forces(S);
  or_ana_init(S);
  /* ana_vmix: only active when iic==forw_start, i.e. never at init (main.F:257);
     with LMD_MIXING mixing.F:163-181 leaves Akv = Akt = 0 */
  if (S->c.case_id != OR_CASE_FILAMENT && !S->c.lmd) {
    for (size_t q = 0; q < S->n3w; q++) S->Akv[q] = S->c.Akv_bak;
    for (int it = 1; it <= S->nTS; it++)
      for (size_t q = 0; q < S->n3w; q++) S->Akt[q + (size_t)(it - 1) * S->n3w] = S->c.Akt_bak[it - 1];
  }
  or_ana_forces(S);
  if (S->c.obc) { or_set_nudgcof(S); or_ana_bry(S); }
  or_set_depth(S);
  or_set_HUV(S);
  or_omega(S);
  or_rho_eos(S, S->nrhs);
  or_diag(S);
  return 0;
}

/* set_frc_data (roms_read_write.F:303-392): up to three records of one
 * field stand for the forcing file; the pair (it1, it2) starts at the two
 * earliest and moves to (it2, next) whenever times(it2) < modtime (:341-350),
 * then cff1*rec(it1) + cff2*rec(it2) at modtime [days] (:376-379) */
int or_frc_record(or_state *S, const char *name, int slot, double time, const double *data) {
  size_t n = 0;
  double *dst = or_field(S, name, &n);
  if (!dst || slot < 0 || slot > 2) return -1;
  int q = 0;
  while (q < S->nfrc && S->frc[q].dst != dst) q++;
  if (q == S->nfrc) {
    if (S->nfrc == 64) return -1;
    S->nfrc++;
    S->frc[q].dst = dst;
    S->frc[q].n = n;
    S->frc[q].bry = strstr(name, "_west") || strstr(name, "_east") || strstr(name, "_south") || strstr(name, "_north");
    S->frc[q].rec[0] = S->frc[q].rec[1] = S->frc[q].rec[2] = NULL;
  }
  S->frc[q].k = 0;
  if (!S->frc[q].rec[slot]) S->frc[q].rec[slot] = zalloc(n);
  memcpy(S->frc[q].rec[slot], data, n * sizeof(double));
  S->frc[q].t[slot] = time;
  return 0;
}
/* set_pipe_frc (pipe_frc.F:33-80): npip pipes; pipe_idx/pipe_flx on the grid,
 * pipe_prf(npip,N), pipe_trc(npip,NT) column-major; npip = 0 switches off */
int or_set_pipes(or_state *S, int npip, const double *idx, const double *flx, const double *prf, const double *trc) {
  if (npip < 0) return -1;
  S->pipe_source = npip > 0;
  if (npip == 0) return 0;
  free(S->pipe_prf); free(S->pipe_trc);
  S->npip = npip;
  S->pipe_prf = zalloc((size_t)npip * S->N);
  S->pipe_trc = zalloc((size_t)npip * S->NT);
  memcpy(S->pipe_prf, prf, (size_t)npip * S->N * sizeof(double));
  memcpy(S->pipe_trc, trc, (size_t)npip * S->NT * sizeof(double));
  memcpy(S->pipe_idx, idx, S->n2 * sizeof(double));
  memcpy(S->pipe_flx, flx, S->n2 * sizeof(double));
  return 0;
}
void or_frc_clock(or_state *S, double start_time, int on) {
  S->frc_clock = on;
  S->frc_start = start_time;
}
static void frc_interp(or_state *S, int bry, double modtime) {
  for (int q = 0; q < S->nfrc; q++) {
    if (S->frc[q].bry != bry) continue;
    int ord[3], n = 0;   /* the loaded records in time order: the "file" */
    for (int s = 0; s < 3; s++)
      if (S->frc[q].rec[s]) {
        int k = n++;
        while (k > 0 && S->frc[q].t[ord[k - 1]] > S->frc[q].t[s]) { ord[k] = ord[k - 1]; k--; }
        ord[k] = s;
      }
    if (n < 2) continue;
    /* refresh: it1 <- it2, it2 <- the next record, while times(it2) < modtime */
    while (S->frc[q].k + 2 < n && S->frc[q].t[ord[S->frc[q].k + 1]] < modtime) S->frc[q].k++;
    const int it1 = ord[S->frc[q].k], it2 = ord[S->frc[q].k + 1];
    const double t1 = S->frc[q].t[it1], t2 = S->frc[q].t[it2];
    const double cff1 = (t2 - modtime) / (t2 - t1), cff2 = (modtime - t1) / (t2 - t1);
    for (size_t m = 0; m < S->frc[q].n; m++)
      S->frc[q].dst[m] = cff1 * S->frc[q].rec[it1][m] + cff2 * S->frc[q].rec[it2][m];
  }
}

/* ---------------------------------------------------------------------- */
/* roms_step (main.F:333-520)                                              */
/* ---------------------------------------------------------------------- */
int or_step(or_state *S) {
  S->iic = S->iic + 1;
  S->nstp = 1 + (S->iic - S->ntstart) % 2;
  S->nrhs = S->nstp;
  S->nnew = 3;
  /* model clock and the set_frc_data times of main.F:373-441 */
  const double sec2day = 1. / 86400., dt = S->dt;
  const double time = S->frc_start + dt * (double)(S->iic - S->ntstart);
  const double tdays = time * sec2day;
  if (S->frc_clock) frc_interp(S, 0, tdays);                        /* set_forces, 'current' */
  or_ana_forces(S);
  if (S->frc_clock) frc_interp(S, 1, tdays + 0.5 * dt * sec2day);   /* set_bry_all, '1/2 fwd' */
  or_rho_eos(S, S->nrhs);
  or_set_HUV(S);
  or_omega(S);
  if (S->c.lmd) or_lmd_vmix(S, S->nstp);
  or_prsgrd(S);
  or_pre_step3d(S);
  or_set_HUV1(S);
  S->nrhs = 3;
  S->nnew = 3 - S->nstp;
  or_omega(S);
  or_rho_eos(S, S->nrhs);
  if (S->frc_clock) frc_interp(S, 0, tdays + 0.5 * dt * sec2day);   /* set_forces, '1/2 fwd' */
  if (S->c.bulk_frc) or_bulk_flux(S);   /* set_forces (main.F:433) */
  if (S->c.lmd) or_lmd_vmix(S, S->nrhs);
  if (S->frc_clock) frc_interp(S, 1, (time + 0.5 * dt) * sec2day + dt * sec2day);   /* 'forward' */
  or_prsgrd(S);
  or_step3d_uv1(S);
  or_visc3d(S);
  for (S->iif = 1; S->iif <= S->nfast; S->iif++) {
    S->kstp = S->knew;
    S->knew = S->kstp + 1;
    if (S->knew > 4) S->knew = 1;
    or_step2d(S);
  }
  S->iif = S->nfast;
  or_step3d_uv2(S);
  or_omega(S);
  or_step3d_t(S);
  or_t3dmix(S);
  or_rho_eos(S, S->nnew);
  or_diag(S);
  return 0;
}

void or_lmd_vmix(or_state *S, int tind) { or_lmd_vmix_impl(S, tind); }

void or_norms(const or_state *S, double out[4]) { for (int q = 0; q < 4; q++) out[q] = S->norms[q]; }
int or_iic(const or_state *S) { return S->iic; }
int or_nfast(const or_state *S) { return S->nfast; }
const double *or_weights(const or_state *S) { return &S->weight[0][0]; }
void or_tindex(const or_state *S, int out[6]) {
  out[0] = S->iic; out[1] = S->kstp; out[2] = S->knew; out[3] = S->nstp; out[4] = S->nrhs; out[5] = S->nnew;
}
void or_set_tindex(or_state *S, const int in[6]) {
  S->iic = in[0]; S->kstp = in[1]; S->knew = in[2]; S->nstp = in[3]; S->nrhs = in[4]; S->nnew = in[5];
}
void or_set_iif(or_state *S, int iif) { S->iif = iif; }

double *or_field(or_state *S, const char *name, size_t *count) {
  struct { const char *n; double *p; size_t c; } tab[] = {
      {"riv_uflx", S->riv_uflx, S->n2}, {"riv_vflx", S->riv_vflx, S->n2},
      {"pipe_idx", S->pipe_idx, S->n2}, {"pipe_flx", S->pipe_flx, S->n2},
      {"uwnd", S->uwnd, S->n2}, {"vwnd", S->vwnd, S->n2}, {"tair", S->tair, S->n2}, {"qair", S->qair, S->n2},
      {"prate", S->prate, S->n2}, {"swrad", S->swrad, S->n2}, {"lwrad", S->lwrad, S->n2},
      {"sustr_r", S->sustr_r, S->n2}, {"svstr_r", S->svstr_r, S->n2},
      {"zeta", S->zeta, 4 * S->n2}, {"ubar", S->ubar, 4 * S->n2}, {"vbar", S->vbar, 4 * S->n2},
      {"u", S->u, 3 * S->n3}, {"v", S->v, 3 * S->n3}, {"t", S->t, 3 * S->n3 * S->NT},
      {"FlxU", S->FlxU, S->n3}, {"FlxV", S->FlxV, S->n3}, {"We", S->We, S->n3w}, {"Wi", S->Wi, S->n3w},
      {"Hz", S->Hz, S->n3}, {"z_r", S->z_r, S->n3}, {"z_w", S->z_w, S->n3w}, {"Hz_u", S->Hz_u, S->n3},
      {"Hz_v", S->Hz_v, S->n3}, {"rho", S->rho, S->n3}, {"rho1", S->rho1, S->n3}, {"qp1", S->qp1, S->n3},
      {"bvf", S->bvf, S->n3w}, {"rhoA", S->rhoA, S->n2}, {"rhoS", S->rhoS, S->n2}, {"rufrc", S->rufrc, S->n2},
      {"rvfrc", S->rvfrc, S->n2}, {"r_D", S->r_D, S->n2}, {"Zt_avg1", S->Zt_avg1, S->n2},
      {"DU_avg1", S->DU_avg1, S->n2}, {"DV_avg1", S->DV_avg1, S->n2}, {"DU_avg2", S->DU_avg2, S->n2},
      {"DV_avg2", S->DV_avg2, S->n2}, {"DU_avg_bak", S->DU_avg_bak, S->n2}, {"DV_avg_bak", S->DV_avg_bak, S->n2},
      {"ru", S->ru, S->n3}, {"rv", S->rv, S->n3}, {"Akv", S->Akv, S->n3w}, {"Akt", S->Akt, S->n3w * S->nTS},
      {"h", S->h, S->n2}, {"hinv", S->hinv, S->n2}, {"f", S->f, S->n2}, {"fomn", S->fomn, S->n2},
      {"pm", S->pm, S->n2}, {"pn", S->pn, S->n2}, {"dm_r", S->dm_r, S->n2}, {"dn_r", S->dn_r, S->n2},
      {"dm_u", S->dm_u, S->n2}, {"dn_u", S->dn_u, S->n2}, {"dm_v", S->dm_v, S->n2}, {"dn_v", S->dn_v, S->n2},
      {"dm_p", S->dm_p, S->n2}, {"dn_p", S->dn_p, S->n2}, {"pmon_u", S->pmon_u, S->n2},
      {"pnom_v", S->pnom_v, S->n2}, {"rmask", S->rmask, S->n2}, {"umask", S->umask, S->n2},
      {"vmask", S->vmask, S->n2}, {"pmask", S->pmask, S->n2}, {"dndx", S->dndx, S->n2}, {"dmde", S->dmde, S->n2}, {"ptide", S->ptide, S->n2}, {"xr", S->xr, S->n2}, {"yr", S->yr, S->n2},
      {"visc2_r", S->visc2_r, S->n2}, {"visc2_p", S->visc2_p, S->n2}, {"diff2", S->diff2, S->n2 * S->NT},
      {"sustr", S->sustr, S->n2}, {"svstr", S->svstr, S->n2}, {"stflx", S->stflx, S->n2 * S->NT},
      {"srflx", S->srflx, S->n2}, {"swflx", S->swflx, S->n2}, {"hbls", S->hbls, S->n2}, {"hbbl", S->hbbl, S->n2},
      {"ghat", S->ghat, S->n3w}, {"swr_frac", S->swr_frac, S->n3w}, {"Cs_w", S->Cs_w, (size_t)S->N + 1},
      {"Cs_r", S->Cs_r, (size_t)S->N + 1},
      {"dRdx", S->dRdx, S->dRdx ? S->n3 : 0}, {"dRde", S->dRde, S->dRde ? S->n3 : 0},
      {"idRz", S->idRz, S->idRz ? S->n3w : 0}, {"diff3u", S->diff3u, S->diff3u ? S->n3 : 0},
      {"diff3v", S->diff3v, S->diff3v ? S->n3 : 0}, {"Akz", S->Akz, S->Akz ? S->n3w : 0},
  };
  for (size_t q = 0; q < sizeof(tab) / sizeof(tab[0]); q++)
    if (strcmp(tab[q].n, name) == 0) { if (count) *count = tab[q].c; return tab[q].p; }
  static const char *side[4] = {"west", "east", "south", "north"};
  for (int q = 0; q < 4; q++) {
    char nm[32];
    const size_t nb = (size_t)S->nbry[q];
    struct { const char *k; double *p; size_t c; } bt[] = {
        {"zeta", S->bry_zeta[q], nb}, {"ubar", S->bry_ubar[q], nb}, {"vbar", S->bry_vbar[q], nb},
        {"u", S->bry_u[q], nb * S->N}, {"v", S->bry_v[q], nb * S->N}, {"t", S->bry_t[q], nb * S->N * S->NT}};
    for (size_t r = 0; r < 6; r++) {
      snprintf(nm, sizeof nm, "%s_%s", bt[r].k, side[q]);
      if (strcmp(nm, name) == 0) { if (count) *count = bt[r].c; return bt[r].p; }
    }
  }
  if (count) *count = 0;
  return NULL;
}

/* SPONGE_TUNE (sponge_tune.F, t3dbc_im.F:73-74): the per-edge binding
 * coefficients ub_west(j), ub_east(j), ub_south(i), ub_north(i) that
 * adjust_orlanski maintains; NULL switches an edge's floor off. */
void or_set_ub(or_state *S, const double *w, const double *e, const double *s, const double *n) {
  const double *src[4] = {w, e, s, n};
  for (int q = 0; q < 4; q++) {
    free(S->ub[q]);
    S->ub[q] = NULL;
    if (!src[q]) continue;
    S->ub[q] = zalloc(S->nbry[q]);
    for (int m = 0; m < S->nbry[q]; m++) S->ub[q][m] = src[q][m];
  }
}

void or_set_river(or_state *S, int nriv, const double *vol, const double *trc) {
  if (nriv < 1 || nriv > 16 || nriv * S->NT > 256) return;
  S->nriv = nriv;
  for (int r = 0; r < nriv; r++) S->riv_vol[r] = vol[r];
  for (int q = 0; q < nriv * S->NT; q++) S->riv_trc[q] = trc[q];
}
