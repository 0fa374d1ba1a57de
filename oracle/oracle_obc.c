/*
 * oracle_obc.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 *
 * Lateral boundary conditions of the split-explicit step, per physical edge:
 *   closed wall (no OBC_<edge>): zero normal flow, free/no-slip tangential
 *   (gamma2), zero-gradient free surface and tracers;
 *   open edge (OBC_<edge>, the Iceland switch set of
 *   Examples/Iceland/Iceland_parent/cppdefs.opt): OBC_M2FLATHER for zeta /
 *   ubar / vbar, OBC_M3ORLANSKI for u / v, OBC_TORLANSKI for tracers, with
 *   Z_FRC_BRY / M2_FRC_BRY / M3_FRC_BRY / T_FRC_BRY boundary data
 *   (zeta_west(j), ubar_west(j), u_west(j,k), t_west(j,k,itrc), ...;
 *   boundary.F:21-39).
 * Each routine keeps the reference's edge order and arithmetic order:
 *   zetabc.F:3-224, u2dbc_im.F:3-481, v2dbc_im.F:3-472, u3dbc_im.F:4-424,
 *   v3dbc_im.F:4-433, t3dbc_im.F:4-422.
 * Quirks kept: with OBC_M2FLATHER the tangential barotropic components use
 * the OBC_M2ORLANSKI branch (u2dbc_im.F:270-273, v2dbc_im.F:273-276); the
 * eastern and northern tracer radiation reads the interior t(nnew)
 * (t3dbc_im.F:133,276) where the western and southern read t(nstp).
 */
#include "oracle_core.h"

#define OBC_W (S->west_edge && (S->c.obc & 1))
#define OBC_E (S->east_edge && (S->c.obc & 2))
#define OBC_S (S->south_edge && (S->c.obc & 4))
#define OBC_N (S->north_edge && (S->c.obc & 8))
/* boundary arrays: west/east indexed by j (0:Mm+1), south/north by i (0:Lm+1) */
#define B1(a, s, m) (S->a[s][(m)])
#define B2(a, s, m, k) (S->a[s][(size_t)(m) + (size_t)S->nbry[s] * (size_t)((k)-1)])
#define BT(s, m, k, it) \
  (S->bry_t[s][(size_t)(m) + (size_t)S->nbry[s] * ((size_t)((k)-1) + (size_t)S->N * (size_t)((it)-1))])
enum { SW = 0, SE = 1, SS = 2, SN = 3 };

static const double kEps = 1.E-33;
static const double kFl = 0.292893218813452;  /* u2dbc_im.F:36 */

/* PRED_STAGE (nnew==3, set_global_definitions.h:356): half step forward */
static double dtfwd(const or_state *S) { return S->nnew == 3 ? 0.5 * S->dt : S->dt; }

/* grad scratch over one edge strip: two rows/columns, indexed by the
 * along-edge coordinate m in (-1 .. max(Lm,Mm)+2) */
typedef struct { double a[2][4200]; } strip2;
#define G(r, m) (gs.a[r][(m) + 2])

/* ---------------------------------------------------------------------- */
void or_zetabc(or_state *S, double *zn) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend, ks = S->kstp;
  const double dtf = S->dtfast, g = S->g;
  if (S->west_edge) {
    if (OBC_W)
      for (int j = S->jstrV - 1; j <= jend; j++) {
        const double cx = dtf * A2(S->pm, istr, j) * sqrt(g * A2(S->h, istr, j));
        A2(zn, istr - 1, j) = ((1. - cx) * ZETA(istr - 1, j, ks) + cx * ZETA(istr, j, ks)) * A2(S->rmask, istr - 1, j);
      }
    else
      for (int j = S->jstrV - 1; j <= jend; j++) A2(zn, istr - 1, j) = A2(zn, istr, j) * A2(S->rmask, istr - 1, j);
  }
  if (S->east_edge) {
    if (OBC_E)
      for (int j = S->jstrV - 1; j <= jend; j++) {
        const double cx = dtf * A2(S->pm, iend, j) * sqrt(g * A2(S->h, iend, j));
        A2(zn, iend + 1, j) = ((1. - cx) * ZETA(iend + 1, j, ks) + cx * ZETA(iend, j, ks)) * A2(S->rmask, iend + 1, j);
      }
    else
      for (int j = S->jstrV - 1; j <= jend; j++) A2(zn, iend + 1, j) = A2(zn, iend, j) * A2(S->rmask, iend + 1, j);
  }
  if (S->south_edge) {
    if (OBC_S)
      for (int i = S->istrU - 1; i <= iend; i++) {
        const double cx = dtf * A2(S->pn, i, jstr) * sqrt(g * A2(S->h, i, jstr));
        A2(zn, i, jstr - 1) = ((1. - cx) * ZETA(i, jstr - 1, ks) + cx * ZETA(i, jstr, ks)) * A2(S->rmask, i, jstr - 1);
      }
    else
      for (int i = S->istrU - 1; i <= iend; i++) A2(zn, i, jstr - 1) = A2(zn, i, jstr) * A2(S->rmask, i, jstr - 1);
  }
  if (S->north_edge) {
    if (OBC_N)
      for (int i = S->istrU - 1; i <= iend; i++) {
        const double cx = dtf * A2(S->pn, i, jend) * sqrt(g * A2(S->h, i, jend));
        A2(zn, i, jend + 1) = ((1. - cx) * ZETA(i, jend + 1, ks) + cx * ZETA(i, jend, ks)) * A2(S->rmask, i, jend + 1);
      }
    else
      for (int i = S->istrU - 1; i <= iend; i++) A2(zn, i, jend + 1) = A2(zn, i, jend) * A2(S->rmask, i, jend + 1);
  }
  if (S->south_edge && S->west_edge) A2(zn, istr - 1, jstr - 1) = 0.5 * (A2(zn, istr, jstr - 1) + A2(zn, istr - 1, jstr));
  if (S->south_edge && S->east_edge) A2(zn, iend + 1, jstr - 1) = 0.5 * (A2(zn, iend, jstr - 1) + A2(zn, iend + 1, jstr));
  if (S->north_edge && S->west_edge) A2(zn, istr - 1, jend + 1) = 0.5 * (A2(zn, istr, jend + 1) + A2(zn, istr - 1, jend));
  if (S->north_edge && S->east_edge) A2(zn, iend + 1, jend + 1) = 0.5 * (A2(zn, iend, jend + 1) + A2(zn, iend + 1, jend));
}

/* Flather zx (u2dbc_im.F:31-40): zb = zeta(boundary,kstp), zi = zeta(interior,kstp), zin = zeta(interior,knew) */
static double flather_zx(double cx, double zi, double zb, double zin) {
  double zx = (0.5 + cx) * zi + (0.5 - cx) * zb;
  if (cx > kFl) {
    const double q = 1. - kFl / cx;
    zx = zx + (zin + cx * zb - (1. + cx) * zi) * (q * q);
  }
  return zx;
}

/* ---------------------------------------------------------------------- */
void or_u2dbc(or_state *S) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend, kn = S->knew, ks = S->kstp;
  const double dtf = S->dtfast, g = S->g;
  static strip2 gs;
  if (S->west_edge) {
    if (OBC_W)
      for (int j = jstr; j <= jend; j++) {
        const double cff = 0.5 * (A2(S->h, istr - 1, j) + A2(S->h, istr, j));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (A2(S->pm, istr - 1, j) + A2(S->pm, istr, j));
        const double zx = flather_zx(cx, ZETA(istr, j, ks), ZETA(istr - 1, j, ks), ZETA(istr, j, kn));
        UBAR(istr, j, kn) = 0.5 * ((1. - cx) * UBAR(istr, j, ks) + cx * UBAR(istr + 1, j, ks) + B1(bry_ubar, SW, j) -
                                   hx * (zx - B1(bry_zeta, SW, j))) *
                            A2(S->umask, istr, j);
      }
    else
      for (int j = jstr; j <= jend; j++) UBAR(istr, j, kn) = 0.0;
  }
  if (S->east_edge) {
    if (OBC_E)
      for (int j = jstr; j <= jend; j++) {
        const double cff = 0.5 * (A2(S->h, iend, j) + A2(S->h, iend + 1, j));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (A2(S->pm, iend, j) + A2(S->pm, iend + 1, j));
        const double zx = flather_zx(cx, ZETA(iend, j, ks), ZETA(iend + 1, j, ks), ZETA(iend, j, kn));
        UBAR(iend + 1, j, kn) = 0.5 * ((1. - cx) * UBAR(iend + 1, j, ks) + cx * UBAR(iend, j, ks) +
                                       B1(bry_ubar, SE, j) + hx * (zx - B1(bry_zeta, SE, j))) *
                                A2(S->umask, iend + 1, j);
      }
    else
      for (int j = jstr; j <= jend; j++) UBAR(iend + 1, j, kn) = 0.0;
  }
  if (S->south_edge) {
    if (OBC_S) {  /* tangential: the OBC_M2ORLANSKI branch (u2dbc_im.F:270-330) */
      for (int i = S->istrU - 1; i <= iend; i++) {
        G(0, i) = UBAR(i + 1, jstr - 1, ks) - UBAR(i, jstr - 1, ks);
        G(1, i) = UBAR(i + 1, jstr, ks) - UBAR(i, jstr, ks);
      }
      for (int i = S->istrU; i <= iend; i++) {
        double cx = -0.125 * dtf * (VBAR(i, jstr, ks) + VBAR(i - 1, jstr, ks)) *
                    (A2(S->pn, i, jstr - 1) + A2(S->pn, i - 1, jstr - 1) + A2(S->pn, i, jstr) + A2(S->pn, i - 1, jstr));
        const double cy = 0.125 * dtf * (UBAR(i, jstr - 1, ks) + UBAR(i, jstr, ks)) *
                          (A2(S->pm, i, jstr - 1) + A2(S->pm, i - 1, jstr - 1) + A2(S->pm, i, jstr) + A2(S->pm, i - 1, jstr));
        double cext;
        if (cx > 0.) cext = 0.;
        else { cext = -cx; cx = 0.; }
        UBAR(i, jstr - 1, kn) = (1. - cx) * (UBAR(i, jstr - 1, ks) - fmax0(cy) * G(0, i - 1) - fmin0(cy) * G(0, i)) +
                                cx * (UBAR(i, jstr, ks) - fmax0(cy) * G(1, i - 1) - fmin0(cy) * G(1, i));
        UBAR(i, jstr - 1, kn) = (1. - cext) * UBAR(i, jstr - 1, kn) + cext * B1(bry_ubar, SS, i);
        UBAR(i, jstr - 1, kn) = UBAR(i, jstr - 1, kn) * A2(S->umask, i, jstr - 1);
      }
    } else {
      const int i0 = S->c.ew_periodic ? S->istrU : istr, i1 = S->c.ew_periodic ? iend : S->iendR;
      for (int i = i0; i <= i1; i++) UBAR(i, jstr - 1, kn) = S->gamma2 * UBAR(i, jstr, kn) * A2(S->umask, i, jstr - 1);
    }
  }
  if (S->north_edge) {
    if (OBC_N) {
      for (int i = S->istrU - 1; i <= iend; i++) {
        G(0, i) = UBAR(i + 1, jend, ks) - UBAR(i, jend, ks);
        G(1, i) = UBAR(i + 1, jend + 1, ks) - UBAR(i, jend + 1, ks);
      }
      for (int i = S->istrU; i <= iend; i++) {
        double cx = 0.125 * dtf * (VBAR(i, jend + 1, ks) + VBAR(i - 1, jend + 1, ks)) *
                    (A2(S->pn, i, jend) + A2(S->pn, i - 1, jend) + A2(S->pn, i, jend + 1) + A2(S->pn, i - 1, jend + 1));
        const double cy = 0.125 * dtf * (UBAR(i, jend, ks) + UBAR(i, jend + 1, ks)) *
                          (A2(S->pm, i, jend) + A2(S->pm, i - 1, jend) + A2(S->pm, i, jend + 1) + A2(S->pm, i - 1, jend + 1));
        double cext;
        if (cx > 0.) cext = 0.;
        else { cext = -cx; cx = 0.; }
        UBAR(i, jend + 1, kn) = (1. - cx) * (UBAR(i, jend + 1, ks) - fmax0(cy) * G(1, i - 1) - fmin0(cy) * G(1, i)) +
                                cx * (UBAR(i, jend, ks) - fmax0(cy) * G(0, i - 1) - fmin0(cy) * G(0, i));
        UBAR(i, jend + 1, kn) = (1. - cext) * UBAR(i, jend + 1, kn) + cext * B1(bry_ubar, SN, i);
        UBAR(i, jend + 1, kn) = UBAR(i, jend + 1, kn) * A2(S->umask, i, jend + 1);
      }
    } else {
      const int i0 = S->c.ew_periodic ? S->istrU : istr, i1 = S->c.ew_periodic ? iend : S->iendR;
      for (int i = i0; i <= i1; i++) UBAR(i, jend + 1, kn) = S->gamma2 * UBAR(i, jend, kn) * A2(S->umask, i, jend + 1);
    }
  }
  if (OBC_S && OBC_W) UBAR(istr, jstr - 1, kn) = 0.5 * (UBAR(istr + 1, jstr - 1, kn) + UBAR(istr, jstr, kn));
  if (OBC_S && OBC_E) UBAR(iend + 1, jstr - 1, kn) = 0.5 * (UBAR(iend, jstr - 1, kn) + UBAR(iend + 1, jstr, kn));
  if (OBC_N && OBC_W) UBAR(istr, jend + 1, kn) = 0.5 * (UBAR(istr + 1, jend + 1, kn) + UBAR(istr, jend, kn));
  if (OBC_N && OBC_E) UBAR(iend + 1, jend + 1, kn) = 0.5 * (UBAR(iend, jend + 1, kn) + UBAR(iend + 1, jend, kn));
}

/* ---------------------------------------------------------------------- */
void or_v2dbc(or_state *S) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend, kn = S->knew, ks = S->kstp;
  const double dtf = S->dtfast, g = S->g;
  static strip2 gs;
  if (S->south_edge) {
    if (OBC_S)
      for (int i = istr; i <= iend; i++) {
        const double cff = 0.5 * (A2(S->h, i, jstr - 1) + A2(S->h, i, jstr));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (A2(S->pn, i, jstr - 1) + A2(S->pn, i, jstr));
        const double zx = flather_zx(cx, ZETA(i, jstr, ks), ZETA(i, jstr - 1, ks), ZETA(i, jstr, kn));
        VBAR(i, jstr, kn) = 0.5 * ((1. - cx) * VBAR(i, jstr, ks) + cx * VBAR(i, jstr + 1, ks) + B1(bry_vbar, SS, i) -
                                   hx * (zx - B1(bry_zeta, SS, i))) *
                            A2(S->vmask, i, jstr);
      }
    else
      for (int i = istr; i <= iend; i++) VBAR(i, jstr, kn) = 0.0;
  }
  if (S->north_edge) {
    if (OBC_N)
      for (int i = istr; i <= iend; i++) {
        const double cff = 0.5 * (A2(S->h, i, jend) + A2(S->h, i, jend + 1));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (A2(S->pn, i, jend) + A2(S->pn, i, jend + 1));
        const double zx = flather_zx(cx, ZETA(i, jend, ks), ZETA(i, jend + 1, ks), ZETA(i, jend, kn));
        VBAR(i, jend + 1, kn) = 0.5 * ((1. - cx) * VBAR(i, jend + 1, ks) + cx * VBAR(i, jend, ks) +
                                       B1(bry_vbar, SN, i) + hx * (zx - B1(bry_zeta, SN, i))) *
                                A2(S->vmask, i, jend + 1);
      }
    else
      for (int i = istr; i <= iend; i++) VBAR(i, jend + 1, kn) = 0.0;
  }
  if (S->west_edge) {
    if (OBC_W) {
      for (int j = S->jstrV - 1; j <= jend; j++) {
        G(0, j) = VBAR(istr - 1, j + 1, ks) - VBAR(istr - 1, j, ks);
        G(1, j) = VBAR(istr, j + 1, ks) - VBAR(istr, j, ks);
      }
      for (int j = S->jstrV; j <= jend; j++) {
        double cx = -0.125 * dtf * (UBAR(istr, j, ks) + UBAR(istr, j - 1, ks)) *
                    (A2(S->pm, istr - 1, j) + A2(S->pm, istr - 1, j - 1) + A2(S->pm, istr, j) + A2(S->pm, istr, j - 1));
        const double cy = 0.125 * dtf * (VBAR(istr - 1, j, ks) + VBAR(istr, j, ks)) *
                          (A2(S->pn, istr - 1, j) + A2(S->pn, istr - 1, j - 1) + A2(S->pn, istr, j) + A2(S->pn, istr, j - 1));
        double cext;
        if (cx > 0.) cext = 0.;
        else { cext = -cx; cx = 0.; }
        VBAR(istr - 1, j, kn) = (1. - cx) * (VBAR(istr - 1, j, ks) - fmax0(cy) * G(0, j - 1) - fmin0(cy) * G(0, j)) +
                                cx * (VBAR(istr, j, ks) - fmax0(cy) * G(1, j - 1) - fmin0(cy) * G(1, j));
        VBAR(istr - 1, j, kn) = (1. - cext) * VBAR(istr - 1, j, kn) + cext * B1(bry_vbar, SW, j);
        VBAR(istr - 1, j, kn) = VBAR(istr - 1, j, kn) * A2(S->vmask, istr - 1, j);
      }
    } else {
      const int j0 = S->c.ns_periodic ? S->jstrV : jstr, j1 = S->c.ns_periodic ? jend : S->jendR;
      for (int j = j0; j <= j1; j++) VBAR(istr - 1, j, kn) = S->gamma2 * VBAR(istr, j, kn) * A2(S->vmask, istr - 1, j);
    }
  }
  if (S->east_edge) {
    if (OBC_E) {
      for (int j = S->jstrV - 1; j <= jend; j++) {
        G(0, j) = VBAR(iend, j + 1, ks) - VBAR(iend, j, ks);
        G(1, j) = VBAR(iend + 1, j + 1, ks) - VBAR(iend + 1, j, ks);
      }
      for (int j = S->jstrV; j <= jend; j++) {
        double cx = 0.125 * dtf * (UBAR(iend + 1, j, ks) + UBAR(iend + 1, j - 1, ks)) *
                    (A2(S->pm, iend, j) + A2(S->pm, iend, j - 1) + A2(S->pm, iend + 1, j) + A2(S->pm, iend + 1, j - 1));
        const double cy = 0.125 * dtf * (VBAR(iend, j, ks) + VBAR(iend + 1, j, ks)) *
                          (A2(S->pn, iend, j) + A2(S->pn, iend, j - 1) + A2(S->pn, iend + 1, j) + A2(S->pn, iend + 1, j - 1));
        double cext;
        if (cx > 0.) cext = 0.;
        else { cext = -cx; cx = 0.; }
        VBAR(iend + 1, j, kn) = (1. - cx) * (VBAR(iend + 1, j, ks) - fmax0(cy) * G(1, j - 1) - fmin0(cy) * G(1, j)) +
                                cx * (VBAR(iend, j, ks) - fmax0(cy) * G(0, j - 1) - fmin0(cy) * G(0, j));
        VBAR(iend + 1, j, kn) = (1. - cext) * VBAR(iend + 1, j, kn) + cext * B1(bry_vbar, SE, j);
        VBAR(iend + 1, j, kn) = VBAR(iend + 1, j, kn) * A2(S->vmask, iend + 1, j);
      }
    } else {
      const int j0 = S->c.ns_periodic ? S->jstrV : jstr, j1 = S->c.ns_periodic ? jend : S->jendR;
      for (int j = j0; j <= j1; j++) VBAR(iend + 1, j, kn) = S->gamma2 * VBAR(iend, j, kn) * A2(S->vmask, iend + 1, j);
    }
  }
  if (OBC_S && OBC_W) VBAR(istr - 1, jstr, kn) = 0.5 * (VBAR(istr - 1, jstr + 1, kn) + VBAR(istr, jstr, kn));
  if (OBC_S && OBC_E) VBAR(iend + 1, jstr, kn) = 0.5 * (VBAR(iend + 1, jstr + 1, kn) + VBAR(iend, jstr, kn));
  if (OBC_N && OBC_W) VBAR(istr - 1, jend + 1, kn) = 0.5 * (VBAR(istr - 1, jend, kn) + VBAR(istr, jend + 1, kn));
  if (OBC_N && OBC_E) VBAR(iend + 1, jend + 1, kn) = 0.5 * (VBAR(iend + 1, jend, kn) + VBAR(iend, jend + 1, kn));
}

/* normal-component Orlanski radiation (u3dbc_im.F:50-110): returns the
 * new boundary value before the M3_FRC_BRY blend; *cx_out < 0 flags inflow */
static double orlanski_normal(double bs, double i1s, double i1n, double i2n, double gb0, double gb1, double gi0,
                              double gi1, int *inflow) {
  const double dft = i1s - i1n, dfx = i1n - i2n;
  const double dfy = (dft * (gi0 + gi1) > 0.) ? gi0 : gi1;
  const double cff = dmax(dfx * dfx + dfy * dfy, kEps);
  double cy = dmin(cff, dmax(dft * dfy, -cff));
  double cx = dft * dfx;
  *inflow = 0;
  if (cx < 0.) { cx = 0.; cy = 0.; *inflow = 1; }
  return (cff * bs + cx * i1n - fmax0(cy) * gb0 - fmin0(cy) * gb1) / (cff + cx);
}

/* ---------------------------------------------------------------------- */
void or_u3dbc(or_state *S) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const int nn = S->nnew, ns = S->nstp, nr = S->nrhs, N = S->N;
  const double dtw = dtfwd(S);
  static strip2 gs;
  if (S->west_edge) {
    if (OBC_W)
      for (int k = 1; k <= N; k++) {
        for (int j = jstr; j <= jend + 1; j++) {
          G(0, j) = (U(istr, j, k, ns) - U(istr, j - 1, k, ns)) * A2(S->pmask, istr, j);
          G(1, j) = (U(istr + 1, j, k, ns) - U(istr + 1, j - 1, k, ns)) * A2(S->pmask, istr + 1, j);
        }
        for (int j = jstr; j <= jend; j++) {
          int inflow;
          double ub = orlanski_normal(U(istr, j, k, ns), U(istr + 1, j, k, ns), U(istr + 1, j, k, nn), U(istr + 2, j, k, nn),
                                      G(0, j), G(0, j + 1), G(1, j), G(1, j + 1), &inflow);
          double cext = 0.;
          if (inflow) {
            cext = B2(bry_u, SW, j, k) > 0. ? B2(bry_u, SW, j, k) : S->c.ubind;
            cext = cext * dtw * 0.5 * (A2(S->pm, istr - 1, j) + A2(S->pm, istr, j));
          }
          U(istr, j, k, nn) = ub;
          if (S->ub[SW]) cext = dmax(cext, dmin(S->ub[SW][j], 1.0));   /* SPONGE_TUNE (u3dbc_im.F:101-103) */
          U(istr, j, k, nn) = (1. - cext) * U(istr, j, k, nn) + cext * B2(bry_u, SW, j, k);
          U(istr, j, k, nn) = U(istr, j, k, nn) * A2(S->umask, istr, j);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int j = jstr; j <= jend; j++) U(istr, j, k, nn) = 0.0;
  }
  if (S->east_edge) {
    if (OBC_E)
      for (int k = 1; k <= N; k++) {
        for (int j = jstr; j <= jend + 1; j++) {
          G(0, j) = (U(iend, j, k, ns) - U(iend, j - 1, k, ns)) * A2(S->pmask, iend, j);
          G(1, j) = (U(iend + 1, j, k, ns) - U(iend + 1, j - 1, k, ns)) * A2(S->pmask, iend + 1, j);
        }
        for (int j = jstr; j <= jend; j++) {
          int inflow;
          double ub = orlanski_normal(U(iend + 1, j, k, ns), U(iend, j, k, ns), U(iend, j, k, nn), U(iend - 1, j, k, nn),
                                      G(1, j), G(1, j + 1), G(0, j), G(0, j + 1), &inflow);
          double cext = 0.;
          if (inflow) {
            cext = B2(bry_u, SE, j, k) < 0. ? -B2(bry_u, SE, j, k) : S->c.ubind;
            cext = cext * dtw * 0.5 * (A2(S->pm, iend, j) + A2(S->pm, iend + 1, j));
          }
          U(iend + 1, j, k, nn) = ub;
          if (S->ub[SE]) cext = dmax(cext, dmin(S->ub[SE][j], 1.0));   /* SPONGE_TUNE (u3dbc_im.F:190-192) */
          U(iend + 1, j, k, nn) = (1. - cext) * U(iend + 1, j, k, nn) + cext * B2(bry_u, SE, j, k);
          U(iend + 1, j, k, nn) = U(iend + 1, j, k, nn) * A2(S->umask, iend + 1, j);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int j = jstr; j <= jend; j++) U(iend + 1, j, k, nn) = 0.0;
  }
  if (S->south_edge) {
    if (OBC_S)
      for (int k = 1; k <= N; k++) {
        for (int i = S->istrU - 1; i <= iend; i++) {
          G(0, i) = U(i + 1, jstr - 1, k, ns) - U(i, jstr - 1, k, ns);
          G(1, i) = U(i + 1, jstr, k, ns) - U(i, jstr, k, ns);
        }
        for (int i = S->istrU; i <= iend; i++) {
          double cx = -0.125 * dtw * (V(i, jstr, k, nr) + V(i - 1, jstr, k, nr)) *
                      (A2(S->pn, i, jstr - 1) + A2(S->pn, i - 1, jstr - 1) + A2(S->pn, i, jstr) + A2(S->pn, i - 1, jstr));
          const double cy = 0.125 * dtw * (U(i, jstr - 1, k, nr) + U(i, jstr, k, nr)) *
                            (A2(S->pm, i, jstr - 1) + A2(S->pm, i - 1, jstr - 1) + A2(S->pm, i, jstr) + A2(S->pm, i - 1, jstr));
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          U(i, jstr - 1, k, nn) = (1. - cx) * (U(i, jstr - 1, k, ns) - fmax0(cy) * G(0, i - 1) - fmin0(cy) * G(0, i)) +
                                  cx * (U(i, jstr, k, ns) - fmax0(cy) * G(1, i - 1) - fmin0(cy) * G(1, i));
          if (S->ub[SS]) cext = dmax(cext, dmin(S->ub[SS][i], 1.0));   /* SPONGE_TUNE (u3dbc_im.F:262-264) */
          U(i, jstr - 1, k, nn) = (1. - cext) * U(i, jstr - 1, k, nn) + cext * B2(bry_u, SS, i, k);
          U(i, jstr - 1, k, nn) = U(i, jstr - 1, k, nn) * A2(S->umask, i, jstr - 1);
        }
      }
    else {
      const int i0 = S->c.ew_periodic ? S->istrU : istr, i1 = S->c.ew_periodic ? iend : S->iendR;
      for (int k = 1; k <= N; k++)
        for (int i = i0; i <= i1; i++) U(i, jstr - 1, k, nn) = S->gamma2 * U(i, jstr, k, nn) * A2(S->umask, i, jstr - 1);
    }
  }
  if (S->north_edge) {
    if (OBC_N)
      for (int k = 1; k <= N; k++) {
        for (int i = S->istrU - 1; i <= iend; i++) {
          G(0, i) = U(i + 1, jend, k, ns) - U(i, jend, k, ns);
          G(1, i) = U(i + 1, jend + 1, k, ns) - U(i, jend + 1, k, ns);
        }
        for (int i = S->istrU; i <= iend; i++) {
          double cx = 0.125 * dtw * (V(i, jend + 1, k, nr) + V(i - 1, jend + 1, k, nr)) *
                      (A2(S->pn, i, jend + 1) + A2(S->pn, i - 1, jend + 1) + A2(S->pn, i, jend) + A2(S->pn, i - 1, jend));
          const double cy = 0.125 * dtw * (U(i, jend, k, nr) + U(i, jend + 1, k, nr)) *
                            (A2(S->pm, i, jend + 1) + A2(S->pm, i - 1, jend + 1) + A2(S->pm, i, jend) + A2(S->pm, i - 1, jend));
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          U(i, jend + 1, k, nn) = (1. - cx) * (U(i, jend + 1, k, ns) - fmax0(cy) * G(1, i - 1) - fmin0(cy) * G(1, i)) +
                                  cx * (U(i, jend, k, ns) - fmax0(cy) * G(0, i - 1) - fmin0(cy) * G(0, i));
          if (S->ub[SN]) cext = dmax(cext, dmin(S->ub[SN][i], 1.0));   /* SPONGE_TUNE (u3dbc_im.F:341-343) */
          U(i, jend + 1, k, nn) = (1. - cext) * U(i, jend + 1, k, nn) + cext * B2(bry_u, SN, i, k);
          U(i, jend + 1, k, nn) = U(i, jend + 1, k, nn) * A2(S->umask, i, jend + 1);
        }
      }
    else {
      const int i0 = S->c.ew_periodic ? S->istrU : istr, i1 = S->c.ew_periodic ? iend : S->iendR;
      for (int k = 1; k <= N; k++)
        for (int i = i0; i <= i1; i++) U(i, jend + 1, k, nn) = S->gamma2 * U(i, jend, k, nn) * A2(S->umask, i, jend + 1);
    }
  }
  for (int k = 1; k <= N; k++) {
    if (OBC_S && OBC_W) U(istr, jstr - 1, k, nn) = 0.5 * (U(istr + 1, jstr - 1, k, nn) + U(istr, jstr, k, nn));
    if (OBC_S && OBC_E) U(iend + 1, jstr - 1, k, nn) = 0.5 * (U(iend, jstr - 1, k, nn) + U(iend + 1, jstr, k, nn));
    if (OBC_N && OBC_W) U(istr, jend + 1, k, nn) = 0.5 * (U(istr + 1, jend + 1, k, nn) + U(istr, jend, k, nn));
    if (OBC_N && OBC_E) U(iend + 1, jend + 1, k, nn) = 0.5 * (U(iend, jend + 1, k, nn) + U(iend + 1, jend, k, nn));
  }
}

/* ---------------------------------------------------------------------- */
void or_v3dbc(or_state *S) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const int nn = S->nnew, ns = S->nstp, nr = S->nrhs, N = S->N;
  const double dtw = dtfwd(S);
  static strip2 gs;
  if (S->south_edge) {
    if (OBC_S)
      for (int k = 1; k <= N; k++) {
        for (int i = istr; i <= iend + 1; i++) {
          G(0, i) = (V(i, jstr, k, ns) - V(i - 1, jstr, k, ns)) * A2(S->pmask, i, jstr);
          G(1, i) = (V(i, jstr + 1, k, ns) - V(i - 1, jstr + 1, k, ns)) * A2(S->pmask, i, jstr + 1);
        }
        for (int i = istr; i <= iend; i++) {
          int inflow;
          double vb = orlanski_normal(V(i, jstr, k, ns), V(i, jstr + 1, k, ns), V(i, jstr + 1, k, nn), V(i, jstr + 2, k, nn),
                                      G(0, i), G(0, i + 1), G(1, i), G(1, i + 1), &inflow);
          double cext = 0.;
          if (inflow) {
            cext = B2(bry_v, SS, i, k) > 0. ? B2(bry_v, SS, i, k) : S->c.ubind;
            cext = cext * dtw * 0.5 * (A2(S->pn, i, jstr - 1) + A2(S->pn, i, jstr));
          }
          V(i, jstr, k, nn) = vb;
          if (S->ub[SS]) cext = dmax(cext, dmin(S->ub[SS][i], 1.0));   /* SPONGE_TUNE (v3dbc_im.F:97-99) */
          V(i, jstr, k, nn) = (1. - cext) * V(i, jstr, k, nn) + cext * B2(bry_v, SS, i, k);
          V(i, jstr, k, nn) = V(i, jstr, k, nn) * A2(S->vmask, i, jstr);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int i = istr; i <= iend; i++) V(i, jstr, k, nn) = 0.0;
  }
  if (S->north_edge) {
    if (OBC_N)
      for (int k = 1; k <= N; k++) {
        for (int i = istr; i <= iend + 1; i++) {
          G(0, i) = (V(i, jend, k, ns) - V(i - 1, jend, k, ns)) * A2(S->pmask, i, jend);
          G(1, i) = (V(i, jend + 1, k, ns) - V(i - 1, jend + 1, k, ns)) * A2(S->pmask, i, jend + 1);
        }
        for (int i = istr; i <= iend; i++) {
          int inflow;
          double vb = orlanski_normal(V(i, jend + 1, k, ns), V(i, jend, k, ns), V(i, jend, k, nn), V(i, jend - 1, k, nn),
                                      G(1, i), G(1, i + 1), G(0, i), G(0, i + 1), &inflow);
          double cext = 0.;
          if (inflow) {
            cext = B2(bry_v, SN, i, k) < 0. ? -B2(bry_v, SN, i, k) : S->c.ubind;
            cext = cext * dtw * 0.5 * (A2(S->pn, i, jend) + A2(S->pn, i, jend + 1));
          }
          V(i, jend + 1, k, nn) = vb;
          if (S->ub[SN]) cext = dmax(cext, dmin(S->ub[SN][i], 1.0));   /* SPONGE_TUNE (v3dbc_im.F:189-191) */
          V(i, jend + 1, k, nn) = (1. - cext) * V(i, jend + 1, k, nn) + cext * B2(bry_v, SN, i, k);
          V(i, jend + 1, k, nn) = V(i, jend + 1, k, nn) * A2(S->vmask, i, jend + 1);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int i = istr; i <= iend; i++) V(i, jend + 1, k, nn) = 0.0;
  }
  if (S->west_edge) {
    if (OBC_W)
      for (int k = 1; k <= N; k++) {
        for (int j = S->jstrV - 1; j <= jend; j++) {
          G(0, j) = V(istr - 1, j + 1, k, ns) - V(istr - 1, j, k, ns);
          G(1, j) = V(istr, j + 1, k, ns) - V(istr, j, k, ns);
        }
        for (int j = S->jstrV; j <= jend; j++) {
          double cx = -0.125 * dtw * (U(istr, j, k, nr) + U(istr, j - 1, k, nr)) *
                      (A2(S->pm, istr - 1, j) + A2(S->pm, istr - 1, j - 1) + A2(S->pm, istr, j) + A2(S->pm, istr, j - 1));
          const double cy = 0.125 * dtw * (V(istr - 1, j, k, nr) + V(istr, j, k, nr)) *
                            (A2(S->pn, istr - 1, j) + A2(S->pn, istr - 1, j - 1) + A2(S->pn, istr, j) + A2(S->pn, istr, j - 1));
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          V(istr - 1, j, k, nn) = (1. - cx) * (V(istr - 1, j, k, ns) - fmax0(cy) * G(0, j - 1) - fmin0(cy) * G(0, j)) +
                                  cx * (V(istr, j, k, ns) - fmax0(cy) * G(1, j - 1) - fmin0(cy) * G(1, j));
          if (S->ub[SW]) cext = dmax(cext, dmin(S->ub[SW][j], 1.0));   /* SPONGE_TUNE (v3dbc_im.F:264-266) */
          V(istr - 1, j, k, nn) = (1. - cext) * V(istr - 1, j, k, nn) + cext * B2(bry_v, SW, j, k);
          V(istr - 1, j, k, nn) = V(istr - 1, j, k, nn) * A2(S->vmask, istr - 1, j);
        }
      }
    else {
      const int j0 = S->c.ns_periodic ? S->jstrV : jstr, j1 = S->c.ns_periodic ? jend : S->jendR;
      for (int k = 1; k <= N; k++)
        for (int j = j0; j <= j1; j++) V(istr - 1, j, k, nn) = S->gamma2 * V(istr, j, k, nn) * A2(S->vmask, istr - 1, j);
    }
  }
  if (S->east_edge) {
    if (OBC_E)
      for (int k = 1; k <= N; k++) {
        for (int j = S->jstrV - 1; j <= jend; j++) {
          G(0, j) = V(iend, j + 1, k, ns) - V(iend, j, k, ns);
          G(1, j) = V(iend + 1, j + 1, k, ns) - V(iend + 1, j, k, ns);
        }
        for (int j = S->jstrV; j <= jend; j++) {
          double cx = 0.125 * dtw * (U(iend + 1, j, k, nr) + U(iend + 1, j - 1, k, nr)) *
                      (A2(S->pm, iend + 1, j) + A2(S->pm, iend + 1, j - 1) + A2(S->pm, iend, j) + A2(S->pm, iend, j - 1));
          const double cy = 0.125 * dtw * (V(iend, j, k, nr) + V(iend + 1, j, k, nr)) *
                            (A2(S->pn, iend + 1, j) + A2(S->pn, iend + 1, j - 1) + A2(S->pn, iend, j) + A2(S->pn, iend, j - 1));
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          V(iend + 1, j, k, nn) = (1. - cx) * (V(iend + 1, j, k, ns) - fmax0(cy) * G(1, j - 1) - fmin0(cy) * G(1, j)) +
                                  cx * (V(iend, j, k, ns) - fmax0(cy) * G(0, j - 1) - fmin0(cy) * G(0, j));
          if (S->ub[SE]) cext = dmax(cext, dmin(S->ub[SE][j], 1.0));   /* SPONGE_TUNE (v3dbc_im.F:344-346) */
          V(iend + 1, j, k, nn) = (1. - cext) * V(iend + 1, j, k, nn) + cext * B2(bry_v, SE, j, k);
          V(iend + 1, j, k, nn) = V(iend + 1, j, k, nn) * A2(S->vmask, iend + 1, j);
        }
      }
    else {
      const int j0 = S->c.ns_periodic ? S->jstrV : jstr, j1 = S->c.ns_periodic ? jend : S->jendR;
      for (int k = 1; k <= N; k++)
        for (int j = j0; j <= j1; j++) V(iend + 1, j, k, nn) = S->gamma2 * V(iend, j, k, nn) * A2(S->vmask, iend + 1, j);
    }
  }
  for (int k = 1; k <= N; k++) {
    if (OBC_S && OBC_W) V(istr - 1, jstr, k, nn) = 0.5 * (V(istr - 1, jstr + 1, k, nn) + V(istr, jstr, k, nn));
    if (OBC_S && OBC_E) V(iend + 1, jstr, k, nn) = 0.5 * (V(iend + 1, jstr + 1, k, nn) + V(iend, jstr, k, nn));
    if (OBC_N && OBC_W) V(istr - 1, jend + 1, k, nn) = 0.5 * (V(istr - 1, jend, k, nn) + V(istr, jend + 1, k, nn));
    if (OBC_N && OBC_E) V(iend + 1, jend + 1, k, nn) = 0.5 * (V(iend + 1, jend, k, nn) + V(iend, jend + 1, k, nn));
  }
}

/* ---------------------------------------------------------------------- */
void or_t3dbc(or_state *S, int it) {
  const int istr = S->istr, iend = S->iend, jstr = S->jstr, jend = S->jend;
  const int nn = S->nnew, ns = S->nstp, nr = S->nrhs, N = S->N;
  const double *rm = S->rmask;
  const double dtw = dtfwd(S);
  static strip2 gs;
  if (S->west_edge) {
    if (OBC_W)
      for (int k = 1; k <= N; k++) {
        for (int j = jstr; j <= jend + 1; j++) {
          G(0, j) = (TT(istr - 1, j, k, ns, it) - TT(istr - 1, j - 1, k, ns, it)) * A2(S->vmask, istr - 1, j);
          G(1, j) = (TT(istr, j, k, ns, it) - TT(istr, j - 1, k, ns, it)) * A2(S->vmask, istr, j);
        }
        for (int j = jstr; j <= jend; j++) {
          double cx = -dtw * U(istr, j, k, nr) * A2(S->pm, istr - 1, j);
          const double cy = 0.5 * dtw * (V(istr - 1, j, k, nr) + V(istr - 1, j + 1, k, nr)) * A2(S->pn, istr - 1, j);
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          TT(istr - 1, j, k, nn, it) = (1. - cx) * (TT(istr - 1, j, k, ns, it) - fmax0(cy) * G(0, j) - fmin0(cy) * G(0, j + 1)) +
                                       cx * (TT(istr, j, k, ns, it) - fmax0(cy) * G(1, j) - fmin0(cy) * G(1, j + 1));
          /* SPONGE_TUNE with ub_tune (t3dbc_im.F:73-74): floor of the binding rate */
          if (S->ub[SW]) cext = dmax(cext, dmin(S->ub[SW][j], 1.0));
          TT(istr - 1, j, k, nn, it) = (1. - cext) * TT(istr - 1, j, k, nn, it) + cext * BT(SW, j, k, it);
          TT(istr - 1, j, k, nn, it) = TT(istr - 1, j, k, nn, it) * A2(rm, istr - 1, j);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int j = jstr; j <= jend; j++) TT(istr - 1, j, k, nn, it) = TT(istr, j, k, nn, it) * A2(rm, istr - 1, j);
  }
  if (S->east_edge) {
    if (OBC_E)
      for (int k = 1; k <= N; k++) {
        for (int j = jstr; j <= jend + 1; j++) {
          G(0, j) = (TT(iend, j, k, ns, it) - TT(iend, j - 1, k, ns, it)) * A2(S->vmask, iend, j);
          G(1, j) = (TT(iend + 1, j, k, ns, it) - TT(iend + 1, j - 1, k, ns, it)) * A2(S->vmask, iend + 1, j);
        }
        for (int j = jstr; j <= jend; j++) {
          double cx = dtw * U(iend + 1, j, k, nr) * A2(S->pm, iend + 1, j);
          const double cy = 0.5 * dtw * (V(iend + 1, j, k, nr) + V(iend + 1, j + 1, k, nr)) * A2(S->pn, iend + 1, j);
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          TT(iend + 1, j, k, nn, it) = (1. - cx) * (TT(iend + 1, j, k, ns, it) - fmax0(cy) * G(1, j) - fmin0(cy) * G(1, j + 1)) +
                                       cx * (TT(iend, j, k, nn, it) - fmax0(cy) * G(0, j) - fmin0(cy) * G(0, j + 1));
          /* SPONGE_TUNE with ub_tune (t3dbc_im.F:73-74): floor of the binding rate */
          if (S->ub[SE]) cext = dmax(cext, dmin(S->ub[SE][j], 1.0));
          TT(iend + 1, j, k, nn, it) = (1. - cext) * TT(iend + 1, j, k, nn, it) + cext * BT(SE, j, k, it);
          TT(iend + 1, j, k, nn, it) = TT(iend + 1, j, k, nn, it) * A2(rm, iend + 1, j);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int j = jstr; j <= jend; j++) TT(iend + 1, j, k, nn, it) = TT(iend, j, k, nn, it) * A2(rm, iend + 1, j);
  }
  if (S->south_edge) {
    if (OBC_S)
      for (int k = 1; k <= N; k++) {
        for (int i = istr; i <= iend + 1; i++) {
          G(1, i) = (TT(i, jstr, k, ns, it) - TT(i - 1, jstr, k, ns, it)) * A2(S->umask, i, jstr);
          G(0, i) = (TT(i, jstr - 1, k, ns, it) - TT(i - 1, jstr - 1, k, ns, it)) * A2(S->umask, i, jstr - 1);
        }
        for (int i = istr; i <= iend; i++) {
          double cx = -dtw * V(i, jstr, k, nr) * A2(S->pn, i, jstr - 1);
          const double cy = 0.5 * dtw * (U(i, jstr - 1, k, nr) + U(i + 1, jstr - 1, k, nr)) * A2(S->pm, i, jstr - 1);
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          TT(i, jstr - 1, k, nn, it) = (1. - cx) * (TT(i, jstr - 1, k, ns, it) - fmax0(cy) * G(0, i) - fmin0(cy) * G(0, i + 1)) +
                                       cx * (TT(i, jstr, k, ns, it) - fmax0(cy) * G(1, i) - fmin0(cy) * G(1, i + 1));
          /* SPONGE_TUNE with ub_tune (t3dbc_im.F:73-74): floor of the binding rate */
          if (S->ub[SS]) cext = dmax(cext, dmin(S->ub[SS][i], 1.0));
          TT(i, jstr - 1, k, nn, it) = (1. - cext) * TT(i, jstr - 1, k, nn, it) + cext * BT(SS, i, k, it);
          TT(i, jstr - 1, k, nn, it) = TT(i, jstr - 1, k, nn, it) * A2(rm, i, jstr - 1);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int i = istr; i <= iend; i++) TT(i, jstr - 1, k, nn, it) = TT(i, jstr, k, nn, it) * A2(rm, i, jstr - 1);
  }
  if (S->north_edge) {
    if (OBC_N)
      for (int k = 1; k <= N; k++) {
        for (int i = istr; i <= iend + 1; i++) {
          G(0, i) = (TT(i, jend, k, ns, it) - TT(i - 1, jend, k, ns, it)) * A2(S->umask, i, jend);
          G(1, i) = (TT(i, jend + 1, k, ns, it) - TT(i - 1, jend + 1, k, ns, it)) * A2(S->umask, i, jend + 1);
        }
        for (int i = istr; i <= iend; i++) {
          double cx = dtw * V(i, jend + 1, k, nr) * A2(S->pn, i, jend + 1);
          const double cy = 0.5 * dtw * (U(i, jend + 1, k, nr) + U(i + 1, jend + 1, k, nr)) * A2(S->pm, i, jend + 1);
          double cext;
          if (cx > 0.) cext = 0.;
          else { cext = -cx; cx = 0.; }
          TT(i, jend + 1, k, nn, it) = (1. - cx) * (TT(i, jend + 1, k, ns, it) - fmax0(cy) * G(1, i) - fmin0(cy) * G(1, i + 1)) +
                                       cx * (TT(i, jend, k, nn, it) - fmax0(cy) * G(0, i) - fmin0(cy) * G(0, i + 1));
          /* SPONGE_TUNE with ub_tune (t3dbc_im.F:73-74): floor of the binding rate */
          if (S->ub[SN]) cext = dmax(cext, dmin(S->ub[SN][i], 1.0));
          TT(i, jend + 1, k, nn, it) = (1. - cext) * TT(i, jend + 1, k, nn, it) + cext * BT(SN, i, k, it);
          TT(i, jend + 1, k, nn, it) = TT(i, jend + 1, k, nn, it) * A2(rm, i, jend + 1);
        }
      }
    else
      for (int k = 1; k <= N; k++)
        for (int i = istr; i <= iend; i++) TT(i, jend + 1, k, nn, it) = TT(i, jend, k, nn, it) * A2(rm, i, jend + 1);
  }
  /* corners: set whenever both edges are physical (t3dbc_im.F:300-415, MASKING) */
#define TCORNER(ic, jc, ia, ja, ib, jb)                                         \
  {                                                                            \
    double cff = A2(rm, ia, ja) + A2(rm, ib, jb);                              \
    if (cff > 0.0) {                                                           \
      cff = 1.0 / cff;                                                         \
      for (int k = 1; k <= N; k++)                                             \
        TT(ic, jc, k, nn, it) = cff * (A2(rm, ia, ja) * TT(ia, ja, k, nn, it) + \
                                       A2(rm, ib, jb) * TT(ib, jb, k, nn, it)); \
    } else                                                                     \
      for (int k = 1; k <= N; k++) TT(ic, jc, k, nn, it) = 0.0;               \
  }
  if (S->south_edge && S->west_edge) TCORNER(istr - 1, jstr - 1, istr, jstr - 1, istr - 1, jstr);
  if (S->south_edge && S->east_edge) TCORNER(iend + 1, jstr - 1, iend, jstr - 1, iend + 1, jstr);
  if (S->north_edge && S->west_edge) TCORNER(istr - 1, jend + 1, istr, jend + 1, istr - 1, jend);
  if (S->north_edge && S->east_edge) TCORNER(iend + 1, jend + 1, iend, jend + 1, iend + 1, jend);
#undef TCORNER
}
