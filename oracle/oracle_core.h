/*
 * oracle_core.h -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 * Private state struct and Fortran-layout index macros of the CPU oracle.
 */
#ifndef ORACLE_CORE_H
#define ORACLE_CORE_H
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "roms_oracle.h"

struct or_state {
  or_cfg c;
  int Lm, Mm, N, NT, nTS;          /* nTS = iTandS */
  int nx2, ny2;                    /* Lm+4, Mm+4 */
  size_t n2, n3, n3w;              /* 2-D size, N*n2, (N+1)*n2 */
  /* tile bounds (single tile covering the domain, tile=0) */
  int istr, iend, jstr, jend;
  int west_edge, east_edge, south_edge, north_edge;  /* physical edges */
  int istrU, istrR, iendR, jstrV, jstrR, jendR;      /* auxiliary bounds */
  int istrE, iendE, jstrE, jendE;                    /* extended bounds */
  /* time indices and scalars */
  int iic, ntstart, forw_start, iif, nfast, kstp, knew, nstp, nrhs, nnew;
  double dt, dtfast, g, rho0, vonKar, qp2, gamma2;
  double weight[2][288];
  double *Cs_w, *Cs_r;
  /* grid */
  double *h, *hinv, *f, *fomn, *xr, *yr, *pm, *pn, *dm_r, *dn_r, *pn_u, *dm_u,
         *dn_u, *dm_v, *pm_v, *dn_v, *dm_p, *dn_p, *iA_u, *iA_v, *pmon_u,
         *pnom_v, *rmask, *pmask, *umask, *vmask;
  double *dndx, *dmde;             /* CURVGRID: d(1/n)/dxi, d(1/m)/deta (setup_grid1.F:89-103) */
  double *ptide;                   /* tides.F:26 surface tidal potential (TIDES) */
  double area, volume;
  /* ocean vars */
  double *zeta, *ubar, *vbar, *u, *v, *t;
  double *FlxU, *FlxV, *We, *Wi, *Hz, *Hz_u, *Hz_v, *z_r, *z_w;
  /* coupling */
  double *rufrc, *rvfrc, *rhoA, *rhoS, *r_D, *Zt_avg1, *DU_avg1, *DV_avg1,
         *DU_avg2, *DV_avg2, *DU_avg_bak, *DV_avg_bak;
  /* eos / mixing */
  double *rho, *rho1, *qp1, *bvf;
  double *Akv, *Akt, *visc2_r, *visc2_p, *diff2;
  double *hbls, *hbbl, *ghat, *swr_frac;
  double *lmdKv, *lmdKt, *lmdKs, *lmdRig;  /* lmd_vmix A3d scratch (0:N) */
  double *lmd2[9];                         /* lmd_kpp A2d scratch */
  /* pipe_frc.F: pipe_idx>0 cells carry pipe_flx of pipe pidx = pipe_idx;
     pipe_prf(npip,N) and pipe_trc(npip,NT) column-major (pipe_frc.F:34-35,198),
     indexed by pidx as omega.F:102-108 and step3d_t_ISO.F:927-934 do */
  int pipe_source, npip;
  double *pipe_flx, *pipe_idx, *pipe_prf, *pipe_trc;
  /* river_frc.F: riv_uflx/riv_vflx = 10*iriver + signed fraction on the
     faces between a river-mouth land cell and its wet neighbours;
     riv_vol(nriv), riv_trc(nriv,NT) column-major */
  int river_source, nriv;
  double *riv_uflx, *riv_vflx, riv_vol[16], riv_trc[16 * 16];
  /* open-boundary data (boundary.F:21-39): [0] west, [1] east (index j, 0:Mm+1),
     [2] south, [3] north (index i, 0:Lm+1); u,v (.,N), t (.,N,NT) */
  int nbry[4];
  double *bry_zeta[4], *bry_ubar[4], *bry_vbar[4], *bry_u[4], *bry_v[4], *bry_t[4];
  double *ub[4];   /* SPONGE_TUNE ub_west/east/south/north (NULL: ub_tune off), indexed like bry_* */
  /* forcing */
  double *sustr, *svstr, *stflx, *srflx, *swflx;
  /* BULK_FRC inputs and rho-point stresses (bulk_frc.F, surf_flux.F) */
  double *uwnd, *vwnd, *tair, *qair, *prate, *swrad, *lwrad, *sustr_r, *svstr_r;
  /* set_frc_data's two records per field (roms_read_write.F:303-392) and the
     in-step interpolation points of roms_step (main.F:373-441) */
  struct { double *dst; size_t n; int bry; double t[3]; double *rec[3]; int k; } frc[64];   /* k: it1's place in time order */
  int nfrc, frc_clock;
  double frc_start;
  /* ADV_ISONEUTRAL (oracle_iso.c): eos_vars.F:28-31 slopes and inverse
     vertical gradient, mixing.F:24-27 diff3u/v, step3d_t's Akz (0:N), and
     the operator's two-slice scratch FSC, dTdz, dTdx, dTde (2 x n2) + LapT */
  double *dRdx, *dRde, *idRz, *diff3u, *diff3v, *Akz;
  double *iso_FSC, *iso_dTdz, *iso_dTdx, *iso_dTde, *iso_LapT;
  /* private scratch (A3d(:,1..4), A2d(:,1..)) */
  double *ru, *rv, *P, *rhos3;         /* 3-D scratch */
  double *s2[14];                      /* 2-D scratch */
  double *c1[6];                       /* 1-D column scratch (i, 0:N) */
  /* diag results */
  double norms[4];
  double avke, avke2b, Cu_Adv, Cu_W;
};

/* Fortran-layout index helpers: horizontal (-1:Lm+2,-1:Mm+2) */
#define O2(i, j) ((size_t)((i) + 1) + (size_t)((j) + 1) * (size_t)S->nx2)
#define A2(a, i, j) ((a)[O2(i, j)])
#define R3(a, i, j, k) ((a)[O2(i, j) + (size_t)((k)-1) * S->n2])  /* 1:N */
#define W3(a, i, j, k) ((a)[O2(i, j) + (size_t)(k) * S->n2])      /* 0:N */
#define L2(a, i, j, l) ((a)[O2(i, j) + (size_t)((l)-1) * S->n2])  /* (:,:,4) */
#define L3(a, i, j, k, l) \
  ((a)[O2(i, j) + (size_t)((k)-1) * S->n2 + (size_t)((l)-1) * S->n3])
#define TT(i, j, k, l, itr)                                         \
  (S->t[O2(i, j) + (size_t)((k)-1) * S->n2 + (size_t)((l)-1) * S->n3 + \
        (size_t)((itr)-1) * 3 * S->n3])
#define C1(a, i, k) ((a)[(size_t)((i) + 1) + (size_t)(k) * (size_t)S->nx2])

#define ZETA(i, j, l) L2(S->zeta, i, j, l)
#define UBAR(i, j, l) L2(S->ubar, i, j, l)
#define VBAR(i, j, l) L2(S->vbar, i, j, l)
#define U(i, j, k, l) L3(S->u, i, j, k, l)
#define V(i, j, k, l) L3(S->v, i, j, k, l)
#define HZ(i, j, k) R3(S->Hz, i, j, k)
#define ZR(i, j, k) R3(S->z_r, i, j, k)
#define ZW(i, j, k) W3(S->z_w, i, j, k)
#define FLXU(i, j, k) R3(S->FlxU, i, j, k)
#define FLXV(i, j, k) R3(S->FlxV, i, j, k)
#define WE(i, j, k) W3(S->We, i, j, k)
#define WI(i, j, k) W3(S->Wi, i, j, k)
#define AKV(i, j, k) W3(S->Akv, i, j, k)
#define AKT(i, j, k, it) ((S->Akt)[O2(i, j) + (size_t)(k) * S->n2 + (size_t)((it)-1) * S->n3w])

static inline double fmax0(double a) { return a > 0.0 ? a : 0.0; }
static inline double fmin0(double a) { return a < 0.0 ? a : 0.0; }
static inline double dmax(double a, double b) { return a > b ? a : b; }
static inline double dmin(double a, double b) { return a < b ? a : b; }

/* exchanges (mpi_exchanges.F semantics for a single rank) */
void or_exch2(or_state *S, double *a);
void or_exch3(or_state *S, double *a, int nlev);
/* lateral boundary conditions for closed walls (zetabc.F, u2dbc_im.F, ...) */
void or_zetabc(or_state *S, double *zeta_new);
void or_u2dbc(or_state *S);
void or_v2dbc(or_state *S);
void or_u3dbc(or_state *S);
void or_v3dbc(or_state *S);
void or_t3dbc(or_state *S, int itrc);
void or_river_uv(or_state *S, int nnew);   /* river velocities in u,v(nnew) */
/* open boundaries: sponge (set_nudgcof.F) and analytic boundary data */
void or_set_nudgcof(or_state *S);
void or_ana_bry(or_state *S);
/* analytic cases */
void or_ana_grid(or_state *S);
void or_ana_init(or_state *S);
void or_ana_forces(or_state *S);
/* LMD/KPP (oracle_lmd.c) */
void or_lmd_vmix_impl(or_state *S, int tind);
void or_lmd_alloc(or_state *S);
/* ADV_ISONEUTRAL (oracle_iso.c) */
void or_iso_dRdx(or_state *S, int k, double *rx, int imin, int imax);
void or_iso_dRde(or_state *S, int k, double *rx, int jmin, int jmax);
void or_iso_exch_slopes(or_state *S);
void or_iso_diff3(or_state *S, int iu0, int iu1, int iv0, int iv1, int j0, int j1);
void or_iso_exch_diff3(or_state *S);
void or_iso_tracer(or_state *S, int itrc);
#endif
