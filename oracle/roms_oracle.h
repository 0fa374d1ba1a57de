/*
 * roms_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99, FP64, no FMA contraction) of the UCLA-ROMS
 * split-explicit time step, used exclusively as the parity checker for the
 * MI355X HIP path (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Nothing in the product links or loads this library.
 *
 * Pinning: the restatement reproduces the reference's own golden log
 * tests/Filament/benchmark.result_github_gnu (per-step KINETIC_ENRG,
 * BAROTR_KE, MAX_ADV_CFL, MAX_VERT_CFL) -- see tests/test_oracle_golden.py.
 *
 * The state layout is the reference's Fortran layout: every horizontal
 * array is (-1:Lm+2, -1:Mm+2), i fastest; rho-point 3-D arrays add (1:N),
 * w-point arrays (0:N); u,v carry 3 time levels, zeta/ubar/vbar 4,
 * t(:,:,:,3,NT).  (/root/reference/src/ocean_vars.F:68-116, tracers.F:327)
 */
#ifndef ROMS_ORACLE_H
#define ROMS_ORACLE_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* analytic case selector */
enum { OR_CASE_FILAMENT = 0, OR_CASE_BASIN = 1, OR_CASE_PIPES = 2, OR_CASE_RIVERS = 3 };
enum { OR_LMD_RIMIX = 8, OR_LMD_CONVEC = 16, OR_LMD_NONLOCAL = 32, OR_LMD_DDMIX = 64 };

typedef struct or_cfg {
  int LLm, MMm, N, NT;           /* interior dims, tracers (T[,S,passive]) */
  int ew_periodic, ns_periodic;
  int salinity, nonlin_eos;      /* nonlin_eos implies SPLIT_EOS */
  int lmd;                       /* 0 or LMD switch bits (as ROMS_LMD_* of include/roms_gpu.h):
                                    1 MIXING, 2 KPP, 4 BKPP (MIXING|KPP|BKPP always together),
                                    8 RIMIX, 16 CONVEC, 32 NONLOCAL, 64 DDMIX */
  int case_id;
  int ntimes;
  double dt; int ndtfast;
  double theta_s, theta_b, hc, rho0;
  double visc2, tnu2;
  double rdrg, rdrg2, Zob;
  double Akv_bak, Akt_bak[2];
  double Tcoef, T0, Scoef, S0;
  double sizex, sizey;           /* analytic domain size [m] */
  int diag_np_xi, diag_np_eta;   /* rank layout emulated in diag sums */
  int surf_flux;                 /* basin: analytic cooling/short-wave/salt fluxes */
  int obc;                       /* open edges: 1 W, 2 E, 4 S, 8 N (OBC_WEST..; Flather/Orlanski + *_FRC_BRY) */
  double ubind;                  /* OBC binding velocity [m/s] (read_inp_mod.F:809) */
  double v_sponge;               /* SPONGE viscosity/diffusivity [m2/s] (set_nudgcof.F:25-111) */
  int island;                    /* basin: circular land mask (MASKING) */
  int curvgrid;                  /* CURVGRID (+UV_ADV) curvature terms; basin: non-uniform metrics */
  int uv_adv, uv_cor;            /* UV_ADV, UV_COR */
  int pot_tides;                 /* TIDES pot_tides: ptide in prsgrd (prsgrd.F:209-211) */
  int bulk_frc;                  /* BULK_FRC (bulk_frc.F); basin: analytic atmosphere (oracle_main.c) */
  int adv_isoneutral;            /* ADV_ISONEUTRAL (+SW_TRIADS, STABILIZE): oracle_iso.c */
} or_cfg;

typedef struct or_state or_state;

or_state *or_create(const or_cfg *cfg);
void      or_destroy(or_state *S);
/* roms_init (main.F:85-321) : grid, ICs, set_depth, set_HUV, omega, rho_eos, diag */
int       or_init(or_state *S);
/* one roms_step (main.F:333-520); returns 0 */
int       or_step(or_state *S);

/* norms printed by diag (diag.F code_check line) for the last diag call */
void      or_norms(const or_state *S, double out[4]);
int       or_iic(const or_state *S);
int       or_nfast(const or_state *S);
const double *or_weights(const or_state *S); /* weight(2,nfast), column-major */

/* field access: returns pointer + element count of a named array */
double   *or_field(or_state *S, const char *name, size_t *count);
/* set_frc_data records (time in days) and the in-step clock (start_time [s]) */
int       or_frc_record(or_state *S, const char *name, int slot, double time, const double *data);
void      or_frc_clock(or_state *S, double start_time, int on);
int       or_set_pipes(or_state *S, int npip, const double *idx, const double *flx, const double *prf,
                       const double *trc);
/* scalar time indices: iic kstp knew nstp nrhs nnew */
void      or_tindex(const or_state *S, int out[6]);

/* individual routines (same names as the reference), for per-routine parity */
void or_rho_eos(or_state *S, int tidx);
void or_set_HUV(or_state *S);
void or_omega(or_state *S);
void or_prsgrd(or_state *S);
void or_pre_step3d(or_state *S);
void or_set_HUV1(or_state *S);
void or_step3d_uv1(or_state *S);
void or_visc3d(or_state *S);
void or_step2d(or_state *S);
void or_step3d_uv2(or_state *S);
void or_step3d_t(or_state *S);
void or_t3dmix(or_state *S);
void or_set_depth(or_state *S);
void or_lmd_vmix(or_state *S, int tind);
void or_swr_frac(or_state *S);
void or_bulk_flux(or_state *S);   /* calc_all_bulk_forces at nrhs (oracle_bulk.c) */
void or_diag(or_state *S);
void or_set_tindex(or_state *S, const int in[6]);
void or_set_iif(or_state *S, int iif);
/* set_river_frc: new riv_vol(nriv), riv_trc(nriv,NT) (faces kept) */
void or_set_river(or_state *S, int nriv, const double *vol, const double *trc);
void or_set_ub(or_state *S, const double *w, const double *e, const double *s, const double *n);

#ifdef __cplusplus
}
#endif
#endif
