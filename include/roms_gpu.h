/*
 * roms_gpu.h -- C ABI of the MI355X-native UCLA-ROMS split-explicit hot path.
 *
 * Drop-in boundary: the reference's hot-path
 * routines are argument-less / (tile) / (tidx) external Fortran subroutines
 * that read and write module arrays (/root/reference/src/main.F:397-479).
 * Each routine below replaces one of them; all state they touch lives in
 * device memory owned by this library, in the reference's Fortran layout
 * (-1:Lm+2, -1:Mm+2 [,levels] [,time] [,tracer]), i fastest.  Host arrays are
 * borrowed only across roms_gpu_register .. roms_gpu_finalize and are copied
 * explicitly with roms_gpu_upload / roms_gpu_download.
 *
 * One process drives one GPU (one MPI rank / one subdomain, like the
 * reference's one rank per tile).  Every entry returns 0 on success and a
 * negative code on failure; roms_gpu_last_error() gives the message (the
 * reference's error_log%raise_* + abort_check, error_handling_mod.F90:144-365).
 * Routine entries enqueue on the library's HIP stream and return immediately;
 * roms_gpu_sync() waits.
 */
#ifndef ROMS_GPU_H
#define ROMS_GPU_H

#ifdef __cplusplus
extern "C" {
#endif

#define ROMS_GPU_ABI_VERSION 16
#define ROMS_MAX_FAST 288

/* Subdomain geometry of this rank: param.F / dimensions.F / mpi_setup.F:39-210 */
typedef struct roms_dims {
  int Lm, Mm, N, NT;             /* local interior size, levels, tracers   */
  int LLm, MMm;                  /* global interior size                   */
  int np_xi, np_eta, inode, jnode;
  int iSW_corn, jSW_corn;        /* offset of this subdomain (mpi_setup.F) */
  int ew_periodic, ns_periodic;  /* EW_PERIODIC / NS_PERIODIC              */
  int west_exchng, east_exchng, south_exchng, north_exchng; /* message edges */
} roms_dims;

/* LMD switch bits of roms_cfg.lmd_mixing / roms_case.lmd_mixing (cppdefs.opt).
 * Accepted sets are the ones the reference builds and runs correctly:
 *   0 (no LMD_MIXING), or MIXING|KPP|BKPP plus any of RIMIX, NONLOCAL,
 *   CONVEC (CONVEC needs RIMIX) and DDMIX (double diffusion, lmd_vmix.F:279-
 *   360; needs SALINITY for t(..,isalt)).  KPP without BKPP does not compile in the
 *   reference (lmd_kpp.F:178 reads hbbl, imported only under LMD_BKPP,
 *   lmd_kpp.F:37-39); MIXING without KPP/BKPP filters Kv(0), Kv(N) that are
 *   never set (lmd_vmix.F:405-420); CONVEC without RIMIX tests an unset Rig
 *   (lmd_vmix.F:269-274).  The Pipes_ana set is ROMS_LMD_ALL, the Iceland
 *   set (Examples/Iceland/Iceland_parent/cppdefs.opt:41-46) ROMS_LMD_ICELAND. */
#define ROMS_LMD_MIXING   1
#define ROMS_LMD_KPP      2
#define ROMS_LMD_BKPP     4
#define ROMS_LMD_RIMIX    8
#define ROMS_LMD_CONVEC   16
#define ROMS_LMD_NONLOCAL 32
#define ROMS_LMD_ALL      63   /* MIXING..NONLOCAL: the Pipes_ana set (no DDMIX) */
#define ROMS_LMD_ICELAND  47   /* all but LMD_CONVEC */
#define ROMS_LMD_DDMIX    64

/* cppdefs.opt switches and run scalars (scalars.F, read_inp_mod.F, set_weights.F).
 * Switches that need no flag here: MASKING is carried by the mask arrays
 * (all-ones masks reproduce a build without it); IMPLICIT_BOTTOM_DRAG is
 * forced on inside step3d_uv1.F:138 / step3d_uv2.F:82 and its only other use
 * (compute_rd_bott_drag.h:41) is masked by IMPLCT_NO_SLIP_BTTM_BC, always
 * defined (set_global_definitions.h:73). */
typedef struct roms_cfg {
  int nonlin_eos;                /* NONLIN_EOS (+SPLIT_EOS)                */
  int salinity;                  /* SALINITY                               */
  int lmd_mixing;                /* 0 or ROMS_LMD_* bits (see above)       */
  int uv_vis2, ts_dif2;          /* UV_VIS2, TS_DIF2                        */
  double dt;                     /* baroclinic step [s]                    */
  int ndtfast, nfast;            /* mode splitting                         */
  double weight[2][ROMS_MAX_FAST]; /* fast-time averaging weights (C order [2][288]) */
  double g, rho0, rdrg, rdrg2, Zob, gamma2;
  double Akv_bak, Akt_bak[2];
  double Tcoef, T0, Scoef, S0;   /* linear EOS                              */
  double theta_s, theta_b, hc;   /* S-coordinate                            */
  int obc;                       /* open edges (OBC_WEST 1, OBC_EAST 2, OBC_SOUTH 4, OBC_NORTH 8) with
                                    OBC_M2FLATHER, OBC_M3ORLANSKI, OBC_TORLANSKI and Z/M2/M3/T_FRC_BRY;
                                    closed walls elsewhere (zetabc.F, u2dbc_im.F ... t3dbc_im.F)  */
  double ubind;                  /* OBC binding velocity [m/s] (scalars.F, read_inp_mod.F:809)    */
  int curvgrid;                  /* CURVGRID (with UV_ADV): curvature terms in the momentum r.h.s. */
  int uv_adv, uv_cor;            /* UV_ADV (horizontal + vertical momentum advection,
                                    compute_horiz_rhs_uv_terms.h:42-291, compute_vert_rhs_uv_terms.h),
                                    UV_COR (Coriolis, compute_horiz_rhs_uv_terms.h:1-38)              */
  int pot_tides;                 /* TIDES with pot_tides (tides.opt): the surface tidal potential
                                    ptide enters the pressure gradient (prsgrd.F:209-211)             */
  int bulk_frc;                  /* BULK_FRC: the surface fluxes come from roms_gpu_bulk_flux (COARE,
                                    bulk_frc.F:143-913) at both set_forces points of the step, and
                                    lmd_kpp's u* from the rho-point stresses (lmd_kpp.F:173-174)     */
  int adv_isoneutral;            /* ADV_ISONEUTRAL (with SW_TRIADS and STABILIZE, step3d_t_ISO.F:15-18):
                                    corrector prsgrd forms the slopes dRdx/dRde (prsgrd.F:307-338),
                                    step3d_uv2 diff3u/diff3v/idRz (step3d_uv2.F:572-697), step3d_t
                                    centred (not UPSTREAM_TS) fluxes, the rotated biharmonic operator
                                    and Akt+Akz in the implicit diffusion (step3d_t_ISO.F:253-1065)  */
} roms_cfg;

/* Time-step indices (scalars.F:32-36).  The step entry updates them. */
typedef struct roms_tlev {
  int iic, ntstart, forw_start, iif, nfast, kstp, knew, nstp, nrhs, nnew;
} roms_tlev;

/* Field identifiers: the reference's module arrays (names as in the source) */
enum roms_field {
  ROMS_ALL = -1,
  /* grid.F */
  ROMS_h = 0, ROMS_hinv, ROMS_f, ROMS_fomn, ROMS_pm, ROMS_pn, ROMS_dm_r, ROMS_dn_r, ROMS_dm_u, ROMS_dn_u,
  ROMS_dm_v, ROMS_dn_v, ROMS_dm_p, ROMS_dn_p, ROMS_pmon_u, ROMS_pnom_v, ROMS_rmask, ROMS_pmask, ROMS_umask,
  ROMS_vmask,
  /* scoord.F (N+1 each) */
  ROMS_Cs_w, ROMS_Cs_r,
  /* ocean_vars.F, tracers.F */
  ROMS_zeta, ROMS_ubar, ROMS_vbar, ROMS_u, ROMS_v, ROMS_t, ROMS_FlxU, ROMS_FlxV, ROMS_We, ROMS_Wi,
  ROMS_Hz, ROMS_Hz_u, ROMS_Hz_v, ROMS_z_r, ROMS_z_w,
  /* coupling.F */
  ROMS_rufrc, ROMS_rvfrc, ROMS_rhoA, ROMS_rhoS, ROMS_r_D, ROMS_Zt_avg1, ROMS_DU_avg1, ROMS_DV_avg1,
  ROMS_DU_avg2, ROMS_DV_avg2, ROMS_DU_avg_bak, ROMS_DV_avg_bak,
  /* eos_vars.F, mixing.F */
  ROMS_rho, ROMS_rho1, ROMS_qp1, ROMS_bvf, ROMS_Akv, ROMS_Akt, ROMS_visc2_r, ROMS_visc2_p, ROMS_diff2,
  ROMS_hbls, ROMS_hbbl, ROMS_ghat, ROMS_swr_frac,
  /* surf_flux.F */
  ROMS_sustr, ROMS_svstr, ROMS_stflx, ROMS_srflx, ROMS_swflx,
  /* private scratch carried between routines (prsgrd -> pre_step3d/step3d_uv1) */
  ROMS_ru, ROMS_rv,
  /* boundary.F:21-39 open-boundary data: *_west/_east indexed j=0:Mm+1, *_south/_north i=0:Lm+1;
     u,v (.,N); t (.,N,NT) -- column-major like the reference allocations (boundary.F:111-129) */
  ROMS_zeta_west, ROMS_zeta_east, ROMS_zeta_south, ROMS_zeta_north,
  ROMS_ubar_west, ROMS_ubar_east, ROMS_ubar_south, ROMS_ubar_north,
  ROMS_vbar_west, ROMS_vbar_east, ROMS_vbar_south, ROMS_vbar_north,
  ROMS_u_west, ROMS_u_east, ROMS_u_south, ROMS_u_north,
  ROMS_v_west, ROMS_v_east, ROMS_v_south, ROMS_v_north,
  ROMS_t_west, ROMS_t_east, ROMS_t_south, ROMS_t_north,
  /* grid.F CURVGRID metric derivatives d(1/n)/dxi, d(1/m)/deta (setup_grid1.F:89-103) */
  ROMS_dndx, ROMS_dmde,
  /* tides.F:26 surface tidal potential [m] (TIDES, pot_tides) */
  ROMS_ptide,
  /* BULK_FRC inputs at rho points (bulk_frc.F:95-111, surf_flux.F): winds [m/s], air temperature
     [degC], specific humidity Q [kg/kg], precipitation [cm/day], short-wave (the data read into
     srflx) and downward long-wave radiation [W/m2]; and the rho-point stresses sustr_r, svstr_r */
  ROMS_uwnd, ROMS_vwnd, ROMS_tair, ROMS_qair, ROMS_prate, ROMS_swrad, ROMS_lwrad, ROMS_sustr_r, ROMS_svstr_r,
  ROMS_NFIELDS
};

/* ---- lifecycle ---- */
int  roms_gpu_abi_version(void);
/* Allocates device state (the only allocating entry).  device: HIP device
 * ordinal; comm: handle from roms_gpu_comm_create / _create_local for a
 * processor grid np_xi*np_eta > 1 (rank = inode + jnode*np_xi, as
 * mpi_setup.F:60-61), NULL for a single rank, whose periodic halos are
 * wrapped on-device.                                                        */
int  roms_gpu_init(const roms_dims *dims, const roms_cfg *cfg, int device, void *comm);
int  roms_gpu_finalize(void);
const char *roms_gpu_last_error(void);
/* element count of a field in the Fortran layout of this rank */
long roms_gpu_field_size(int field_id);
/* host mirror for upload/download (init_arrays.F; host keeps ownership)     */
int  roms_gpu_register(int field_id, double *host_ptr, long count);
int  roms_gpu_upload(int field_id);      /* host -> device, ROMS_ALL allowed */
int  roms_gpu_download(int field_id);    /* device -> host, ROMS_ALL allowed */
/* direct synchronous copies without registration                            */
int  roms_gpu_copy_in(int field_id, const double *src, long count);
int  roms_gpu_copy_out(int field_id, double *dst, long count);
/* ROMS_Hz_u / ROMS_Hz_v (set_HUV's cell heights, set_depth.F:220,227) are
 * read by no routine of the step, only by extract_data.F:726.  roms_gpu_step
 * stores them only while either is registered for transfer or the
 * environment sets ROMS_GPU_HZ_UV=1 (2 array passes per step saved); after a
 * step that did not, downloading or copying them out returns -5.  The
 * routine roms_gpu_set_huv always stores them. */
int  roms_gpu_sync(void);
void *roms_gpu_stream(void);             /* hipStream_t the routines run on  */

/* ---- hot-path routines (reference entry points they replace) ---- */
int roms_gpu_rho_eos(int tidx, const roms_tlev *t);   /* rho_eos(tidx)   rho_eos.F:6      */
int roms_gpu_set_huv(const roms_tlev *t);             /* set_HUV          set_depth.F:190  */
int roms_gpu_omega(const roms_tlev *t);               /* omega            omega.F:4        */
int roms_gpu_lmd_vmix(int tind, const roms_tlev *t);  /* lmd_vmix(tind)   lmd_vmix.F:5     */
int roms_gpu_prsgrd(const roms_tlev *t);              /* prsgrd           prsgrd.F:4       */
int roms_gpu_pre_step3d(const roms_tlev *t);          /* pre_step3d(tile) pre_step3d4S.F:4 */
int roms_gpu_set_huv1(const roms_tlev *t);           /* set_HUV1(tile)   set_depth.F:239  */
int roms_gpu_step3d_uv1(const roms_tlev *t);          /* step3d_uv1(tile) step3d_uv1.F:5   */
int roms_gpu_visc3d(const roms_tlev *t);              /* visc3d           visc3d_S.F:4     */
int roms_gpu_step2d(const roms_tlev *t);              /* step2d           step2d_FB.F:3    */
int roms_gpu_step3d_uv2(const roms_tlev *t);          /* step3d_uv2(tile) step3d_uv2.F:6   */
int roms_gpu_step3d_t(const roms_tlev *t);            /* step3d_t(tile)   step3d_t_ISO.F:20*/
int roms_gpu_t3dmix(const roms_tlev *t);              /* t3dmix           t3dmix_S.F:4     */
int roms_gpu_swr_frac(const roms_tlev *t);            /* swr_frac(tile)   lmd_swr_frac.F:4 */
/* set_pipe_frc (pipe_frc.F:33-80): the host's pipe_idx (0 = no pipe) and
 * pipe_flx on the (-1:Lm+2,-1:Mm+2) grid, pipe_prf(npip,N) and
 * pipe_trc(npip,NT) column-major.  npip = 0 switches pipe sources off.
 * Call again whenever set_forces updates them; the next step uses them.      */
int roms_gpu_set_pipe_frc(int npip, const int *pipe_idx, const double *pipe_flx, const double *pipe_prf,
                          const double *pipe_trc);
/* set_river_frc (river_frc.F:57-96, init_river_frc :98-222, calc_river_flux
 * :224-282): riv_uflx and riv_vflx as calc_river_flux leaves them on the
 * (-1:Lm+2,-1:Mm+2) grid (10*iriver + the signed flux fraction on every face
 * between a river-mouth cell and a wet neighbour, 0 elsewhere), riv_vol(nriv)
 * [m3/s] and riv_trc(nriv,NT) column-major for the current time.  Passing
 * riv_uflx = riv_vflx = NULL keeps the face arrays of an earlier call and
 * updates only the time-dependent riv_vol/riv_trc.  nriv = 0 switches river
 * sources off.  Returns 0, or -1 on a bad argument. */
int roms_gpu_set_river_frc(int nriv, const double *riv_uflx, const double *riv_vflx, const double *riv_vol,
                           const double *riv_trc);
/* set_bulk_frc -> calc_all_bulk_forces (bulk_frc.F:85-913) on the device:
 * from the uploaded ROMS_uwnd .. ROMS_lwrad fields and the surface t, u, v at
 * t->nrhs, sets srflx, stflx(itemp), swflx, sustr_r, svstr_r, sustr and
 * svstr.  roms_gpu_step calls it itself at both set_forces points when the
 * library was initialised with bulk_frc; the host only uploads the
 * time-interpolated atmospheric fields (set_frc_data) before each step.
 * Returns -4 when the library was initialised without bulk_frc. */
int roms_gpu_bulk_flux(const roms_tlev *t);
/* SPONGE_TUNE with ub_tune (sponge_tune.F, t3dbc_im.F:73-74): the per-edge
 * binding coefficients ub_west(j), ub_east(j) (j = 0..Mm+1) and ub_south(i),
 * ub_north(i) (i = 0..Lm+1) that the host's adjust_orlanski maintains from
 * the parent/child baroclinic pressure fluxes; t3dbc's Orlanski blend then
 * uses cext = max(cext, min(ub(j), 1)).  NULL switches an edge off (the
 * reference default ub_tune = .false., sponge_tune.opt).  Call again after
 * every adjust_orlanski; the next step uses the new values.                 */
int roms_gpu_set_ub_tune(const double *ub_west, const double *ub_east, const double *ub_south, const double *ub_north);
int roms_gpu_set_depth(const roms_tlev *t);           /* set_depth(tile)  set_depth.F:4    */

/* One whole roms_step (main.F:333-520, forcing held fixed): advances t->iic
 * and leaves nstp/nrhs/nnew/kstp/knew as the reference does.  Steady-state
 * steps replay a captured HIP graph.                                        */
int roms_gpu_step(roms_tlev *t);
/* roms_init device sequence after the host uploaded grid + initial state:
 * set_depth, set_HUV, omega, rho_eos(nrhs) (main.F:268-288).                 */
int roms_gpu_init_sequence(roms_tlev *t);

/* ---- analytic cases (host-side ana_grid/ana_init restatements) ---- */
enum roms_case_id { ROMS_CASE_FILAMENT = 0, ROMS_CASE_BASIN = 1, ROMS_CASE_PIPES = 2, ROMS_CASE_RIVERS = 3 };
typedef struct roms_case {
  int case_id, LLm, MMm, N, NT;
  int salinity, nonlin_eos, lmd_mixing;  /* lmd_mixing: 0 or ROMS_LMD_* bits */
  double dt; int ndtfast;
  double sizex, sizey;
  int surf_flux;  /* basin only: analytic cooling, short-wave and salt fluxes (else 0) */
  int obc;        /* basin only: open edges (roms_cfg.obc) with analytic boundary data, ubind 0.1 */
  double v_sponge;/* basin only: SPONGE band viscosity/diffusivity [m2/s] (set_nudgcof.F)      */
  int island;     /* basin only: circular land mask (MASKING)                                   */
  int curvgrid;   /* basin only: non-uniform metrics pm(j), pn(i) and CURVGRID                  */
  int uv_adv, uv_cor;  /* UV_ADV, UV_COR (every reference case defines both: set 1, 1)          */
  int bulk_frc;   /* basin only: BULK_FRC with an analytic atmosphere (westerly jet, cool humid air)
                     uploaded as ROMS_uwnd .. ROMS_lwrad; roms_cfg.bulk_frc                         */
  int adv_isoneutral;  /* ADV_ISONEUTRAL (roms_cfg.adv_isoneutral), any case                            */
} roms_case;
/* Builds the analytic grid/ICs on the host (setup_grid1/2, set_scoord,
 * set_weights, ana_init), initialises the device and runs roms_init.        */
int roms_gpu_init_case(const roms_case *c, int device, roms_tlev *t);
/* Same on this rank's subdomain of an np_xi x np_eta processor grid
 * (mpi_setup.F:39-154 bounds); comm's rank selects inode,jnode.             */
int roms_gpu_init_case_comm(const roms_case *c, int np_xi, int np_eta, void *comm, int device, roms_tlev *t);

/* ---- communicators for the halo exchange (mpi_exchanges.F) ----
 * RCCL: rank 0 calls roms_gpu_comm_unique_id, the 128-byte id is broadcast
 * by the host's own means (MPI_Bcast in a Fortran driver, torch.distributed
 * in the Python one), then every rank calls roms_gpu_comm_create.
 * _create_local: subdomains driven by threads of ONE process (testing).     */
int roms_gpu_comm_unique_id(void *id128);
int roms_gpu_comm_create(const void *id128, int nranks, int rank, int device, void **comm);
int roms_gpu_comm_create_local(int group, int nranks, int rank, void **comm);
/* Host channel: the host supplies its own allgather (every rank calls it
 * with the same nbytes; recv holds nranks * nbytes, rank r's bytes at
 * r * nbytes; returns 0 on success) -- MPI_Allgather(MPI_BYTE) over the
 * reference's communicator (mpi_exchanges.F, mpi_setup.F), a file or socket
 * channel in a test.  It carries only the IPC handles at init and the small
 * diag / area-volume gathers; every halo exchange moves GPU to GPU by IPC
 * peer writes, with RCCL out of the loop.  roms_gpu_init fails if the IPC
 * transport cannot be set up (its self-test reference is a host-staged
 * exchange over the same channel).                                          */
typedef int (*roms_host_allgather_fn)(void *ctx, const void *send, long nbytes, void *recv);
int roms_gpu_comm_create_host(int nranks, int rank, int device, roms_host_allgather_fn allgather, void *ctx,
                              void **comm);
int roms_gpu_comm_destroy(void *comm);
/* Halo transport of this rank after roms_gpu_init: 0 = RCCL send/recv (or
 * single rank / in-process), 1 = IPC peer writes (RCCL communicator: enabled
 * after a start-up self-test against RCCL, ROMS_GPU_HALO_IPC=0 disables;
 * host-channel communicator: always), -1 = IPC with a timed-out arrival wait
 * since init.                                                               */
int roms_gpu_halo_transport(void);
/* Halo exchanges (one reference exchange_xxx call each) in the last whole
 * step this rank enqueued (eager or graph capture; 0 on one rank without a
 * communicator), and the fast-loop exchange interval: the barotropic loop
 * exchanges zeta/ubar/vbar after every *fast_interval-th fast step over
 * 2*fast_interval-deep halos and recomputes the overlap in between (1: every
 * fast step, as step2d_FB.F:572-574; multi-rank runs without open edges
 * default to 4, ROMS_GPU_S2D_K=1..8; K is lowered until 2K+2 fits the
 * smallest subdomain of the mpi_setup.F split, the same on every rank;
 * rivers and pipes take every step).                                         */
int roms_gpu_halo_exchanges(long *per_step, int *fast_interval);
/* 1 if whole steps defer each producer's 3-D exchange onto the halo stream
 * beside the next routine that reads none of its halo (the default with
 * > 1 rank when every rank drives its own GPU; ROMS_GPU_XOVERLAP=1 forces
 * it on, =0 off), 0 if every exchange runs in place, as the reference's
 * exchange_xxx calls do (mpi_exchanges.F:672-800).                          */
int roms_gpu_halo_overlap(void);
/* 1 if the fused fast step addresses its 2-D fields through one buffer
 * window (the fields allocated side by side within 2 GiB; the default),
 * 0 if through their pointers (ROMS_GPU_S2D_WIN=0, or a subdomain whose
 * 2-D fields span more).  Same results either way.                         */
int roms_gpu_s2d_window(void);
/* Self-test of the allocation path: `chunks` arrays of n doubles filled
 * with ones and freed, then allocated again through the library's
 * zero-filling allocator; on the library's stream each is read at once
 * (elements not zero: stale data) and overwritten with ones, and after the
 * device drains the elements not one are counted (writes undone by a late
 * fill).  *bad = both counts (0 unless the null-stream fill races the
 * library's non-blocking stream, the round-2 failure mode).                 */
int roms_gpu_selftest_zero_fill(long n, int chunks, long *bad);
/* Host-only: neighbour ranks (-1 none), per-level message sizes for the 8
 * directions W,E,S,N,SW,SE,NW,NE, and the strip extents {i0,i1,j0,j1}.      */
int roms_gpu_halo_plan(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic,
                       int ns_periodic, int peer[8], long count[8], int strip[4]);
/* Host-only: the (i,j) cells, in message order, that direction dir packs
 * (unpack=0, from this rank's interior) or unpacks into (unpack=1, halo).
 * Returns the per-level count (<= cap) or -1.                               */
long roms_gpu_halo_map(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic,
                       int ns_periodic, int dir, int unpack, int *i, int *j, long cap);
/* Host-only: roms_gpu_halo_map for a `width`-deep exchange (2: the
 * reference's halo, as roms_gpu_halo_map; 2K: the fast loop's swap every K
 * fast steps, roms_gpu_halo_exchanges).  width <= Lm, Mm.                   */
long roms_gpu_halo_map_wide(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic,
                            int ns_periodic, int width, int dir, int unpack, int *i, int *j, long cap);

/* ---- forcing and boundary producers on the device (set_forces.F,
 * set_frc_data roms_read_write.F:303-392, set_bry_all boundary.F:227,
 * set_tides tides.F:86-254) ----
 * roms_gpu_frc_record uploads one record (time rec_time in days, like the
 * reference's forcing times) of a field into record slot 0, 1 or 2 (ABI 13:
 * a third slot); the host uploads a record only when the model time leaves
 * the window of those it holds (as fill_frc_slice does).  At a model time
 * modtime the pair (it1, it2) is the one set_frc_data would hold: the
 * earliest consecutive pair of the loaded records, in time order, whose
 * later time is >= modtime (the reference refreshes to (it2, next record)
 * once times(it2) < modtime, roms_read_write.F:341-350).  A modtime past
 * every loaded record fails with -8 before anything is queued (load the
 * next record first).  roms_gpu_frc_interp forms every field holding two or
 * more records, of the kinds in `kinds` (ROMS_FRC_SURFACE: 2-D
 * surface/atmospheric fields, ROMS_FRC_BRY: the *_west.._north boundary
 * arrays), as cff1*rec(it1) + cff2*rec(it2) at modtime [days], with
 * set_frc_data's out-of-window error (-1).  roms_gpu_set_tide_data hands over
 * the tidal constituents (frequencies ftide [1/s]; potential and boundary
 * elevation/velocity real/imaginary parts, ntides x the field layout,
 * column-major like the reference's (GLOBAL_2D_ARRAY, ntides) arrays; NULL
 * pairs switch that part off); roms_gpu_set_tides(time) then sets ptide
 * (pot_tides) and adds the tides to the open-boundary zeta/ubar/vbar data
 * (bry_tides) at omT = ftide*(time + dt/2), as set_tides_tile does.       */
#define ROMS_FRC_SURFACE 1
#define ROMS_FRC_BRY     2
int roms_gpu_frc_record(int field_id, int slot, double rec_time, const double *data);
int roms_gpu_frc_interp(double modtime, int kinds);
/* In-step forcing: with on = 1, every roms_gpu_step interpolates each field
 * that holds two records at the reference's own points of roms_step, with
 * time = start_time + dt*(iic - ntstart) [s] (main.F:373): surface fields at
 * frc_time 'current' before the first set_forces work (BULK_FRC flux), the
 * open-boundary data at '1/2 fwd' followed by set_tides, surface fields at
 * '1/2 fwd' before the second set_forces, boundary data at 'forward' (from
 * tdays = time + dt/2) followed by set_tides (main.F:384-441,
 * roms_read_write.F:330-336).  The weights are formed on the host per step
 * and read by the step graph from device memory; each of the four points
 * picks its own record pair, so with three records loaded a refresh that
 * falls inside a step (t2 between the '1/2 fwd' and 'forward' points) is
 * reproduced.  A step with any point past a field's last record fails with
 * -8, one outside the window (roms_read_write.F:381-388) with -1, both
 * before anything is queued; with boundary tides on, every open side's
 * zeta/ubar/vbar data must hold two records (set_bry_all re-sets them before
 * each set_tides).  on = 0: the host interpolates (roms_gpu_frc_interp).  */
int roms_gpu_frc_clock(double start_time, int on);
int roms_gpu_set_tide_data(int ntides, const double *ftide, const double *pot_re, const double *pot_im,
                           const double *ztide_re, const double *ztide_im, const double *utide_re,
                           const double *utide_im, const double *vtide_re, const double *vtide_im);
int roms_gpu_set_tides(double time);

/* ---- on-disk formats: partitioned netCDF restart and history files ----
 * One file per rank, as the reference's PARALLEL_FILES build writes them
 * (file name chosen by the host: roms_read_write.F:1389-1447 appends the date
 * and the rank), in the netCDF classic 64-bit-offset format (nf90_open reads
 * it like the reference's own netCDF-4 files), with the reference's
 * dimensions (xi_rho, xi_u, eta_rho, eta_v, s_rho, s_w, time, auxil),
 * variables, attributes and 'partition' global attribute.
 * roms_gpu_wrt_rst replaces wrt_restart_file (basic_output.F:568-682): it
 * writes record rec (1-based; rec 1 creates the file, def_vars_rst_ocean_vars
 * :873-1034) with ocean_time = time, time_step = (t->iic, rec, total_rec, 0,
 * 0, 0), zeta/ubar/vbar(knew), u/v/tracers(nnew), the EXACT_RESTART
 * DU/DV_avg1/avg2/avg_bak, hbls/hbbl (LMD) and riv_umask/riv_vmask.
 * roms_gpu_wrt_his replaces wrt_his_ocean_vars (:273-419) for the fields in
 * wrt_mask (ocean_vars.opt wrt_* switches).  Both snapshot the record on the
 * device, in stream order, and return; the PCIe copy and the file write run
 * behind the next steps.  roms_gpu_io_wait joins the pending write and
 * returns its status.  roms_gpu_get_init replaces get_init (get_init.F): see
 * rst_io.hip for the EXACT_RESTART protocol (call it with tindx 2 on record
 * rec-1, then tindx 1 on rec, then roms_gpu_init_sequence).  With LMD,
 * roms_gpu_swr_frac must have run once at rest (after roms_gpu_set_depth
 * on zeta = 0, main.F:216-220) before get_init; init_sequence fails
 * otherwise.  After a negative return of get_init the fields it had read
 * are already replaced: the model state is invalid until re-initialised.    */
#define ROMS_WRT_Z    1
#define ROMS_WRT_UB   2
#define ROMS_WRT_VB   4
#define ROMS_WRT_U    8
#define ROMS_WRT_V    16
#define ROMS_WRT_T    32     /* all tracers (tracers.opt wrt_t)              */
#define ROMS_WRT_R    64     /* rho1 (SPLIT_EOS) or rho                      */
#define ROMS_WRT_O    128    /* omega = pm*pn*(We+Wi), m/s (basic_output.F:374-384) */
#define ROMS_WRT_AKV  256
#define ROMS_WRT_AKT  512
#define ROMS_WRT_AKS  1024
#define ROMS_WRT_HBLS 2048
#define ROMS_WRT_HBBL 4096
#define ROMS_WRT_DEFAULT 63  /* ocean_vars.opt defaults: Z, Ub, Vb, U, V + tracers */
int roms_gpu_wrt_rst(const char *path, int rec, int total_rec, double time, const roms_tlev *t);
int roms_gpu_wrt_his(const char *path, int rec, int total_rec, double time, const roms_tlev *t, int wrt_mask);
int roms_gpu_io_wait(void);
/* t_vname/t_units/t_lname of tracer itrc (tracers.opt); default temp, salt, trcNN */
int roms_gpu_io_tracer_name(int itrc, const char *name, const char *units, const char *long_name);
/* Returns 0 (read), 1 (tindx 2: records not consecutive steps, nothing read),
 * or a negative error.                                                       */
int roms_gpu_get_init(const char *path, int req_rec, int tindx, roms_tlev *t, double *start_time);

/* ---- diagnostics (diag.F code_check norms, device reduction) ----
 * KE, KE2b (barotropic), max advective Courant and the vertical Courant at
 * that point, in the reference's reduction order.  The grid area/volume of
 * setup_grid2.F are formed on first use from the device's h, pm, pn, rmask
 * (per-rank pairwise sums, tree over ranks), so a host that registered its
 * own arrays gets the same norms as roms_gpu_init_case.  Collective.        */
int roms_gpu_diag(const roms_tlev *t, double norms[4]);
/* Host-only: set_weights.F restatement -- the fast-time averaging weights of
 * ndtfast (written into weight, C order [2][288]); returns nfast, or -1.    */
int roms_gpu_set_weights(int ndtfast, double weight[2][ROMS_MAX_FAST]);
/* event-timed replay of n steps on the library stream: total milliseconds  */
int roms_gpu_time_steps(roms_tlev *t, int n, double *ms);
/* Runs nsteps steps eagerly with HIP events on the library stream around
 * every launch of one routine; returns the mean duration of one launch
 * (one call of the routine, incl. its boundary/exchange kernels).            */
enum roms_routine {
  ROMS_R_RHO_EOS = 0, ROMS_R_SET_HUV, ROMS_R_OMEGA, ROMS_R_PRSGRD, ROMS_R_PRE_STEP3D, ROMS_R_SET_HUV1,
  ROMS_R_STEP3D_UV1, ROMS_R_VISC3D, ROMS_R_STEP2D, ROMS_R_STEP3D_UV2, ROMS_R_STEP3D_T, ROMS_R_T3DMIX,
  ROMS_R_LMD_VMIX,
  ROMS_R_K_S2D_FB,  /* kernel level: the fused barotropic kernel k_s2d_fb alone (one fast step) */
  ROMS_R_K_PRE_UV_SEG,     /* kernel level: pre_step3d's momentum segment solver (N > 63) */
  ROMS_R_K_UV1_SEG,        /* kernel level: step3d_uv1's momentum segment solver (N > 63) */
  ROMS_R_K_STEP3D_T_SEG,   /* kernel level: step3d_t's tracer segment solver (N > 63) */
  ROMS_R_K_PRSGRD_UV,      /* kernel level: prsgrd's ru/rv kernel (with the horizontal momentum r.h.s. in whole steps) */
  ROMS_R_K_HALO_PACK,      /* halo path: the pack of every exchange (IPC: straight into the neighbours' buffers) */
  ROMS_R_K_HALO_WAIT,      /* halo path: the transport (IPC: signal + arrival wait; RCCL: the send/recv group) */
  ROMS_R_K_HALO_UNPACK,    /* halo path: the unpack of every exchange */
  ROMS_R_COUNT
};
int roms_gpu_time_routine(int routine, int nsteps, roms_tlev *t, double *avg_ms, long *launches);

#ifdef __cplusplus
}
#endif
#endif /* ROMS_GPU_H */
