// roms_dev.h -- device-side state and index helpers of the MI355X ROMS hot path.
//
// Every array keeps the reference's Fortran layout (ocean_vars.F:68-116):
// horizontal extent (-1:Lm+2, -1:Mm+2), i fastest; rho-point 3-D arrays stack
// N levels (1:N), w-point arrays N+1 levels (0:N); u,v add 3 time levels,
// zeta/ubar/vbar 4, t(...,3,NT).  On the device a row j holds nx2 doubles:
// Lm+4 rounded up to kRowAlign (128 B), and every array's base is shifted by
// kAlignOff doubles, so element (i,j) sits at (i+1) + (j+1)*nx2 and i = 1 of
// every row and level starts a 128-B line: a wavefront of 64 consecutive i
// from i = 1 reads exactly four lines (at nx2 = Lm+4 the rows drift 32 B per
// row against the lines and most such runs touch five).  Host copies re-pitch
// the rows (roms_shim.cpp); no transpose anywhere.
//
// Wide fast-time halos (multi-rank, Bounds::gx > 0): every plane also holds
// gx extra ghost rows below j = -1 and above j = Mm+2, and every row gx extra
// ghost columns left of i = -1 and right of i = Lm+2.  The indexing above is
// unchanged: the plane stride n2 covers Mm+4+2gx rows, the base of every
// array sits gx rows into its allocation, and the columns i < -1 of row j are
// the last gx doubles of row j-1's pitch (nx2 >= Lm+4+2gx keeps them apart
// from that row's own columns).  Only the barotropic fast loop reads them
// (launch_step2d: 2+gx-wide exchanges every 1+gx/2 fast steps).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace roms {

constexpr int kMaxFast = 288;  // coupling.F:19, weight(2,288)
constexpr int kRowAlign = 16;  // device row pitch granule: 16 doubles = one 128-B line
constexpr int kAlignOff = 14;  // base shift: element i = 1 (index 2 of a row) on a line start

// Loop bounds of the single tile that covers one rank's subdomain
// (compute_tile_bounds.h, compute_auxiliary_bounds.h, compute_extended_bounds.h).
struct Bounds {
  int Lm, Mm, N, NT, nTS, nx2;   // nx2: device row pitch (>= Lm+4+2gx)
  long n2, n3, n3w;              // n2 = nx2 * (Mm+4+2gx): plane stride
  int gx;                        // extra ghost rows/columns beyond the reference's 2 (wide fast halos)
  int istr, iend, jstr, jend;
  int istrU, istrR, iendR, jstrV, jstrR, jendR;   // auxiliary
  int istrE, iendE, jstrE, jendE;                  // extended
  int west_edge, east_edge, south_edge, north_edge;  // physical (closed) edges
  int ew_periodic, ns_periodic;
  int west_exch, east_exch, south_exch, north_exch;  // message edges (rank neighbours)
};

// Physics switches (cppdefs.opt) and scalars of the run.
struct Params {
  int nonlin_eos, salinity, lmd, uv_vis2, ts_dif2;
  int lmd_rimix, lmd_convec, lmd_nonlocal;  // LMD_RIMIX, LMD_CONVEC, LMD_NONLOCAL (lmd != 0: MIXING+KPP+BKPP)
  int lmd_ddmix;                            // LMD_DDMIX (needs SALINITY)
  int iso;                                  // ADV_ISONEUTRAL (+SW_TRIADS, STABILIZE): k_iso.hip
  int uv_adv, uv_cor;                       // UV_ADV, UV_COR
  int tides;                                // TIDES pot_tides: ptide in prsgrd
  int bulk_frc;                             // BULK_FRC (k_bulk.hip; u* from sustr_r/svstr_r in lmd_kpp)
  int prs_split;                            // 1: two-kernel prsgrd (default), 0: k_prsgrd_fused (ROMS_GPU_PRSGRD_FUSED=1)
  int s2d_split;  // 1: step2d as separate zeta / momentum kernels (ROMS_GPU_S2D_SPLIT=1)
  int colseg;     // 1: segment-partitioned column solvers (k_colseg.h; N > 63, ROMS_GPU_COLSEG=0/1)
  int colreg;     // 1: register-resident column solvers where compiled for N (ROMS_GPU_COLREG=0 disables)
  int uv2_fused;  // 1: one-pass step3d_uv2 (k_uv2_fused; ROMS_GPU_UV2_FUSED=0 disables)
  int chain;      // 1: chained 4-lane set_HUV1 (k_chain.h; ROMS_GPU_CHAIN=0 disables)
  int seg_order;  // block order of the segment solvers (seg_tile; ROMS_GPU_SEG_ORDER)
  int seg_xg;     // x-blocks per group of seg_order 3 (ROMS_GPU_SEG_XG)
  int s2d_fold;   // closed-wall edges of the fast step inside k_s2d_fb (ROMS_GPU_S2D_EDGES=1: separate kernels)
  int hoist;        // per-level horizontal kernels with every global load at entry (ROMS_GPU_HOIST=0: per-phase forms)
  int chain_dirz;   // chain kernels (set_HUV1, uv2): one direction per block (ROMS_GPU_CHAIN_DIRZ=0: both in turn)
  int prs_fuse_uv;  // whole steps: horizontal momentum r.h.s. inside prsgrd (ROMS_GPU_PRS_UV=0: separate)
  int h_ty;       // tile rows of the hoisted horizontal kernels: 4 or 8 (ROMS_GPU_HTY)
  int h_jc;       // rows per block of the j-marching horizontal kernels (multiple of 4; ROMS_GPU_HJC, 0: 64 x h_ty tiles)
  int prs_ty;     // tile rows of k_prsgrd_uv: 4 or 8 (ROMS_GPU_PRS_TY)
  int ld16;       // padded pitch: LDS windows read two doubles per lane (16-B loads; ROMS_GPU_LD16=0: 8-B)
  int prs_buf;    // k_prsgrd_uv windows through buffer loads (ROMS_GPU_PRS_BUF)
  int prs_strip;  // prsgrd + momentum r.h.s. in j-marching strips (k_prsgrd_strip; ROMS_GPU_PRS_STRIP=0: tiles)
  int t_strip;    // horizontal tracer advection in j-marching strips (k_tracer_strip; ROMS_GPU_T_STRIP=0: tiles)
  int visc_stg;   // visc3d: raw u/v/Hz windows staged in LDS per level (default; ROMS_GPU_VISC_STG=0: per-point loads)
  int t3dmix_stg; // t3dmix (two tracers): Hz/T/S windows staged in LDS per level (default; ROMS_GPU_T3DMIX_STG=0: per-point loads)
  int kpp_ty;     // k_kpp_int: 4 (default) staged Rig windows on 64x4 blocks, 8 on 64x8, 43 64x4 at 3 waves/SIMD, 0 one row per block (ROMS_GPU_KPP_TY)
  int tile_grp;   // h_tile group width of the hoisted per-level kernels (ROMS_GPU_TILE_GRP; 0: xcd_tile order)
  int uv1_lds;    // k_uv1_seg: Hz pairs kept in LDS from the spline phase, rufrc chained (ROMS_GPU_UV1_LDS=0: reloads)
  int omega_seg;  // omega: segment form k_omega_seg, one read of each input (ROMS_GPU_OMEGA_SEG=0: two-pass k_omega)
  int omega_cw;   // k_omega_seg columns per block: 64, 32 or 16 (ROMS_GPU_OMEGA_CW)
  int omega_ord;  // k_omega_seg block order: 0 xcd_tile, 1..3 seg_tile's orders (ROMS_GPU_OMEGA_ORD)
  int omega_par;  // k_omega_seg: segment partial sums in parallel, one barrier (ROMS_GPU_OMEGA_PAR; not bitwise to the k-order chain)
  int p_in_rho;   // rho_eos's sweep also forms prsgrd's P (ROMS_GPU_P_IN_RHO=0: k_prsgrd_P)
  int omega_hb;   // the predictor's omega forms pre_step3d's Hz_bak/Hz_fwd (ROMS_GPU_OMEGA_HB=0: pre_step3d does)
  int preuv_lds;  // k_pre_uv_seg: u(indx) stored and u(nstp)/u(indx) combined in the spline phase (ROMS_GPU_PREUV_LDS=0: reloads)
  int seg_jrows;  // rows j per block of the momentum segment solvers (1..kSegJMax; ROMS_GPU_SEG_JROWS)
  int t_chunk;    // tracer horizontal part + column solve alternating over strips of t_chunk rows (ROMS_GPU_TCHUNK; 0: off)
  int seg_buf;    // segment solvers with buffer loads, wave-uniform level offsets (ROMS_GPU_SEG_BUF bits)
  int seg_vtile;  // v columns of the momentum segment solvers on 16 x 4 tiles per wavefront (ROMS_GPU_SEG_VTILE=0: rows of 64)
  int s2d_k;      // fast steps per zeta/ubar/vbar exchange (multi-rank, wide halos of 2*s2d_k; 1: every step)
  int uv2e_nc, uv2e_nf;   // lengths of Fields::uv2e_couple / uv2e_flux
  int npip;       // pipe_frc.F: number of pipes (0: pipe_source off)
  int nriv, nrivf;  // river_frc.F: number of rivers (0: river_source off), river faces
  int curvgrid;   // CURVGRID && UV_ADV: curvature terms (compute_horiz_rhs_uv_terms.h:8-11)
  int obc;        // open edges: 1 W, 2 E, 4 S, 8 N (Flather / Orlanski + *_FRC_BRY)
  double ubind;   // OBC binding velocity
  double dt, dtfast, g, rho0, vonKar, qp2, gamma2, hc;
  double rdrg, Zob, Tcoef, T0, Scoef, S0;
  double Akv_bak, Akt_bak[2];  // scalars.F:83
};

// Device pointers of the model state (the "module arrays") plus scratch.
struct Fields {
  // grid (grid.F)
  double *h, *hinv, *f, *fomn, *pm, *pn, *dm_r, *dn_r, *dm_u, *dn_u, *dm_v, *dn_v, *dm_p, *dn_p,
      *pmon_u, *pnom_v, *rmask, *pmask, *umask, *vmask;
  double *dndx, *dmde;  // CURVGRID metric derivatives
  double* ptide;        // tides.F surface tidal potential (TIDES)
  // BULK_FRC inputs (rho points) and rho-point stresses (bulk_frc.F, surf_flux.F)
  double *uwnd, *vwnd, *tair, *qair, *prate, *swrad, *lwrad, *sustr_r, *svstr_r;
  double *Cs_w, *Cs_r;  // scoord.F (N+1)
  // ocean vars
  double *zeta, *ubar, *vbar, *u, *v, *t;
  double *FlxU, *FlxV, *We, *Wi, *Hz, *Hz_u, *Hz_v, *z_r, *z_w;
  // coupling.F
  double *rufrc, *rvfrc, *rhoA, *rhoS, *r_D, *Zt_avg1, *DU_avg1, *DV_avg1, *DU_avg2, *DV_avg2,
      *DU_avg_bak, *DV_avg_bak;
  // eos_vars.F / mixing.F
  double *rho, *rho1, *qp1, *bvf, *Akv, *Akt, *visc2_r, *visc2_p, *diff2;
  double *hbls, *hbbl, *ghat, *swr_frac;
  // surf_flux.F
  double *sustr, *svstr, *stflx, *srflx, *swflx;
  // private scratch: A3d(:,1..4) and per-column work arrays
  double *ru, *rv, *P, *rhos;
  double *c0, *c1, *c2, *c3;   // (0:N) column scratch, w-point layout
  double *s0, *s1, *s2, *s3, *s4, *s5, *s6, *s7, *s8, *s9;  // 2-D scratch (step2d, diag)
  // lmd_vmix / lmd_kpp private work arrays: raw Richardson number (0:N) and
  // the 2-D boundary-layer fields carried from the extended-range pass
  double *lmd_rig, *lmd_hbl, *lmd_bbl, *lmd_Bo, *lmd_Bosol, *lmd_ustar;
  // pipe_frc.F: pipe_idx (0: none), pipe_flx, pipe_prf(npip,N), pipe_trc(npip,NT)
  int* pipe_idx;
  double *pipe_flx, *pipe_prf, *pipe_trc;
  // river_frc.F: riv_uflx/riv_vflx (10*iriver + signed fraction on river
  // faces), riv_vol(nriv), riv_trc(nriv,NT); riv_face: (dir, i, j) of every
  // face with |riv_flx| > 1e-3, three ints per face (Params::nrivf of them)
  double *riv_uflx, *riv_vflx, *riv_vol, *riv_trc;
  int* riv_face;
  // step3d_uv2's closed-edge columns (uv2_edge_lists): (dir, i, j) triples of
  // the couple and the flux pass (Params::uv2e_nc / uv2e_nf of them; nullptr: the one-lane edge mode)
  int *uv2e_couple, *uv2e_flux;
  // boundary.F open-boundary data, [0] west, [1] east (index j, 0:Mm+1),
  // [2] south, [3] north (index i, 0:Lm+1); u, v (.,N); t (.,N,NT)
  double *bzeta[4], *bubar[4], *bvbar[4], *bu[4], *bv[4], *bt[4];
  double* ub[4];   // SPONGE_TUNE ub_west/east/south/north (sponge_tune.F; nullptr: ub_tune off)
  // column-solver scratch in global memory, 2*max(NT,2) slots of (0:N) levels
  // (nullptr: the solvers keep their columns in LDS; see ColGlb in k_common.h)
  double* colscr;
  // ADV_ISONEUTRAL (k_iso.hip; nullptr when off): eos_vars.F:28-31 dRdx, dRde
  // (N) and idRz (0:N), mixing.F:24-27 diff3u, diff3v (N), step3d_t's Akz
  // (0:N), and the operator's 3-D work fields dTdz, FSC (0:N), dTdx, dTde, LapT (N)
  double *dRdx, *dRde, *idRz, *diff3u, *diff3v, *Akz;
  double *iso_dTdz, *iso_FSC, *iso_dTdx, *iso_dTde, *iso_LapT;
};

// The fast step's 2-D fields addressed from one buffer window (k_s2d_fb):
// one descriptor plus a 32-bit byte offset per field in place of a 64-bit
// base each -- the fused fast step reads and writes 25 of them, and their
// bases alone held more scalar registers than the kernel has.  roms_gpu_init
// allocates these fields next to each other and fills the window when they
// span less than 2 GiB (base = nullptr: the pointer form).
enum S2dWinField : int {
  kW_zeta, kW_ubar, kW_vbar, kW_h, kW_dn_u, kW_dm_v, kW_pm, kW_pn, kW_swflx, kW_rmask, kW_rhoS, kW_rhoA, kW_umask,
  kW_vmask, kW_rufrc, kW_rvfrc, kW_DU_avg1, kW_DV_avg1, kW_DU_avg2, kW_DV_avg2, kW_Zt_avg1, kW_DU_avg_bak,
  kW_DV_avg_bak, kW_s0, kW_s1, kWinN
};
struct S2dWin {
  const double* base;   // nullptr: no window
  int lead;             // element (i,j) of a field sits (IJ + lead) doubles past its window origin
  unsigned off[kWinN];  // byte offset of each field's origin (its element IJ = -lead) from base
};

struct Halo;  // halo.h: multi-rank exchange state (host object; nullptr = single rank)
struct Dev {
  Bounds b;
  Params p;
  Fields f;
  const Halo* halo;
  S2dWin w2;
};

// ---- index helpers (device + host) ----
__host__ __device__ __forceinline__ long IJ(const Bounds& b, int i, int j) {
  return (long)(i + 1) + (long)(j + 1) * b.nx2;
}
__host__ __device__ __forceinline__ long IJK(const Bounds& b, int i, int j, int k) {  // 1:N
  return IJ(b, i, j) + (long)(k - 1) * b.n2;
}
__host__ __device__ __forceinline__ long IJW(const Bounds& b, int i, int j, int k) {  // 0:N
  return IJ(b, i, j) + (long)k * b.n2;
}
__host__ __device__ __forceinline__ long IJL(const Bounds& b, int i, int j, int l) {  // (:,:,4)
  return IJ(b, i, j) + (long)(l - 1) * b.n2;
}
__host__ __device__ __forceinline__ long IJKL(const Bounds& b, int i, int j, int k, int l) {  // (:,:,N,3)
  return IJ(b, i, j) + (long)(k - 1) * b.n2 + (long)(l - 1) * b.n3;
}
__host__ __device__ __forceinline__ long TIDX(const Bounds& b, int i, int j, int k, int l, int itrc) {
  return IJKL(b, i, j, k, l) + (long)(itrc - 1) * 3 * b.n3;
}

__device__ __forceinline__ double fmax0(double a) { return a > 0.0 ? a : 0.0; }
__device__ __forceinline__ double fmin0(double a) { return a < 0.0 ? a : 0.0; }
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ int iclamp(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

// XCD-aware tile order.  Workgroups are dealt round-robin to the 8 XCDs
// (MI355X_MICROARCH.md: blocks b and b+8 share an XCD and its L2), so with
// the plain grid order the four neighbours of a tile live in other XCDs' L2s
// and every halo row is fetched from HBM twice.  xcd_tile() maps the
// physical block id to a logical tile so that each XCD walks one contiguous
// 1/8 of the (x fastest, then y, then z) tile sequence: neighbouring tiles of
// a level are processed by the same XCD at about the same time.
__device__ __forceinline__ uint3 xcd_tile() {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned total = gx * gy * gridDim.z;
  const unsigned phys = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned q = total >> 3, r = total & 7u, x = phys & 7u, slot = phys >> 3;
  const unsigned logical = x * q + (x < r ? x : r) + slot;
  uint3 t;
  t.x = logical % gx;
  t.y = (logical / gx) % gy;
  t.z = logical / (gx * gy);
  return t;
}

// Per-level horizontal kernels with halo windows: xcd_tile()'s sequence
// re-ordered within each level (z) so that y runs fastest inside groups of
// grp x-tiles (grp <= 0: plain xcd_tile order).  The tiles resident on one
// XCD then cover a grp-wide strip of consecutive rows, whose shared halo
// rows (j-neighbours) and halo lines (i-neighbours inside the group) are
// fetched by neighbours close together in time.
__device__ __forceinline__ uint3 h_tile(int grp) {
  uint3 t = xcd_tile();
  if (grp <= 0) return t;
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned L = t.x + gx * t.y;
  const unsigned G = (unsigned)grp < gx ? (unsigned)grp : gx;
  const unsigned nfull = gx / G, inf = nfull * G * gy;
  if (L < inf) {
    const unsigned rem = L % (G * gy);
    t.x = (L / (G * gy)) * G + rem % G;
    t.y = rem / G;
  } else {
    const unsigned Gl = gx - nfull * G, rem = L - inf;
    t.x = nfull * G + rem % Gl;
    t.y = rem / Gl;
  }
  return t;
}

// Compiler fence between the levels of a fully unrolled column walk: memory
// operations are not moved across it, so the scheduler cannot hoist the loads
// of all N levels to the top (which would need N x (loads per level)
// registers and spill); a few levels of look-ahead remain within a chunk.
#define ROMS_LEVEL_FENCE() __asm__ volatile("" ::: "memory")
#ifndef ROMS_FENCE_EVERY
#define ROMS_FENCE_EVERY 1000
#endif
#define ROMS_LEVEL_FENCE_AT(k) do { if ((k) % ROMS_FENCE_EVERY == 0) ROMS_LEVEL_FENCE(); } while (0)

// 2-D launch over an inclusive index rectangle [i0,i1]x[j0,j1]: one lane per
// (i,j) column, 64 consecutive i per wavefront (coalesced), 4 rows per block.
struct Range {
  int i0, i1, j0, j1;
};
constexpr int kBX = 64, kBY = 4;
// First tile column of a launch over [i0, i1]: i0 rounded down to a line
// start of the device rows (i = 1 mod kRowAlign, roms_dev.h layout), so the
// wavefront rows of every tile read whole 128-B lines; the lanes left of i0
// in the first tile idle.  (Ranges from istrR/istrE = 0 or -1, istrU = 2 and
// the multi-rank rim strips all start off a line.)
#ifndef ROMS_TILE_ALIGN
#define ROMS_TILE_ALIGN 1   // 0: tiles start at the range's first column (A/B builds, tools/build_variant.sh)
#endif
__host__ __device__ __forceinline__ int tile_i0(int i0) { return ROMS_TILE_ALIGN ? i0 - ((i0 - 1) & (kRowAlign - 1)) : i0; }
inline dim3 grid_of(const Range& r) {
  int ni = r.i1 - tile_i0(r.i0) + 1, nj = r.j1 - r.j0 + 1;
  if (ni < 1) ni = 1;
  if (nj < 1) nj = 1;
  return dim3((ni + kBX - 1) / kBX, (nj + kBY - 1) / kBY, 1);
}
// 3-D launch: same (i,j) tiling with one grid z-slice per level k=1..nk
inline dim3 grid3_of(const Range& r, int nk) {
  dim3 g = grid_of(r);
  g.z = nk;
  return g;
}
// Column launch: one wavefront of 64 consecutive i per block, one row j per
// block row; column scratch lives in LDS (see ColLds in k_common.h).
constexpr int kCX = 64;
// segment-partitioned column solvers (k_colseg.h)
#ifndef ROMS_SEG_ROWS
#define ROMS_SEG_ROWS 13
#endif
#ifndef ROMS_SEG_MAXS
#define ROMS_SEG_MAXS 8
#endif
constexpr int kSegRows = ROMS_SEG_ROWS;   // cells per segment (register arrays of kSegRows + 2)
constexpr int kSegMaxS = ROMS_SEG_MAXS;   // segments per block (kSegCW columns each): N <= kSegRows * kSegMaxS
#ifndef ROMS_SEG_CW
// round 5: 16-column blocks (four segments per wavefront, 128-thread
// blocks, four per CU): against 64 columns pre_step3d 11.1 -> 9.9 ms,
// step3d_uv1 4.55 -> 3.93 ms at C3 (r5_q_seg_cw32_default_ab.txt,
// r5_s_seg_cw16_ab.txt); round 3 had measured 64 ahead of 16
// (r3_l_seg_shape_ab.txt, before the solvers kept their reloads in LDS)
#define ROMS_SEG_CW 16
#endif
constexpr int kSegCW = ROMS_SEG_CW;       // columns per segment-solver block (lanes of one segment)
constexpr int kSegBlock = ((kSegMaxS * kSegCW + 63) / 64) * 64;   // threads of a segment-solver block (max)
// The momentum solvers' blocks may hold several rows j (blockDim.z) of the
// same kSegCW columns, so the v columns' j-1, j-2, j+1 stencil rows are loaded
// by the neighbouring rows' waves of the same block, close together in time.
#ifndef ROMS_SEG_JMAX
#define ROMS_SEG_JMAX 1
#endif
constexpr int kSegJMax = ROMS_SEG_JMAX;
// the fewest rows any segment of a launch may have (k_colseg.h seg_live)
#ifndef ROMS_SEG_NMIN
#define ROMS_SEG_NMIN 11   // 0: every row select kept (the round-4 code; A/B builds)
#endif
constexpr int kSegNMin = ROMS_SEG_NMIN;
// waves per SIMD the buffer-addressed segment solvers are built for (2: one
// 512-thread block per CU at <= 256 VGPRs; 4: two blocks at <= 128)
#ifndef ROMS_SEG_BUF_WAVES
#define ROMS_SEG_BUF_WAVES 2
#endif
#ifndef ROMS_PRE_T_SEG_WAVES   // k_pre_tracer_segb alone (A/B builds)
#define ROMS_PRE_T_SEG_WAVES ROMS_SEG_BUF_WAVES
#endif
#ifndef ROMS_T_SEG_WAVES       // k_step3d_t_segb alone (A/B builds)
#define ROMS_T_SEG_WAVES ROMS_SEG_BUF_WAVES
#endif
// segments of an N-level column (one per wavefront at kSegCW = 64, seg_waves)
// and whether each of them gets at least kSegNMin rows
inline int seg_count(int N) {
  const int per = kCX / kSegCW, S = (N + kSegRows - 1) / kSegRows;
  return (S + per - 1) / per * per;
}
inline bool seg_rows_ok(int N) { return N / seg_count(N) >= kSegNMin; }
inline dim3 gridc_of(const Range& r) {
  int ni = r.i1 - tile_i0(r.i0) + 1, nj = r.j1 - r.j0 + 1;
  if (ni < 1) ni = 1;
  if (nj < 1) nj = 1;
  return dim3((ni + kCX - 1) / kCX, nj, 1);
}
#define ROMS_IJC_OR_RETURN(R)                                       \
  const uint3 bI = xcd_tile();                                      \
  const int i = tile_i0((R).i0) + (int)(bI.x * kCX + threadIdx.x);  \
  const int j = (R).j0 + (int)bI.y;                                 \
  if (i < (R).i0 || i > (R).i1 || j > (R).j1) return;
#define ROMS_IJ_OR_RETURN(R)                                        \
  const uint3 bI = xcd_tile();                                      \
  const int i = tile_i0((R).i0) + (int)(bI.x * kBX + threadIdx.x); \
  const int j = (R).j0 + (int)(bI.y * kBY + threadIdx.y);           \
  if (i < (R).i0 || i > (R).i1 || j > (R).j1) return;

// ---- launcher declarations (one translation unit per routine family) ----
// Each takes the rank's device state and a stream; all enqueue asynchronously.
struct Tlev {
  int iic, ntstart, forw_start, iif, nfast, kstp, knew, nstp, nrhs, nnew;
};

// kernel-level timing hook (roms_gpu_time_routine with a kernel id): HIP
// events on the launch stream opening (end = 0) and closing (end = 1) an
// interval that covers `count` launches of one kernel
constexpr int kTimedS2dFb = 13;   // ROMS_R_K_S2D_FB
constexpr int kTimedPreUvSeg = 14, kTimedUv1Seg = 15, kTimedStep3dTSeg = 16;   // ROMS_R_K_*_SEG
constexpr int kTimedPrsgrdUv = 17;   // ROMS_R_K_PRSGRD_UV
constexpr int kTimedHaloPack = 18, kTimedHaloWait = 19, kTimedHaloUnpack = 20;   // ROMS_R_K_HALO_*
void ktimer_mark(hipStream_t s, int kernel_id, int end, int count = 0);

// The buffer-addressed kernels (BufF64, k_common.h) address one field with
// 32-bit byte offsets that must stay below 2 GiB (kBufOff = 2^31 marks a lane
// whose access the hardware drops): every field -- the largest is a w-point
// field, n2*(N+1) doubles on the padded pitch -- must fit.  roms_gpu_init
// refuses a subdomain that does not (1024^2 x 100 uses 0.85 GiB).
inline bool buffer_span_ok(const Bounds& b) { return b.n3w * 8 < 2147483648L; }

void launch_exchange(const Dev& d, hipStream_t s, double* a, int nlev);
// several arrays in one launch (one reference exchange_xxx(A,B,C,D) call);
// w > 2: a wide exchange (halo w deep, Bounds::gx >= w-2; the fast loop's)
constexpr int kExchMax = 16;
struct ExchList {
  double* p[kExchMax];
  int nlev[kExchMax];
  int n;
  int w = 2;
};
void launch_exchange_list(const Dev& d, hipStream_t s, const ExchList& L);
// ---- rim-first overlap of a producer's trailing exchange (SURVEY.md 8(e);
// mpi_exchanges.F's swaps overlapped with interior compute).  `run(R')`
// launches the producer's kernels on a sub-range.  On a multi-rank run the
// four rim strips (the two rows / columns next to each edge: every cell the
// exchange packs) go first, then `edges()` (kernels that fill ghost cells
// from the rim; they travel with the strips), then the exchange of L is
// forked onto the halo stream while the interior runs on s, and s joins it
// before the next routine.  Single rank / overlap off: run(R), edges(),
// exchange.  Opt-in (ROMS_GPU_OVERLAP3D=1), see halo_setup. ----
bool rim_overlap_on(const Dev& d, const Range& R);
void rim_fork(const Dev& d, hipStream_t s, const ExchList& L);
void rim_join(const Dev& d, hipStream_t s);
template <class Run, class Edges>
void launch_rim_first(const Dev& d, hipStream_t s, const Range& R, const ExchList& L, Run&& run, Edges&& edges) {
  if (!rim_overlap_on(d, R)) {
    run(R);
    edges();
    launch_exchange_list(d, s, L);
    return;
  }
  run(Range{R.i0, R.i0 + 1, R.j0, R.j1});
  run(Range{R.i1 - 1, R.i1, R.j0, R.j1});
  run(Range{R.i0 + 2, R.i1 - 2, R.j0, R.j0 + 1});
  run(Range{R.i0 + 2, R.i1 - 2, R.j1 - 1, R.j1});
  edges();
  rim_fork(d, s, L);
  run(Range{R.i0 + 2, R.i1 - 2, R.j0 + 2, R.j1 - 2});
  rim_join(d, s);
}
// the tracer list t(:,:,:,tlev,1:NT) as one exchange list (false if NT > 8)
bool tracer_exch_list(const Dev& d, int tlev, ExchList& L);
void launch_exchange_tracers(const Dev& d, hipStream_t s, int tlev);  // t(:,:,:,tlev,1:NT)
// Column kernels keep 2 (N+1)-level scratch columns per lane in LDS; opt in to
// the full 160 KB when N needs more than the default 64 KB.  Returns false if
// N is too deep for one wavefront's columns to fit.
bool setup_column_kernels(int N);
void setup_uv1_seg();      // k_uv1_seg's dynamic LDS limit (k_step3d_uv.hip)
void setup_pre_uv_seg();   // k_pre_uv_seg<true>'s dynamic LDS limit (k_pre_step3d.hip)
inline size_t col_smem_bytes(const Dev& d, int nslots) {
  return d.f.colscr ? 0 : (size_t)nslots * (d.b.N + 1) * 64 * sizeof(double);
}
// exchange = false: the caller exchanges z_w, z_r, Hz itself (merged with its own list);
// last: end of the fast loop, zeta(knew) = Zt_avg1 stored first (step2d_FB.F:566)
void launch_set_depth(const Dev& d, hipStream_t s, const Tlev& t, bool exchange = true, bool last = false);
// store_huv: also Hz_u/Hz_v (set_depth.F:220,227), read only by extract_data.F
void launch_set_huv(const Dev& d, hipStream_t s, const Tlev& t, bool store_huv = true);
void launch_set_huv1(const Dev& d, hipStream_t s, const Tlev& t);
// hcff > 0: the predictor's call also forms pre_step3d's Hz_bak/Hz_fwd (c3/c2) of the
// interior cells with 0.5*dtau = hcff; returns whether it did (k_vertical.hip)
bool launch_omega(const Dev& d, hipStream_t s, const Tlev& t, double hcff = 0.0);
void setup_omega_seg();   // k_omega_seg<true>'s dynamic LDS limit
double pre_step3d_dtau(const Dev& d, const Tlev& t);   // pre_step3d's dtau (k_pre_step3d.hip)
void launch_rho_eos(const Dev& d, hipStream_t s, const Tlev& t, int tidx);
// uv_up >= 0: also add the horizontal momentum r.h.s. (UPSTREAM_UV if 1) of
// the following pre_step3d / step3d_uv1 (prsgrd_can_fuse_uv; the caller then
// passes uv_done to it)
// p_ready: P is current from the last rho_eos (p_in_rho), k_prsgrd_P is skipped
void launch_prsgrd(const Dev& d, hipStream_t s, const Tlev& t, int uv_up = -1, bool p_ready = false);
// k_tracer_strip.hip: rows jA..jB of R's horizontal tracer advection in
// j-marching strips (mode 0 step3d_t, 1 pre_step3d); false: not covered
bool launch_tracer_strip(const Dev& d, hipStream_t s, const Range& R, int mode, bool up, bool hb_done, int nnew,
                         int nrhs, double dtau, double cf_stp, double cf_bak, int nstp, int& jA, int& jB);
bool p_in_rho(const Dev& d);   // every rho_eos also forms prsgrd's P (k_vertical.hip)
void launch_prsgrd_P(const Dev& d, hipStream_t s);   // prsgrd's P alone (k_prsgrd_P)
bool prsgrd_can_fuse_uv(const Dev& d);
// A second stream for work with no data dependence on the main stream's
// (enqueue_step, single rank): the callee forks `s2` off `s` with `efork`
// and joins it back with `ejoin` before returning.
struct Side {
  hipStream_t s2;
  hipEvent_t efork, ejoin;
};
// hb_done: the interior cells' Hz_bak/Hz_fwd are in c3/c2 already (launch_omega)
// side: the tracer solves (and their boundary conditions and exchange) run on
// side->s2 beside the momentum ones
void launch_pre_step3d(const Dev& d, hipStream_t s, const Tlev& t, bool uv_done = false, bool hb_done = false,
                       const Side* side = nullptr);
void launch_step3d_uv1(const Dev& d, hipStream_t s, const Tlev& t, bool uv_done = false);
void launch_visc3d(const Dev& d, hipStream_t s, const Tlev& t);
void launch_step2d(const Dev& d, hipStream_t s, const Tlev& t, const double* w1, const double* w2);
void launch_step3d_uv2(const Dev& d, hipStream_t s, const Tlev& t);
// exchange = false: skip the closing t(nnew) exchange (whole steps with
// TS_DIF2: t3dmix reads only t(nrhs) and its own cells of t(nnew), and its
// own exchange of t(nnew) follows; the closed-wall ghosts are still set here)
void launch_step3d_t(const Dev& d, hipStream_t s, const Tlev& t, bool exchange = true);
void launch_t3dmix(const Dev& d, hipStream_t s, const Tlev& t);
void launch_u3dbc(const Dev& d, hipStream_t s, const Tlev& t);
// river_frc.F hooks (k_river.hip): ubar/vbar(knew) and DU/DV_avg1 at river
// faces after each fast step; u,v(nnew) at river faces (pred: predictor ranges)
void launch_river_s2d(const Dev& d, hipStream_t s, int knew);
// BULK_FRC: calc_all_bulk_forces (k_bulk.hip)
void launch_bulk_flux(const Dev& d, hipStream_t s, int nrhs);
void launch_river_uv(const Dev& d, hipStream_t s, int nnew, int pred);
void launch_v3dbc(const Dev& d, hipStream_t s, const Tlev& t);
void launch_t3dbc(const Dev& d, hipStream_t s, const Tlev& t, int itrc);
// out (device, 6 doubles): avzeta, KE, KE2b sums, Cu_adv, Cu_w, blow-up flag
void launch_diag(const Dev& d, hipStream_t s, const Tlev& t, double* out);
void launch_swr_frac(const Dev& d, hipStream_t s);
void launch_lmd_vmix(const Dev& d, hipStream_t s, const Tlev& t, int tind);
// ADV_ISONEUTRAL (k_iso.hip): prsgrd's corrector slopes (+ their exchange),
// step3d_uv2's diff3u/diff3v/idRz over its flux-correction ranges and their
// exchange, and step3d_t's rotated biharmonic operator for one tracer
void launch_iso_slopes(const Dev& d, hipStream_t s);
void launch_iso_diff3(const Dev& d, hipStream_t s, const Tlev& t, int iu0, int iu1, int iv0, int iv1, int j0, int j1);
void launch_iso_exch_diff3(const Dev& d, hipStream_t s);
void launch_iso_tracer(const Dev& d, hipStream_t s, const Tlev& t, int itrc);

}  // namespace roms
