// roms_shim.cpp -- C-ABI implementation (include/roms_gpu.h): device state
// registry, host<->device transfers, per-routine entries mirroring the
// reference's hot-path subroutines, the roms_step driver (main.F:333-520)
// with per-phase HIP-graph replay, analytic-case setup and diag norms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/roms_gpu.h"
#include "halo.h"
#include "host_init.h"
#include "roms_dev.h"
#include "shim_state.h"

using namespace roms;

namespace {

struct FieldDesc {
  double* d = nullptr;
  long count = 0;        // elements in the device layout (rows nx2 apart)
  long hcount = 0;       // elements in the host (reference) layout: what the ABI exchanges
  bool planar = false;   // (i,j)-planes of the horizontal grid (rows to re-pitch); Cs_*/boundary arrays not
  double* host = nullptr;
  long host_count = 0;
};

struct Ctx {
  bool inited = false;
  Dev d{};
  hipStream_t s = nullptr;
  FieldDesc f[ROMS_NFIELDS];
  std::vector<double*> scratch;
  roms_dims dims{};
  roms_cfg cfg{};
  double w1[kMaxFast], w2[kMaxFast];
  double area = 0.0, volume = 0.0;
  bool have_volume = false;   // area/volume formed (init_case, or on first diag)
  long riv_maxidx = 0;        // largest river index nint(riv_flx/10) of the faces on the device
  bool have_swr = false;      // swr_frac formed (at rest, main.F:216-220)
  long graph_frc_gen = 0;     // frc_step_gen() the step graphs were captured with
  // rho_eos reuse: the T slot whose rho1/qp1/bvf/rhoA/rhoS are current because
  // the last thing done to the model was a step, which ended with
  // rho_eos(nnew) (main.F:479).  The next step's opening rho_eos(nrhs)
  // (main.F:397) reads the same t(nstp), z_r, Hz, z_w (set_depth ran in the
  // last fast step, step2d_FB.F:569) and would rewrite the same values, so it
  // is skipped.  Every entry that may change the state clears it
  // (REQUIRE_INIT); the read-only ones keep it (REQUIRE_INIT_RO).
  int rho_slot = 0;
  // Hz_u/Hz_v (set_HUV's cell heights at u/v points) are read by no kernel of
  // the step, only by the reference's extract_data.F:726: whole steps store
  // them when the host registered either for transfer or set
  // ROMS_GPU_HZ_UV=1; otherwise they go stale and reading them fails
  bool hzuv_env = false;
  bool hzuv_valid = true;
  bool rho_reuse = true;      // ROMS_GPU_RHO_REUSE=0 turns the skip off
  std::string err;
  // graph cache: key = (nstp, knew at step start)
  std::map<long, hipGraphExec_t> graphs;
  bool use_graphs = true;
  double* h_diag = nullptr;   // pinned: the diag numbers
  double* d_diag = nullptr;   // device: the diag numbers (launch_diag)
  Halo halo;               // multi-rank exchange (halo.comm == nullptr: single rank)
  // per-routine timing (roms_gpu_time_routine): events around every launch
  int timed = -1;
  std::vector<hipEvent_t> ev;
  size_t nev = 0;
  long kcount = 0;   // kernel-level timing: launches covered by the intervals
  // ROMS_GPU_GUARD=1 (debug): every field and init-time scratch array gets
  // NaN-filled guard bands before and after it, so an out-of-bounds read
  // turns into NaN instead of a value of whatever array lies next to it
  bool guard = false;
  std::map<double*, double*> guard_base;   // array -> its allocation (nullptr: inside the 2-D arena)
  // The 2-D fields and 2-D scratch come from one allocation (roms_gpu_init),
  // so the fast step's fields always share one buffer window (S2dWin)
  double* arena = nullptr;
  long arena_n = 0, arena_used = 0;   // doubles
  double* small = nullptr;   // shim_scratch_small
  long small_n = 0;
  // Device row pitch (roms_dev.h): rows of nx2 = Lm+4 rounded up to 16
  // doubles (128 B), every array's base shifted by kAlignOff so that i = 1 of
  // every row starts a 128-B line.  Host copies re-pitch rows through a
  // device staging buffer (ROMS_GPU_PITCH=0: the host layout on the device).
  long off = 0;
  Bounds hb{};               // the host layout's Bounds (nx2 = Lm+4)
  double* stage = nullptr;
  long stage_n = 0;
  // Routines with no data dependence between them run on two streams inside
  // the step (single rank; opt-in, ROMS_GPU_PAR=1): see enqueue_step
  int par = 0;               // two-stream pair mask (enqueue_step)
  long step_exch = 0;        // halo exchanges in the last enqueued step (roms_gpu_halo_exchanges)
  hipStream_t s2 = nullptr;
  hipEvent_t pev[8] = {};
};
// One context per host thread: a process normally drives one GPU/subdomain
// from one thread; tests drive several subdomains from threads of one process.
thread_local Ctx g;

// reference tree reduction over ranks (diag.F:488-535): receiver r adds r+step
double tree_sum(std::vector<double> v) {
  int size = (int)v.size();
  while (size > 1) {
    const int step = (size + 1) / 2;
    for (int r = 0; r < size - step; r++) v[r] = v[r] + v[r + step];
    size = step;
  }
  return v.empty() ? 0.0 : v[0];
}
// local sub-domain extent along one direction (mpi_setup.F:110-154)
void rank_extent(int LL, int np, int node, int& len, int& sw) {
  const int base = (LL + np - 1) / np, off = np * base - LL;
  sw = node == 0 ? 0 : node * base - off / 2;
  len = base;
  if (node == 0) len -= off / 2;
  if (node == np - 1) len -= (off + 1) / 2;
}
// the smallest subdomain extent of any rank along one direction: the edge
// ranks lose the uneven-split remainder (mpi_setup.F:115-125), the interior
// ones keep the base width (LL/np is not a lower bound)
int min_rank_extent(int LL, int np) {
  int mn = LL, len, sw;
  for (int node : {0, np - 1}) {
    rank_extent(LL, np, node, len, sw);
    mn = len < mn ? len : mn;
  }
  if (np > 2) {
    rank_extent(LL, np, 1, len, sw);
    mn = len < mn ? len : mn;
  }
  return mn;
}

#define CHECK_HIP(x)                                                                  \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      g.err = std::string(#x) + ": " + hipGetErrorString(e_);                         \
      return -2;                                                                      \
    }                                                                                 \
  } while (0)

#define REQUIRE_INIT_NOJOIN()                           \
  do {                                                  \
    if (!g.inited) {                                    \
      g.err = "roms_gpu: not initialised";              \
      return -1;                                        \
    }                                                   \
  } while (0)
// A timed-out IPC halo wait is fatal (the reference's MPI_Waitall never
// gives up; here the wait is bounded so a lost peer cannot hang the GPU):
// every later entry reports it instead of computing on stale halos.
#define REQUIRE_HALO_OK()                                                                    \
  do {                                                                                       \
    if (g.d.halo && halo_failed(g.halo)) {                                                   \
      g.err = "roms_gpu: a halo exchange wait timed out (IPC transport, ROMS_GPU_IPC_TIMEOUT);" \
              " the state since is invalid";                                                 \
      return -6;                                                                             \
    }                                                                                        \
  } while (0)
// every entry but step2d first joins a fast-loop exchange still in flight on
// the halo stream (launch_step2d overlaps it with the next fast step)
#define REQUIRE_INIT()                                  \
  do {                                                  \
    REQUIRE_INIT_NOJOIN();                              \
    REQUIRE_HALO_OK();                                  \
    if (g.d.halo) halo_join(g.halo, g.s);               \
    g.rho_slot = 0;                                     \
  } while (0)
// entries that leave every model field as it was keep g.rho_slot
#define REQUIRE_INIT_RO()                               \
  const int rho_keep_ = g.rho_slot;                     \
  REQUIRE_INIT();                                       \
  g.rho_slot = rho_keep_

int post_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g.err = std::string("kernel launch: ") + hipGetErrorString(e);
    return -3;
  }
  return 0;
}

Bounds make_bounds(const roms_dims& D, int pitch, int gx = 0) {
  Bounds b{};
  b.Lm = D.Lm; b.Mm = D.Mm; b.N = D.N; b.NT = D.NT;
  b.nTS = 1;
  b.nx2 = pitch;
  b.gx = gx;
  b.n2 = (long)pitch * (D.Mm + 4 + 2 * gx);
  b.n3 = b.n2 * D.N;
  b.n3w = b.n2 * (D.N + 1);
  b.istr = 1; b.iend = D.Lm; b.jstr = 1; b.jend = D.Mm;
  b.ew_periodic = D.ew_periodic; b.ns_periodic = D.ns_periodic;
  b.west_exch = D.west_exchng; b.east_exch = D.east_exchng;
  b.south_exch = D.south_exchng; b.north_exch = D.north_exchng;
  // WESTERN_EDGE etc. are only defined without periodicity (set_global_definitions.h:174-191)
  b.west_edge = !D.ew_periodic && !D.west_exchng;
  b.east_edge = !D.ew_periodic && !D.east_exchng;
  b.south_edge = !D.ns_periodic && !D.south_exchng;
  b.north_edge = !D.ns_periodic && !D.north_exchng;
  b.istrR = b.west_edge ? b.istr - 1 : b.istr;
  b.istrU = b.west_edge ? b.istr + 1 : b.istr;
  b.iendR = b.east_edge ? b.iend + 1 : b.iend;
  b.jstrR = b.south_edge ? b.jstr - 1 : b.jstr;
  b.jstrV = b.south_edge ? b.jstr + 1 : b.jstr;
  b.jendR = b.north_edge ? b.jend + 1 : b.jend;
  b.istrE = (D.ew_periodic || D.west_exchng) ? b.istr - 2 : b.istr - 1;
  b.iendE = (D.ew_periodic || D.east_exchng) ? b.iend + 2 : b.iend + 1;
  b.jstrE = (D.ns_periodic || D.south_exchng) ? b.jstr - 2 : b.jstr - 1;
  b.jendE = (D.ns_periodic || D.north_exchng) ? b.jend + 2 : b.jend + 1;
  return b;
}

// boundary arrays and the vertical stretching curves are not (i,j) planes
bool planar_field(int id) { return !(id == ROMS_Cs_w || id == ROMS_Cs_r || (id >= ROMS_zeta_west && id <= ROMS_t_north)); }

long field_count(int id, const Bounds& b) {
  const long n2 = b.n2, n3 = b.n3, n3w = b.n3w;
  switch (id) {
    case ROMS_Cs_w: case ROMS_Cs_r: return b.N + 1;
    case ROMS_zeta: case ROMS_ubar: case ROMS_vbar: return 4 * n2;
    case ROMS_u: case ROMS_v: return 3 * n3;
    case ROMS_t: return 3 * n3 * b.NT;
    case ROMS_FlxU: case ROMS_FlxV: case ROMS_Hz: case ROMS_Hz_u: case ROMS_Hz_v: case ROMS_z_r: case ROMS_rho:
    case ROMS_rho1: case ROMS_qp1: case ROMS_ru: case ROMS_rv: return n3;
    case ROMS_We: case ROMS_Wi: case ROMS_z_w: case ROMS_bvf: case ROMS_Akv: case ROMS_ghat: case ROMS_swr_frac:
      return n3w;
    case ROMS_Akt: return n3w * b.nTS;
    case ROMS_diff2: case ROMS_stflx: return n2 * b.NT;
    default: break;
  }
  if (id >= ROMS_zeta_west && id <= ROMS_t_north) {
    const int side = (id - ROMS_zeta_west) % 4, var = (id - ROMS_zeta_west) / 4;
    const long nb = side < 2 ? b.Mm + 2 : b.Lm + 2;
    return var < 3 ? nb : var < 5 ? nb * b.N : nb * b.N * b.NT;
  }
  return n2;
}

double** field_slot(Fields& F, int id) {
  switch (id) {
    case ROMS_h: return &F.h; case ROMS_hinv: return &F.hinv; case ROMS_f: return &F.f; case ROMS_fomn: return &F.fomn;
    case ROMS_pm: return &F.pm; case ROMS_pn: return &F.pn; case ROMS_dm_r: return &F.dm_r; case ROMS_dn_r: return &F.dn_r;
    case ROMS_dm_u: return &F.dm_u; case ROMS_dn_u: return &F.dn_u; case ROMS_dm_v: return &F.dm_v;
    case ROMS_dn_v: return &F.dn_v; case ROMS_dm_p: return &F.dm_p; case ROMS_dn_p: return &F.dn_p;
    case ROMS_pmon_u: return &F.pmon_u; case ROMS_pnom_v: return &F.pnom_v; case ROMS_rmask: return &F.rmask;
    case ROMS_pmask: return &F.pmask; case ROMS_umask: return &F.umask; case ROMS_vmask: return &F.vmask;
    case ROMS_Cs_w: return &F.Cs_w; case ROMS_Cs_r: return &F.Cs_r;
    case ROMS_zeta: return &F.zeta; case ROMS_ubar: return &F.ubar; case ROMS_vbar: return &F.vbar;
    case ROMS_u: return &F.u; case ROMS_v: return &F.v; case ROMS_t: return &F.t; case ROMS_FlxU: return &F.FlxU;
    case ROMS_FlxV: return &F.FlxV; case ROMS_We: return &F.We; case ROMS_Wi: return &F.Wi; case ROMS_Hz: return &F.Hz;
    case ROMS_Hz_u: return &F.Hz_u; case ROMS_Hz_v: return &F.Hz_v; case ROMS_z_r: return &F.z_r; case ROMS_z_w: return &F.z_w;
    case ROMS_rufrc: return &F.rufrc; case ROMS_rvfrc: return &F.rvfrc; case ROMS_rhoA: return &F.rhoA;
    case ROMS_rhoS: return &F.rhoS; case ROMS_r_D: return &F.r_D; case ROMS_Zt_avg1: return &F.Zt_avg1;
    case ROMS_DU_avg1: return &F.DU_avg1; case ROMS_DV_avg1: return &F.DV_avg1; case ROMS_DU_avg2: return &F.DU_avg2;
    case ROMS_DV_avg2: return &F.DV_avg2; case ROMS_DU_avg_bak: return &F.DU_avg_bak;
    case ROMS_DV_avg_bak: return &F.DV_avg_bak; case ROMS_rho: return &F.rho; case ROMS_rho1: return &F.rho1;
    case ROMS_qp1: return &F.qp1; case ROMS_bvf: return &F.bvf; case ROMS_Akv: return &F.Akv; case ROMS_Akt: return &F.Akt;
    case ROMS_visc2_r: return &F.visc2_r; case ROMS_visc2_p: return &F.visc2_p; case ROMS_diff2: return &F.diff2;
    case ROMS_hbls: return &F.hbls; case ROMS_hbbl: return &F.hbbl; case ROMS_ghat: return &F.ghat;
    case ROMS_swr_frac: return &F.swr_frac; case ROMS_sustr: return &F.sustr; case ROMS_svstr: return &F.svstr;
    case ROMS_stflx: return &F.stflx; case ROMS_srflx: return &F.srflx; case ROMS_swflx: return &F.swflx;
    case ROMS_ru: return &F.ru; case ROMS_rv: return &F.rv;
    case ROMS_dndx: return &F.dndx; case ROMS_dmde: return &F.dmde; case ROMS_ptide: return &F.ptide;
    case ROMS_uwnd: return &F.uwnd; case ROMS_vwnd: return &F.vwnd; case ROMS_tair: return &F.tair;
    case ROMS_qair: return &F.qair; case ROMS_prate: return &F.prate; case ROMS_swrad: return &F.swrad;
    case ROMS_lwrad: return &F.lwrad; case ROMS_sustr_r: return &F.sustr_r; case ROMS_svstr_r: return &F.svstr_r;
    default: break;
  }
  if (id >= ROMS_zeta_west && id <= ROMS_t_north) {
    const int side = (id - ROMS_zeta_west) % 4, var = (id - ROMS_zeta_west) / 4;
    double** tab[6] = {F.bzeta, F.bubar, F.bvbar, F.bu, F.bv, F.bt};
    return &tab[var][side];
  }
  return nullptr;
}

double* dev_base(double* p) {
  auto it = g.guard_base.find(p);
  return it == g.guard_base.end() ? p : it->second;
}
// doubles one dev_alloc of n takes (guard bands, alignment lead, wide-halo
// rows), rounded up to 256 B so that arena slices keep hipMalloc's alignment
long dev_alloc_size(long n) {
  const Bounds& b = g.d.b;
  const long G = g.guard ? 4096 : 0;
  const long pad = (g.off || b.gx) ? kRowAlign : 0;
  return (n + 2 * G + pad + (long)b.gx * b.nx2 + 31) / 32 * 32;
}
// zero-initialised device array of n doubles (guard bands when g.guard),
// sliced from g.arena while it has room, else its own hipMalloc
hipError_t dev_alloc(double*& p, long n) {
  const long G = g.guard ? 4096 : 0;
  const Bounds& b = g.d.b;
  // alignment shift (hipMalloc is 256-B aligned) and, with wide fast halos,
  // the gx ghost rows below the first plane's j = -1 plus the gx columns left
  // of its i = -1 (roms_dev.h); the last plane's extra rows are inside n
  const long lead = g.off ? g.off : b.gx;   // g.off = kAlignOff >= gx (checked at init)
  const long pre = (long)b.gx * b.nx2 + lead;
  const long pad = (g.off || b.gx) ? kRowAlign : 0;
  double* base = nullptr;
  const long sz = dev_alloc_size(n);
  const bool sliced = g.arena && g.arena_used + sz <= g.arena_n;
  hipError_t e = hipSuccess;
  if (sliced) {
    base = g.arena + g.arena_used;
    g.arena_used += sz;
  } else {
    e = hipMalloc(&base, (size_t)(n + 2 * G + pad + (long)b.gx * b.nx2) * sizeof(double));
  }
  if (e != hipSuccess) return e;
  if (G) {
    e = hipMemsetD32((hipDeviceptr_t)base, 0x7FF87FF8, (size_t)(n + 2 * G + pad + (long)b.gx * b.nx2) * 2);   // NaN bit pattern
    if (e != hipSuccess) return e;
  }
  p = base + G + pre;
  if (sliced) g.guard_base[p] = nullptr;   // freed with the arena (hipFree(nullptr) is a no-op)
  else if (G || pre) g.guard_base[p] = base;
  // The library's kernels run on a non-blocking stream, which does not wait
  // for work on the null stream: the zero fill must have landed before the
  // first kernel reads the array, or it may see what a previous model left in
  // the same memory (or be zeroed after the kernel wrote it).  The fill covers
  // the leading ghost rows too.
  e = hipMemset(p - pre + lead - b.gx, 0, (size_t)(n + pre - lead + b.gx) * sizeof(double));
  return e != hipSuccess ? e : hipStreamSynchronize(nullptr);
}

void free_all() {
  io_free();
  frc_free();
  if (g.small) { (void)hipFree(g.small); g.small = nullptr; g.small_n = 0; }
  if (g.stage) { (void)hipFree(g.stage); g.stage = nullptr; g.stage_n = 0; }
  for (hipEvent_t e : g.ev) (void)hipEventDestroy(e);
  g.ev.clear();
  halo_free(g.halo);
  g.halo = Halo{};
  g.d.halo = nullptr;
  for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
  g.graphs.clear();
  for (int id = 0; id < ROMS_NFIELDS; id++)
    if (g.f[id].d) { (void)hipFree(dev_base(g.f[id].d)); g.f[id] = FieldDesc{}; }
  for (double* p : g.scratch) (void)hipFree(dev_base(p));
  g.guard_base.clear();
  if (g.arena) { (void)hipFree(g.arena); g.arena = nullptr; g.arena_n = g.arena_used = 0; }
  g.scratch.clear();
  if (g.d.f.pipe_idx) { (void)hipFree(g.d.f.pipe_idx); g.d.f.pipe_idx = nullptr; }
  if (g.d.f.riv_face) { (void)hipFree(g.d.f.riv_face); g.d.f.riv_face = nullptr; }
  if (g.d.f.uv2e_couple) { (void)hipFree(g.d.f.uv2e_couple); g.d.f.uv2e_couple = nullptr; }
  if (g.d.f.uv2e_flux) { (void)hipFree(g.d.f.uv2e_flux); g.d.f.uv2e_flux = nullptr; }
  g.riv_maxidx = 0;
  g.have_swr = false;
  for (double*& p : g.d.f.ub)
    if (p) { (void)hipFree(p); p = nullptr; }
  if (g.h_diag) { (void)hipHostFree(g.h_diag); g.h_diag = nullptr; }
  if (g.d_diag) { (void)hipFree(g.d_diag); g.d_diag = nullptr; }
  if (g.s) { (void)hipStreamDestroy(g.s); g.s = nullptr; }
  if (g.s2) { (void)hipStreamDestroy(g.s2); g.s2 = nullptr; }
  for (hipEvent_t& e : g.pev)
    if (e) { (void)hipEventDestroy(e); e = nullptr; }
  g.inited = false;
}

Tlev to_tlev(const roms_tlev* t) {
  Tlev r;
  r.iic = t->iic; r.ntstart = t->ntstart; r.forw_start = t->forw_start; r.iif = t->iif; r.nfast = t->nfast;
  r.kstp = t->kstp; r.knew = t->knew; r.nstp = t->nstp; r.nrhs = t->nrhs; r.nnew = t->nnew;
  return r;
}

// bracket one routine's launches with HIP events when it is the timed one
#define TIMED(id, stmt)                                                     \
  do {                                                                      \
    const bool on_ = g.timed == (id) && g.nev + 2 <= g.ev.size();           \
    if (on_) (void)hipEventRecord(g.ev[g.nev], s);                          \
    stmt;                                                                   \
    if (on_) { (void)hipEventRecord(g.ev[g.nev + 1], s); g.nev += 2; }      \
  } while (0)

// host <-> device layout copies (defined below)
hipError_t field_h2d(int id, double* dev, const double* host);
hipError_t rows_h2d(double* dev, const double* host, long rows);
}  // namespace
int roms::shim_enter(ShimState& S, bool read_only) {
  const int rho_keep = g.rho_slot;
  REQUIRE_INIT();
  if (read_only) g.rho_slot = rho_keep;
  S.d = &g.d; S.s = g.s; S.dims = &g.dims; S.cfg = &g.cfg; S.err = &g.err;
  return 0;
}
void roms::shim_set_error(const std::string& e) { g.err = e; }
double* roms::shim_field(int id) { return (id >= 0 && id < ROMS_NFIELDS) ? g.f[id].d : nullptr; }
long roms::shim_field_dev_count(int id) { return (id >= 0 && id < ROMS_NFIELDS) ? g.f[id].count : -1; }
hipError_t roms::shim_field_h2d(int id, double* dev, const double* host) { return field_h2d(id, dev, host); }
hipError_t roms::shim_rows_h2d(double* dev, const double* host, long rows) { return rows_h2d(dev, host, rows); }
double* roms::shim_scratch_small(long n) {
  if (g.small_n < n) {
    if (g.small) { (void)hipStreamSynchronize(g.s); (void)hipFree(g.small); g.small = nullptr; }
    if (hipMalloc(&g.small, (size_t)n * sizeof(double)) != hipSuccess) { g.small_n = 0; return nullptr; }
    g.small_n = n;
  }
  return g.small;
}
void roms::ktimer_mark(hipStream_t s, int id, int end, int count) {
  if (g.timed != id) return;
  if (!end) {
    if (g.nev + 2 <= g.ev.size()) (void)hipEventRecord(g.ev[g.nev], s);
  } else if (g.nev + 2 <= g.ev.size()) {
    (void)hipEventRecord(g.ev[g.nev + 1], s);
    g.nev += 2;
    g.kcount += count;
  }
}
namespace {

// the roms_step sequence for one step whose indices are already set in *t
// (nstp,nrhs=nstp,nnew=3 on entry); enqueues everything on g.s
// rho_current: rho_eos(nrhs) is already current (g.rho_slot, see there)
void enqueue_step(roms_tlev* t, bool rho_current, bool store_huv) {
  const Dev& d = g.d;
  hipStream_t s = g.s;
  Tlev T = to_tlev(t);
  const long exch0 = g.halo.nexch;
  const bool pot = g.cfg.pot_tides != 0;
  g.rho_slot = 0;
  // Two streams where the reference's order has no data dependence (single
  // rank -- a multi-rank halo exchange keeps one order on its transport --
  // and not while one routine is being timed):
  //   predictor: lmd_vmix(nstp) (writes Akv, Akt, hbls, hbbl, ghat and its
  //     own work arrays) beside prsgrd (writes ru, rv); pre_step3d reads both
  //   corrector: omega (We, Wi) beside rho_eos (rho1, qp1, P, bvf, rhoA,
  //     rhoS), then lmd_vmix(nrhs) beside prsgrd; step3d_uv1 reads all
  // Same kernels, same inputs: the results are bitwise those of one stream.
  // The low-occupancy column kernels (KPP, omega) fill CUs the other
  // routine leaves idle.
  // g.par: a mask of the pairs (ROMS_GPU_PAR=1: all; ROMS_GPU_PAR_MASK=bits):
  // 1 predictor lmd_vmix | prsgrd, 2 corrector omega | rho_eos, 4 corrector
  // lmd_vmix | prsgrd, 8 pre_step3d tracer | momentum solves, 16 predictor P
  // (linear EOS) | set_HUV, omega
  const int pm = d.halo == nullptr && g.timed < 0 ? g.par : 0;
  hipStream_t s2 = g.s2;
  auto fork = [&](int k) {   // s2 continues after everything queued on s so far
    (void)hipEventRecord(g.pev[k], s);
    (void)hipStreamWaitEvent(s2, g.pev[k], 0);
  };
  auto join = [&](int k) {   // s continues after everything queued on s2 so far
    (void)hipEventRecord(g.pev[k], s2);
    (void)hipStreamWaitEvent(s, g.pev[k], 0);
  };
  // Multi-rank runs (Halo::xoverlap: the default with > 1 rank when every
  // rank drives its own GPU; not while one routine is timed): the trailing exchange of a producer in DEFER(...) runs
  // on the halo stream beside the routines that follow it, and XJOIN(t) makes
  // the library stream wait for it just before the first routine that reads
  // its halo (mpi_exchanges.F:672-800 posts and waits on every
  // exchange in place).  Where the reference's order allows (no data
  // dependence either way) a routine that reads none of the halo moves in
  // between: lmd_vmix(nstp) ahead of omega, rho_eos(nrhs) ahead of the
  // corrector's omega.  Same kernels on the same inputs, so the fields are
  // bitwise those of the serial order (tests/test_gpu_multirank.py, with a
  // delay hook that makes a missing join read stale halos).
  const bool xo = d.halo != nullptr && g.halo.xoverlap > 0 && g.timed < 0;
  long xt = -1;   // ticket of the last deferred exchange
#define DEFER(call)                          \
  do {                                       \
    if (xo) g.halo.defer = 1;                \
    call;                                    \
    g.halo.defer = 0;                        \
    if (xo) xt = g.halo.nfork - 1;           \
  } while (0)
#define XJOIN(t)                                   \
  do {                                             \
    if (xo) halo_join_to(g.halo, s, (t));          \
  } while (0)
  // Halo::xskip (test hook): leave out the joins whose bit is set
#define XJOIN_T(bit, t)                            \
  do {                                             \
    if (!(g.halo.xskip & (bit))) XJOIN(t);         \
  } while (0)
  frc_step_phase(d, s, 0, pot);     // set_forces, frc_time 'current' (main.F:384-385)
  launch_bulk_flux(d, s, T.nrhs);   // set_forces (main.F:386): BULK_FRC only
  frc_step_phase(d, s, 1, pot);     // set_bry_all '1/2 fwd' + set_tides (main.F:389-394)
  if (!rho_current) TIMED(ROMS_R_RHO_EOS, launch_rho_eos(d, s, T, T.nrhs));
  // every rho_eos of the library leaves P current (p_in_rho): the
  // step-opening one, or the previous step's closing one it reuses; else
  // (linear EOS) prsgrd's P integral (rho, z_r, z_w: nothing set_HUV or
  // omega writes) runs on the side stream beside them
  const bool p_ready = p_in_rho(d);
  const bool p_side = (pm & 16) && !p_ready && d.p.prs_split;
  if (p_side) {
    fork(7);
    launch_prsgrd_P(d, s2);
  }
  TIMED(ROMS_R_SET_HUV, DEFER(launch_set_huv(d, s, T, store_huv)));   // FlxU, FlxV
  const long x_huv = xt;
  const bool lmd2 = g.cfg.lmd_mixing && (pm & 1);
  // lmd_vmix(nstp) reads u, v(nstp), bvf, Hz, z_r, z_w and the surface fluxes:
  // none of set_HUV's or omega's outputs, so on a multi-rank run it goes first
  // and covers set_HUV's exchange (Akv, Akt, hbls, hbbl follow on the halo stream)
  const bool lmd_early = xo && g.cfg.lmd_mixing && !lmd2;
  if (lmd_early) TIMED(ROMS_R_LMD_VMIX, DEFER(launch_lmd_vmix(d, s, T, T.nstp)));
  XJOIN_T(1, x_huv);   // omega reads FlxU(iend+1), FlxV(jend+1)
  // the predictor's omega also forms pre_step3d's Hz_bak/Hz_fwd (nothing in
  // between -- lmd_vmix, prsgrd -- writes FlxU, FlxV, Hz, We or Wi)
  bool hb_done = false;
  TIMED(ROMS_R_OMEGA, DEFER(hb_done = launch_omega(d, s, T, d.p.omega_hb && d.p.hoist && T.nrhs != 3 ?
                                                                 0.5 * pre_step3d_dtau(d, T) : 0.0)));
  if (p_side) join(7);
  if (lmd2) {
    fork(0);
    launch_lmd_vmix(d, s2, T, T.nstp);
  } else if (g.cfg.lmd_mixing && !lmd_early) {
    TIMED(ROMS_R_LMD_VMIX, launch_lmd_vmix(d, s, T, T.nstp));
  }
  // the horizontal momentum r.h.s. of pre_step3d / step3d_uv1 rides in the
  // prsgrd kernel just before them (prsgrd_can_fuse_uv; nothing between the
  // two touches u, v(nrhs), FlxU, FlxV, Hz or ru, rv); it reads neither We, Wi
  // nor the mixing coefficients, whose exchanges it covers
  const bool fuse_uv = prsgrd_can_fuse_uv(d);
  TIMED(ROMS_R_PRSGRD, launch_prsgrd(d, s, T, fuse_uv ? 0 : -1, p_ready || p_side));
  if (lmd2) join(1);
  XJOIN_T(2, xt);   // pre_step3d reads We, Akv, Akt across the halo
  const Side side{s2, g.pev[5], g.pev[6]};
  TIMED(ROMS_R_PRE_STEP3D,
        DEFER(launch_pre_step3d(d, s, T, fuse_uv, hb_done, (pm & 8) ? &side : nullptr)));   // t(nnew)
  const long x_pre = xt;
  // set_HUV1 reads u, v(nnew), Hz and the barotropic averages, no tracer
  TIMED(ROMS_R_SET_HUV1, DEFER(launch_set_huv1(d, s, T)));   // FlxU, FlxV, u, v(nnew)
  const long x_huv1 = xt;
  t->nrhs = 3;
  t->nnew = 3 - t->nstp;
  T = to_tlev(t);
  if (xo) {
    // rho_eos(nrhs) reads t(nrhs) across the halo (pre_step3d's exchange) and
    // none of set_HUV1's outputs: it covers set_HUV1's exchange, then omega
    XJOIN_T(4, x_pre);
    TIMED(ROMS_R_RHO_EOS, launch_rho_eos(d, s, T, T.nrhs));
    XJOIN_T(8, x_huv1);
    TIMED(ROMS_R_OMEGA, DEFER(launch_omega(d, s, T)));   // We, Wi
  } else {
    if (pm & 2) {
      fork(2);
      launch_omega(d, s2, T);
    } else {
      TIMED(ROMS_R_OMEGA, launch_omega(d, s, T));
    }
    TIMED(ROMS_R_RHO_EOS, launch_rho_eos(d, s, T, T.nrhs));
  }
  frc_step_phase(d, s, 2, pot);     // set_forces, '1/2 fwd' (main.F:433)
  launch_bulk_flux(d, s, T.nrhs);   // set_forces (main.F:433): BULK_FRC only
  const bool lmd2c = g.cfg.lmd_mixing && (pm & 4);
  if (lmd2c) {
    fork(3);   // after rho_eos (bvf) and the bulk fluxes (stflx, srflx, sustr_r)
    launch_lmd_vmix(d, s2, T, T.nrhs);
  } else if (g.cfg.lmd_mixing) {
    TIMED(ROMS_R_LMD_VMIX, DEFER(launch_lmd_vmix(d, s, T, T.nrhs)));   // Akv, Akt, hbls, hbbl
  }
  frc_step_phase(d, s, 3, pot);     // set_bry_all 'forward' + set_tides (main.F:438-441)
  TIMED(ROMS_R_PRSGRD, launch_prsgrd(d, s, T, fuse_uv ? 1 : -1, p_ready));
  if ((pm & 2) || lmd2c) join(4);
  XJOIN_T(16, xt);   // step3d_uv1 reads We and Akv across the halo
  TIMED(ROMS_R_STEP3D_UV1, launch_step3d_uv1(d, s, T, fuse_uv));
  if (g.cfg.uv_vis2) TIMED(ROMS_R_VISC3D, launch_visc3d(d, s, T));
  // the fast loop is timed as one interval over its nfast steps (kernel-level
  // count, as the graph replays it: no event between two fast steps)
  const bool t2d = g.timed == ROMS_R_STEP2D && g.nev + 2 <= g.ev.size();
  if (t2d) (void)hipEventRecord(g.ev[g.nev], s);
  for (int iif = 1; iif <= t->nfast; iif++) {
    t->iif = iif;
    t->kstp = t->knew;
    t->knew = t->kstp + 1;
    if (t->knew > 4) t->knew = 1;
    T = to_tlev(t);
    launch_step2d(d, s, T, g.w1, g.w2);
  }
  if (t2d) {
    (void)hipEventRecord(g.ev[g.nev + 1], s);
    g.nev += 2;
    g.kcount += t->nfast;
  }
  TIMED(ROMS_R_STEP3D_UV2, launch_step3d_uv2(d, s, T));
  // step3d_t reads We, Wi in its own columns only (the vertical fluxes and
  // the implicit solve): omega's exchange runs beside it, and the tracer
  // exchange that closes the step (t3dmix's or step3d_t's) joins it
  TIMED(ROMS_R_OMEGA, DEFER(launch_omega(d, s, T)));
  // with TS_DIF2 the tracer exchange after step3d_t is overwritten by
  // t3dmix's before anything reads the halo (t3dmix_S.F reads t(nrhs)): one
  TIMED(ROMS_R_STEP3D_T, launch_step3d_t(d, s, T, !g.cfg.ts_dif2 || d.p.iso));
  if (g.cfg.ts_dif2) TIMED(ROMS_R_T3DMIX, launch_t3dmix(d, s, T));
  XJOIN(xt);
  TIMED(ROMS_R_RHO_EOS, launch_rho_eos(d, s, T, T.nnew));
  if (d.halo) halo_join(g.halo, s);   // nothing forked outlives the step (graph capture)
#undef DEFER
#undef XJOIN
#undef XJOIN_T
  g.rho_slot = T.nnew;
  g.step_exch = g.halo.nexch - exch0;
}

}  // namespace

namespace {
// ---- host (rows of Lm+4) <-> device (rows of nx2) copies, blocking on the
// library stream.  Equal pitches: one DMA.  Otherwise the compact rows go
// through the device staging buffer and one row-copy kernel re-pitches them
// (a strided hipMemcpy2D from pageable memory would move row by row). ----
double* stage_get(long n) {
  if (g.stage_n < n) {
    if (g.stage) { (void)hipStreamSynchronize(g.s); (void)hipFree(g.stage); g.stage = nullptr; g.stage_n = 0; }
    if (hipMalloc(&g.stage, (size_t)n * sizeof(double)) != hipSuccess) return nullptr;
    g.stage_n = n;
  }
  return g.stage;
}
// `rows` host rows: whole planes of Mm+4 rows (plane stride hb.n2 on the
// host, b.n2 on the device)
bool same_layout() { return g.d.b.nx2 == g.hb.nx2 && g.d.b.n2 == g.hb.n2; }
hipError_t rows_h2d(double* dev, const double* host, long rows) {
  const Bounds& b = g.d.b;
  const long hx = g.hb.nx2, n = rows * hx;
  if (same_layout()) return copy_on(dev, host, (size_t)n * sizeof(double), hipMemcpyHostToDevice, g.s);
  double* st = stage_get(n);
  if (!st) return hipErrorOutOfMemory;
  hipError_t e = hipMemcpyAsync(st, host, (size_t)n * sizeof(double), hipMemcpyHostToDevice, g.s);
  if (e != hipSuccess) return e;
  launch_rows_copy(dev, b.nx2, b.n2, st, hx, g.hb.n2, hx, rows, b.Mm + 4, g.s);
  return hipStreamSynchronize(g.s);
}
hipError_t rows_d2h(double* host, const double* dev, long rows) {
  const Bounds& b = g.d.b;
  const long hx = g.hb.nx2, n = rows * hx;
  if (same_layout()) return copy_on(host, dev, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, g.s);
  double* st = stage_get(n);
  if (!st) return hipErrorOutOfMemory;
  launch_rows_copy(st, hx, g.hb.n2, dev, b.nx2, b.n2, hx, rows, b.Mm + 4, g.s);
  hipError_t e = hipMemcpyAsync(host, st, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, g.s);
  return e != hipSuccess ? e : hipStreamSynchronize(g.s);
}
hipError_t field_h2d(int id, double* dev, const double* host) {
  const FieldDesc& f = g.f[id];
  if (!f.planar) return copy_on(dev, host, (size_t)f.hcount * sizeof(double), hipMemcpyHostToDevice, g.s);
  return rows_h2d(dev, host, f.hcount / g.hb.nx2);
}
hipError_t field_d2h(int id, double* host, const double* dev) {
  const FieldDesc& f = g.f[id];
  if (!f.planar) return copy_on(host, dev, (size_t)f.hcount * sizeof(double), hipMemcpyDeviceToHost, g.s);
  return rows_d2h(host, dev, f.hcount / g.hb.nx2);
}
// a host-layout int / double plane array as a device-layout host vector
template <class T>
std::vector<T> to_dev_layout(const T* h, long planes) {
  const Bounds& b = g.d.b;
  const long hx = g.hb.nx2, prow = b.Mm + 4;
  std::vector<T> v((size_t)(b.n2 * planes), T(0));
  for (long p = 0; p < planes; p++)
    for (long r = 0; r < prow; r++)
      std::memcpy(v.data() + p * b.n2 + r * b.nx2, h + (p * prow + r) * hx, (size_t)hx * sizeof(T));
  return v;
}

}  // namespace

extern "C" {

int roms_gpu_abi_version(void) { return ROMS_GPU_ABI_VERSION; }

// The zero fill of a new array must land before the library's stream uses
// it (dev_alloc): `chunks` arrays of n doubles are filled with ones on the
// library stream and freed, then allocated again one by one through
// dev_alloc (recycled memory, as between models of one process); on the
// library stream at once each is counted for elements that are not zero
// (a fill that lands late: stale data read) and then overwritten with ones;
// after the whole device has drained, the elements that are not one are
// counted (a fill that lands late: the stream's writes zeroed).  The sum of
// both counts is 0 unless the fill and the stream race.
int roms_gpu_selftest_zero_fill(long n, int chunks, long* bad) {
  REQUIRE_INIT();
  if (n < 1 || chunks < 1 || chunks > 1024 || !bad) { g.err = "roms_gpu_selftest_zero_fill: bad argument"; return -1; }
  std::vector<double*> a((size_t)chunks, nullptr);
  unsigned long long* cnt = nullptr;
  bool guarded = false;   // a[] came from dev_alloc (guard_base entries when g.guard)
  // every exit frees what was taken, on error paths too
  auto release = [&]() {
    (void)hipStreamSynchronize(g.s);
    for (double*& p : a) {
      if (!p) continue;
      if (guarded) {   // dev_alloc offsets whenever it records a base (guard, pitch offset or wide ghosts)
        (void)hipFree(dev_base(p));
        g.guard_base.erase(p);
      } else {
        (void)hipFree(p);
      }
      p = nullptr;
    }
    if (cnt) { (void)hipFree(cnt); cnt = nullptr; }
  };
  auto fail = [&](hipError_t e, const char* what) -> int {
    g.err = std::string("roms_gpu_selftest_zero_fill: ") + what + ": " + hipGetErrorString(e);
    release();
    return -2;
  };
  hipError_t e;
  for (double*& p : a) {
    if ((e = hipMalloc(&p, (size_t)n * sizeof(double))) != hipSuccess) { p = nullptr; return fail(e, "hipMalloc"); }
    launch_fill_ones(p, n, g.s);
  }
  if ((e = hipStreamSynchronize(g.s)) != hipSuccess) return fail(e, "fill");
  for (double*& p : a) {
    (void)hipFree(p);
    p = nullptr;
  }
  if ((e = hipMalloc(&cnt, 2 * sizeof(unsigned long long))) != hipSuccess) { cnt = nullptr; return fail(e, "hipMalloc"); }
  if ((e = hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned long long), g.s)) != hipSuccess) return fail(e, "memset");
  if ((e = hipStreamSynchronize(g.s)) != hipSuccess) return fail(e, "memset");
  guarded = true;
  for (double*& p : a) {
    if ((e = dev_alloc(p, n)) != hipSuccess) { p = nullptr; return fail(e, "dev_alloc"); }
    launch_count_nonzero(p, n, cnt, g.s, 0.0);
    launch_fill_ones(p, n, g.s);
  }
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail(e, "drain");
  for (double* p : a) launch_count_nonzero(p, n, cnt + 1, g.s, 1.0);
  unsigned long long h[2] = {0, 0};
  if ((e = hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, g.s)) != hipSuccess) return fail(e, "copy");
  if ((e = hipStreamSynchronize(g.s)) != hipSuccess) return fail(e, "copy");
  release();
  *bad = (long)(h[0] + h[1]);
  return 0;
}
const char* roms_gpu_last_error(void) { return g.err.c_str(); }
void* roms_gpu_stream(void) { return (void*)g.s; }

int roms_gpu_init(const roms_dims* dims, const roms_cfg* cfg, int device, void* comm) {
  if (g.inited) free_all();
  if (!dims || !cfg) { g.err = "roms_gpu_init: null argument"; return -1; }
  if (dims->N < 2 || dims->Lm < 2 || dims->Mm < 2 || dims->NT < 1) { g.err = "roms_gpu_init: bad dims"; return -1; }
  if (cfg->nfast < 1 || cfg->nfast > ROMS_MAX_FAST) { g.err = "roms_gpu_init: bad nfast"; return -1; }
  const int nranks = dims->np_xi * dims->np_eta;
  if (nranks < 1) { g.err = "roms_gpu_init: bad processor grid"; return -1; }
  if (nranks > 1 && comm == nullptr) { g.err = "roms_gpu_init: np_xi*np_eta > 1 needs a communicator"; return -1; }
  if (comm != nullptr) {
    RomsComm* c = (RomsComm*)comm;
    if (comm_size(c) != nranks || comm_rank(c) != dims->inode + dims->jnode * dims->np_xi) {
      g.err = "roms_gpu_init: communicator size/rank does not match np_xi*np_eta / inode+jnode*np_xi";
      return -1;
    }
  }
  g.dims = *dims;
  g.cfg = *cfg;
  g.have_volume = false;
  g.area = g.volume = 0.0;
  g.d = Dev{};
  {
    // device row pitch: Lm+4 rounded up to 128 B, base shifted so that i = 1
    // starts a line (roms_dev.h); ROMS_GPU_PITCH=0 keeps the host layout
    const char* e = getenv("ROMS_GPU_PITCH");
    const bool pad = !(e && e[0] == '0');
    const int hx = dims->Lm + 4;
    // Multi-rank runs: the barotropic fast loop exchanges zeta/ubar/vbar
    // every s2d_k fast steps over 2*s2d_k-wide halos and recomputes the
    // steps between on the overlap (launch_step2d), so the device planes
    // carry gx = 2*(s2d_k-1) extra ghost rows/columns (roms_dev.h).  Not with
    // open boundaries (their 1-D boundary arrays end at the reference's halo)
    // or the split fast-step kernels; rivers and pipes fall back to every step
    // at run time.  ROMS_GPU_S2D_K=1..8 (default 4; 1: every step).  One
    // GPU with every exchange self-addressed through IPC (C2, 92 exchanges
    // per step at K = 1): 7.48 / 7.11 / 7.01 / 6.98 ms per step at K = 1..4
    // against 6.49 without a communicator (profiles/r4_j_fast_exchange_interval_ab.txt).
    int k = 4;
    const char* ek = getenv("ROMS_GPU_S2D_K");   // 1..8 (an interconnect slower than one GPU's may want 6-8)
    if (ek && atoi(ek) >= 1 && atoi(ek) <= 8) k = atoi(ek);
    const char* es = getenv("ROMS_GPU_S2D_SPLIT");
    const bool split = es && es[0] == '1';
    const int obc = cfg->obc & ((dims->ew_periodic ? 0 : 3) | (dims->ns_periodic ? 0 : 12));
    // every rank decides alike, from the global sizes: the 2k-wide strips
    // (and the 2(k-1) cells a widened fast step reaches into its neighbour)
    // must lie inside the neighbour's own cells on every rank, so k shrinks
    // until 2k+2 fits the smallest subdomain of the mpi_setup split
    if (comm == nullptr || split || obc) k = 1;
    const int mext = std::min(min_rank_extent(dims->LLm, dims->np_xi), min_rank_extent(dims->MMm, dims->np_eta));
    while (k > 1 && mext < 2 * k + 2) k--;
    const int gx = 2 * (k - 1);
    g.off = pad ? kAlignOff : 0;
    const int w = hx + 2 * gx;
    g.d.b = make_bounds(*dims, pad ? (w + kRowAlign - 1) / kRowAlign * kRowAlign : w, gx);
    g.hb = make_bounds(*dims, hx);
    g.d.p.s2d_k = k;
  }
  if (!buffer_span_ok(g.d.b)) {
    // checked before the device is touched (a host-only test calls this)
    g.err = "roms_gpu_init: subdomain too large for one GPU rank: a w-point field (n2*(N+1)*8 B) reaches 2 GiB, "
            "the limit of the kernels' 32-bit buffer offsets (k_common.h BufF64); split the grid over more ranks";
    return -1;
  }
  CHECK_HIP(hipSetDevice(device));
  g.d.b.nTS = g.hb.nTS = cfg->salinity ? 2 : 1;
  Params& P = g.d.p;
  {
    const int m = cfg->lmd_mixing, base = ROMS_LMD_MIXING | ROMS_LMD_KPP | ROMS_LMD_BKPP;
    if (m != 0 && ((m & ~(ROMS_LMD_ALL | ROMS_LMD_DDMIX)) || (m & base) != base ||
                   ((m & ROMS_LMD_CONVEC) && !(m & ROMS_LMD_RIMIX)) || ((m & ROMS_LMD_DDMIX) && !cfg->salinity))) {
      g.err = "roms_gpu_init: lmd_mixing must be 0 or LMD_MIXING|LMD_KPP|LMD_BKPP [|RIMIX|NONLOCAL|CONVEC(needs RIMIX)"
              "|DDMIX(needs SALINITY)]";
      return -1;
    }
  }
  P.nonlin_eos = cfg->nonlin_eos; P.salinity = cfg->salinity; P.lmd = cfg->lmd_mixing != 0;
  P.lmd_rimix = (cfg->lmd_mixing & ROMS_LMD_RIMIX) != 0;
  P.lmd_convec = (cfg->lmd_mixing & ROMS_LMD_CONVEC) != 0;
  P.lmd_nonlocal = (cfg->lmd_mixing & ROMS_LMD_NONLOCAL) != 0;
  P.lmd_ddmix = (cfg->lmd_mixing & ROMS_LMD_DDMIX) != 0;
  P.uv_adv = cfg->uv_adv != 0; P.uv_cor = cfg->uv_cor != 0;
  P.tides = cfg->pot_tides != 0;
  P.bulk_frc = cfg->bulk_frc != 0;
  P.iso = cfg->adv_isoneutral != 0;
  {
    // fused one-kernel prsgrd (k_prsgrd_fused): bit-identical, fewer bytes,
    // but measured slower at C2 (0.50 vs 0.38 ms per call: a per-level walk
    // of 2 blocks per CU hides less latency than the level-parallel grid)
    // and only 4% faster at C3 -- opt-in, ROMS_GPU_PRSGRD_FUSED=1
    const char* e = getenv("ROMS_GPU_PRSGRD_FUSED");
    P.prs_split = !(e && e[0] == '1');
  }
  P.uv_vis2 = cfg->uv_vis2; P.ts_dif2 = cfg->ts_dif2;
  {
    const char* e = getenv("ROMS_GPU_S2D_SPLIT");
    P.s2d_split = e && e[0] == '1';
  }
  P.dt = cfg->dt; P.dtfast = cfg->dt / (double)cfg->ndtfast; P.g = cfg->g; P.rho0 = cfg->rho0;
  P.vonKar = 0.41; P.qp2 = 0.0000172; P.gamma2 = cfg->gamma2; P.hc = cfg->hc;
  P.rdrg = cfg->rdrg; P.Zob = cfg->Zob; P.Tcoef = cfg->Tcoef; P.T0 = cfg->T0; P.Scoef = cfg->Scoef; P.S0 = cfg->S0;
  P.Akv_bak = cfg->Akv_bak; P.Akt_bak[0] = cfg->Akt_bak[0]; P.Akt_bak[1] = cfg->Akt_bak[1];
  P.npip = 0;
  if (cfg->obc < 0 || cfg->obc > 15) { g.err = "roms_gpu_init: obc must be a 4-bit edge mask"; return -1; }
  P.obc = cfg->obc & ((dims->ew_periodic ? 0 : 3) | (dims->ns_periodic ? 0 : 12));
  P.ubind = cfg->ubind;
  P.curvgrid = cfg->curvgrid && cfg->uv_adv;   // the curvature terms are part of UV_ADV
  if (P.obc) P.s2d_split = 1;  // open edges: separate zeta / zetabc / momentum kernels (step2d)
  for (int i = 0; i < kMaxFast; i++) { g.w1[i] = cfg->weight[0][i]; g.w2[i] = cfg->weight[1][i]; }
  // segment-partitioned column solvers (k_colseg.h) where the sequential
  // solvers' two LDS coefficient columns no longer fit (N > 63, up to 8
  // segments of 13 levels); the bit-exact sequential LDS solvers otherwise
  // (measured: at N = 50 the LDS sweep is faster, the partitioned solve
  // costs ~3x the VALU instructions per level).
  // ROMS_GPU_COLSEG=0/1 forces either (A/B and parity runs).
  // (every segment must hold at least kSegNMin rows: seg_rows_ok, k_colseg.h)
  const bool seg_fits = dims->N <= kSegRows * kSegMaxS && seg_rows_ok(dims->N);
  P.colseg = (size_t)2 * (dims->N + 1) * kCX * sizeof(double) > 64 * 1024 && seg_fits;
  {
    const char* e = getenv("ROMS_GPU_COLSEG");
    if (e && e[0] == '0') P.colseg = 0;
    if (e && e[0] == '1') P.colseg = seg_fits;
  }
  // register-resident sequential solvers (bit-exact) for the depths they are
  // compiled for; ROMS_GPU_COLREG=0 falls back to the LDS form (A/B runs)
  // bits: 1 step3d_uv1 (k_uv1_reg), 2 pre_step3d tracers (k_pre_tracer_v_reg);
  // ROMS_GPU_COLREG=<mask> (0: the LDS forms).  Measured at C2 (round 2):
  // bit 2 pre_step3d 2.06 -> 1.96 ms; bit 1 step3d_uv1 1.23 ms against 1.16
  // for the LDS form, so bit 1 is off by default.  (The LDS form once failed
  // the C2 100-step parity test in some test-process histories: that was the
  // zero fill of a new model's arrays racing with its first kernels, see
  // dev_alloc, not the solver; both forms are equal bitwise.)  Register
  // forms of pre_uv_col (2.06 -> 2.20 ms) and k_step3d_t_v (its extra
  // per-level KPP inputs spill at 2 waves/SIMD; 0.84 vs 0.81 ms at 1
  // wave/SIMD) were slower and are not kept.
  P.colreg = 2;
  {
    const char* e = getenv("ROMS_GPU_COLREG");
    if (e && e[0] >= '0' && e[0] <= '9') P.colreg = atoi(e);
  }
  P.uv2_fused = 1;
  {
    const char* e = getenv("ROMS_GPU_UV2_FUSED");
    if (e && e[0] == '0') P.uv2_fused = 0;
  }
  P.chain = 1;
  {
    const char* e = getenv("ROMS_GPU_CHAIN");
    if (e && e[0] == '0') P.chain = 0;
  }
  // order 3 in groups of 8 x-blocks: on 16-column blocks the resident
  // blocks of an XCD then cover 8 x 16 columns of consecutive rows, sharing
  // their i- and j-neighbour lines in L2 (pre_step3d 9.81-9.84 -> 9.61-9.65
  // ms, step3d_uv1 3.92-3.94 -> 3.81-3.83 ms per C3 call against order 0,
  // r5_x_seg_order_ab.txt)
  P.seg_order = 3;
  {
    const char* e = getenv("ROMS_GPU_SEG_ORDER");
    if (e && e[0] >= '0' && e[0] <= '3') P.seg_order = e[0] - '0';
  }
  P.seg_xg = 8;
  {
    const char* e = getenv("ROMS_GPU_SEG_XG");
    if (e && atoi(e) > 0) P.seg_xg = atoi(e);
  }
  {
    const char* e = getenv("ROMS_GPU_S2D_EDGES");
    P.s2d_fold = !(e && e[0] == '1');
  }
  {
    const char* e = getenv("ROMS_GPU_CHAIN_DIRZ");
    P.chain_dirz = !(e && e[0] == '0');   // set_HUV1 2.55 -> 2.03 ms at C3 (r3_s_chain_dirz_ab.txt)
  }
  {
    const char* e = getenv("ROMS_GPU_PRS_UV");
    P.prs_fuse_uv = !(e && e[0] == '0');
  }
  {
    const char* e = getenv("ROMS_GPU_TILE_GRP");
    P.tile_grp = e ? atoi(e) : 0;
  }
  {
    const char* e = getenv("ROMS_GPU_UV1_LDS");
    P.uv1_lds = !(e && e[0] == '0');
  }
  {
    const char* e = getenv("ROMS_GPU_P_IN_RHO");
    P.p_in_rho = !(e && e[0] == '0');
  }
  {
    const char* e = getenv("ROMS_GPU_OMEGA_HB");
    P.omega_hb = !(e && e[0] == '0');
  }
  {
    const char* e = getenv("ROMS_GPU_OMEGA_SEG");
    P.omega_seg = !(e && e[0] == '0');
  }
  {
    // 16-column blocks (four segments per wavefront, 4 blocks per CU) with
    // the k-order chain: omega 1.41 -> 1.24 ms per C3 call, as fast as the
    // parallel partial sums and bitwise to the 64-column form
    // (r5_w_omega_cw_par_ab.txt)
    // (at N <= 63, C2, 64 columns stay: 0.161 against 0.167 ms per call)
    const char* e = getenv("ROMS_GPU_OMEGA_CW");
    const int v = e ? atoi(e) : (dims->N > 63 ? 16 : 64);
    P.omega_cw = v == 32 || v == 64 ? v : 16;
    e = getenv("ROMS_GPU_OMEGA_ORD");
    P.omega_ord = e && e[0] >= '1' && e[0] <= '3' ? e[0] - '0' : 0;
    e = getenv("ROMS_GPU_OMEGA_PAR");
    P.omega_par = e && e[0] == '1';
  }
  {
    const char* e = getenv("ROMS_GPU_PREUV_LDS");
    P.preuv_lds = !(e && e[0] == '0');
  }
  {
    const char* e = getenv("ROMS_GPU_HTY");
    P.h_ty = (e && atoi(e) == 8) ? 8 : 4;
  }
  {
    // j-marching per-level horizontal kernels: rows per block (ROMS_GPU_HJC;
    // 0 = off, the default: k_pre_tracer_hj measured slower at C3, 12.15 ->
    // 12.65 ms per pre_step3d, r4c: the 64 x 4 tiles' j-halo rows are mostly
    // L2 hits already (PMC 16.2 passes against 14), and the ring's in-flight
    // rows and lanes halve the waves per SIMD)
    const char* e = getenv("ROMS_GPU_HJC");
    P.h_jc = 0;
    if (e && atoi(e) >= 0) P.h_jc = atoi(e) / 4 * 4;
  }
  {
    const char* e = getenv("ROMS_GPU_PRS_TY");
    P.prs_ty = (e && atoi(e) == 8) ? 8 : 4;
  }
  {
    // 16-B window loads (they need every row's i0-2 on a 16-B boundary: the
    // padded device pitch, g.off, gives that, roms_dev.h) measured slower at
    // C3 (k_prsgrd_uv 4.20-4.26 vs 3.96 ms per call, same box, the 8-B form
    // with a 67-wide window 3.6 ms): opt-in, ROMS_GPU_LD16=1
    const char* e = getenv("ROMS_GPU_LD16");
    P.ld16 = g.off != 0 && e && e[0] == '1';
  }
  {
    // visc3d with staged raw windows (bitwise): C3 2.34 -> 1.94 ms, C2 0.35 -> 0.30 ms
    // (r3_zq_visc_stg_ab.txt); ROMS_GPU_VISC_STG=0 for per-point loads
    const char* e = getenv("ROMS_GPU_VISC_STG");
    P.visc_stg = !(e && e[0] == '0');
  }
  {
    // t3dmix with staged windows (bitwise): C3 1.65 -> 1.31 ms, C2 0.218 -> 0.145 ms
    // (r3_zs_t3dmix_stg_ab.txt); ROMS_GPU_T3DMIX_STG=0 for per-point loads
    const char* e = getenv("ROMS_GPU_T3DMIX_STG");
    P.t3dmix_stg = !(e && e[0] == '0');
  }
  {
    // staged Rig windows in k_kpp_int (bitwise): lmd_vmix 3.49 -> 3.22 ms per
    // call at C3 (r3_zp_kpp_ty_ab.txt); ROMS_GPU_KPP_TY=0 for one row per block
    const char* e = getenv("ROMS_GPU_KPP_TY");
    P.kpp_ty = 4;
    if (e && (atoi(e) == 0 || atoi(e) == 2 || atoi(e) == 8 || atoi(e) == 43)) P.kpp_ty = atoi(e);
  }
  {
    const char* e = getenv("ROMS_GPU_HOIST");
    P.hoist = !(e && e[0] == '0');
  }
  {
    // default on: C3 prsgrd 3.62-3.63 -> 3.55 ms per call (r5_d_seg_buf_chunk_prs_ab.txt)
    const char* e = getenv("ROMS_GPU_PRS_BUF");
    P.prs_buf = !(e && e[0] == '0');
  }
  {
    // prsgrd's ru/rv with the momentum r.h.s. in j-marching strips (one
    // evaluation per face, neighbours through DPP lane shifts; bitwise equal
    // to the k_prsgrd_uv tiles); ROMS_GPU_PRS_STRIP=0: tiles everywhere
    const char* e = getenv("ROMS_GPU_PRS_STRIP");
    P.prs_strip = !(e && e[0] == '0');
  }
  {
    // horizontal tracer advection of pre_step3d / step3d_t in j-marching
    // strips (k_tracer_strip, bitwise equal to the k_*_h1 tiles): measured
    // slower at C3 (pre_step3d 9.65 -> 10.56, step3d_t 4.75 -> 5.66 ms per
    // call, profiles/r6_e_tracer_strip_ab.txt: too little arithmetic per row
    // to cover each row's loads), so opt-in, ROMS_GPU_T_STRIP=1
    const char* e = getenv("ROMS_GPU_T_STRIP");
    P.t_strip = e && e[0] == '1';
  }
  {
    const char* e = getenv("ROMS_GPU_TCHUNK");
    P.t_chunk = e ? atoi(e) : 0;
    if (P.t_chunk < 0) P.t_chunk = 0;
  }
  {
    const char* e = getenv("ROMS_GPU_SEG_BUF");
    // bits: 1 k_pre_tracer_segb, 2 k_step3d_t_segb, 4 its t(nnew) prefetch,
    // 8 its Hz reload, 16 k_pre_tracer_segb's prefetch, 32 k_uv1_segb, 64 its
    // u(nnew) prefetch, 128 k_pre_uv_segb, 256 its Hz_fwd prefetch, 512 the
    // momentum solvers' buffer forms without seg_uniform (level offsets in
    // the VGPR offset), 1024 the same for the tracer solvers.  Default 679
    // (7 + the momentum solvers' buffer forms with VGPR level offsets):
    // pre_step3d 11.24-11.31 -> 10.88-11.08 ms, step3d_uv1 4.63 -> 4.50-4.53
    // (profiles/r5_l_seg_buf_vgpr_ab.txt)  Default 7: C3
    // 57.4-57.7 -> 56.7 ms/step, step3d_t 5.98 -> 5.75 ms, pre_step3d
    // 11.5 -> 11.3 ms (same box, profiles/r5_c_seg_buf_ab.txt); the momentum
    // solvers' buffer forms (32, 128, + prefetch) measured slower (step3d_uv1
    // 4.6 -> 6.0-6.6 ms, pre_step3d +0.3-2.1 ms: r5_d_seg_buf_chunk_prs_ab.txt)
    P.seg_buf = e ? atoi(e) : 679;
  }
  {
    const char* e = getenv("ROMS_GPU_SEG_VTILE");
    P.seg_vtile = !(e && e[0] == '0');
  }
  P.seg_jrows = kSegJMax < 2 ? kSegJMax : 2;
  {
    const char* e = getenv("ROMS_GPU_SEG_JROWS");
    if (e && atoi(e) >= 1 && atoi(e) <= kSegJMax) P.seg_jrows = atoi(e);
  }
  // column-solver scratch: LDS while two (N+1)-level slots per wave fit the
  // default 64 KB (N < 63), global memory for deeper grids;
  // ROMS_GPU_COL_GLOBAL=1/0 forces either (A/B runs)
  bool col_global = (size_t)2 * (dims->N + 1) * kCX * sizeof(double) > 64 * 1024;
  {
    const char* e = getenv("ROMS_GPU_COL_GLOBAL");
    if (e && e[0] == '1') col_global = true;
    if (e && e[0] == '0') col_global = false;
  }
  setup_uv1_seg();
  setup_pre_uv_seg();
  setup_omega_seg();
  if (!col_global && !setup_column_kernels(dims->N)) {
    g.err = "roms_gpu_init: N too large for the LDS column kernels (2*(N+1)*512 B > 160 KB)";
    return -2;
  }
  CHECK_HIP(hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking));
  CHECK_HIP(hipStreamCreateWithFlags(&g.s2, hipStreamNonBlocking));
  for (hipEvent_t& e : g.pev) CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  {
    // measured slower than one stream (C3 60.5 -> 62.5, C2 6.40 -> 6.46 ms per
    // step, profiles/r4_j_two_stream_ab.txt): the concurrent kernels compete
    // for CUs and LDS (the segment solvers hold one block per CU), so the
    // second stream is opt-in, ROMS_GPU_PAR=1
    const char* e = getenv("ROMS_GPU_PAR");
    const char* em = getenv("ROMS_GPU_PAR_MASK");
    g.par = e && e[0] == '1' ? 31 : 0;
    if (em) g.par = atoi(em) & 31;
  }
  {
    const char* e = getenv("ROMS_GPU_GUARD");
    g.guard = e && e[0] == '1';
  }
  const Bounds& b = g.d.b;
  // the 2-D fields first and next to each other (then the 2-D scratch), so
  // that the fast step's fields share one buffer window (S2dWin below)
  auto field = [&](int id) -> int {
    const long n = field_count(id, b);
    double* p = nullptr;
    CHECK_HIP(dev_alloc(p, n));
    g.f[id].d = p;
    g.f[id].count = n;
    g.f[id].hcount = field_count(id, g.hb);
    g.f[id].planar = planar_field(id);
    *field_slot(g.d.f, id) = p;
    return 0;
  };
  auto planar2d = [&](int id) { return planar_field(id) && field_count(id, b) <= 4 * b.n2; };
  {
    // one allocation for them (dev_alloc slices it); a subdomain whose 2-D
    // set passes 2 GiB allocates them one by one (and runs the pointer form)
    long n = 10 * dev_alloc_size(b.n2);   // s0..s9
    for (int id = 0; id < ROMS_NFIELDS; id++)
      if (planar2d(id)) n += dev_alloc_size(field_count(id, b));
    if (n * 8 < 2147483648L - (1L << 20)) {
      CHECK_HIP(hipMalloc(&g.arena, (size_t)n * sizeof(double)));
      g.arena_n = n;
      g.arena_used = 0;
    }
  }
  for (int id = 0; id < ROMS_NFIELDS; id++)
    if (planar2d(id) && field(id)) return -2;
  auto scratch = [&](double*& p, long n) -> int {
    CHECK_HIP(dev_alloc(p, n));
    g.scratch.push_back(p);
    return 0;
  };
  Fields& F = g.d.f;
  double** s2[] = {&F.s0, &F.s1, &F.s2, &F.s3, &F.s4, &F.s5, &F.s6, &F.s7, &F.s8, &F.s9};
  for (double** q : s2)
    if (scratch(*q, b.n2)) return -2;
  g.arena_n = g.arena_used;   // nothing else is sliced from it
  for (int id = 0; id < ROMS_NFIELDS; id++)
    if (!planar2d(id) && field(id)) return -2;
  if (scratch(F.P, b.n3) || scratch(F.rhos, b.n3) || scratch(F.c0, b.n3w) || scratch(F.c1, b.n3w) ||
      scratch(F.c2, b.n3w) || scratch(F.c3, b.n3w))
    return -2;
  {
    // the fast step's buffer window (k_s2d_fb): every field's origin IJ = -lead
    // and its last element within 2 GiB of one base; else (or with
    // ROMS_GPU_S2D_WIN=0) the kernel addresses them through their pointers
    const char* e = getenv("ROMS_GPU_S2D_WIN");
    g.d.w2 = S2dWin{};
    const double* wp[kWinN] = {F.zeta,  F.ubar,  F.vbar,    F.h,       F.dn_u,    F.dm_v,       F.pm,
                               F.pn,    F.swflx, F.rmask,   F.rhoS,    F.rhoA,    F.umask,      F.vmask,
                               F.rufrc, F.rvfrc, F.DU_avg1, F.DV_avg1, F.DU_avg2, F.DV_avg2,    F.Zt_avg1,
                               F.DU_avg_bak, F.DV_avg_bak, F.s0, F.s1};
    const long lead = (long)b.gx * b.nx2 + b.gx + kRowAlign;   // below the lowest IJ the kernel forms
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (int f = 0; f < kWinN; f++) {
      const long cnt = f <= kW_vbar ? 4 * b.n2 : b.n2;
      lo = std::min(lo, (uintptr_t)wp[f] - (uintptr_t)lead * 8u);
      hi = std::max(hi, (uintptr_t)wp[f] + (uintptr_t)cnt * 8u);
    }
    if (!(e && e[0] == '0') && hi - lo < (uintptr_t)2147483648u - (1u << 20)) {
      g.d.w2.base = (const double*)lo;
      g.d.w2.lead = (int)lead;
      for (int f = 0; f < kWinN; f++) g.d.w2.off[f] = (unsigned)((uintptr_t)wp[f] - (uintptr_t)lead * 8u - lo);
    }
  }
  if (col_global && scratch(F.colscr, 2L * (b.NT > 2 ? b.NT : 2) * b.n3w)) return -2;
  if (P.iso) {   // ADV_ISONEUTRAL fields (k_iso.hip), zero like the reference's allocations (eos_vars.F:50-52)
    double** r3[] = {&F.dRdx, &F.dRde, &F.diff3u, &F.diff3v, &F.iso_dTdx, &F.iso_dTde, &F.iso_LapT};
    for (double** q : r3)
      if (scratch(*q, b.n3)) return -2;
    double** w3[] = {&F.idRz, &F.Akz, &F.iso_dTdz, &F.iso_FSC};
    for (double** q : w3)
      if (scratch(*q, b.n3w)) return -2;
  }
  if (P.lmd) {
    if (scratch(F.lmd_rig, b.n3w)) return -2;
    double** l2[] = {&F.lmd_hbl, &F.lmd_bbl, &F.lmd_Bo, &F.lmd_Bosol, &F.lmd_ustar};
    for (double** q : l2)
      if (scratch(*q, b.n2)) return -2;
  }
  {
    // step3d_uv2's closed-edge columns in the chain form (k_uv2_edge): C3
    // uv2 3.93 -> 3.39 ms, step 60.8 -> 59.7 ms same box
    // (profiles/r4_p_uv2_edge_colreg_ab.txt); ROMS_GPU_UV2_EDGE=0: the
    // one-lane edge mode
    const char* e = getenv("ROMS_GPU_UV2_EDGE");
    std::vector<int> lc, lf;
    if (!(e && e[0] == '0')) uv2_edge_lists(b, lc, lf);
    if (!lc.empty() && !lf.empty()) {
      CHECK_HIP(hipMalloc(&F.uv2e_couple, lc.size() * sizeof(int)));
      CHECK_HIP(hipMalloc(&F.uv2e_flux, lf.size() * sizeof(int)));
      CHECK_HIP(copy_on(F.uv2e_couple, lc.data(), lc.size() * sizeof(int), hipMemcpyHostToDevice, g.s));
      CHECK_HIP(copy_on(F.uv2e_flux, lf.data(), lf.size() * sizeof(int), hipMemcpyHostToDevice, g.s));
      P.uv2e_nc = (int)(lc.size() / 3);
      P.uv2e_nf = (int)(lf.size() / 3);
    }
  }
  CHECK_HIP(hipHostMalloc(&g.h_diag, 8 * sizeof(double), hipHostMallocDefault));
  CHECK_HIP(hipMalloc(&g.d_diag, 8 * sizeof(double)));
  if (comm != nullptr) {
    HaloPlan plan = halo_plan(dims->Lm, dims->Mm, dims->np_xi, dims->np_eta, dims->inode, dims->jnode,
                              dims->ew_periodic, dims->ns_periodic);
    plan.g.nx2 = b.nx2;   // the device row pitch: pack/unpack index the device arrays
    plan.g.n2 = b.n2;
    HaloPlan wide{};
    if (P.s2d_k > 1) {
      wide = halo_plan(dims->Lm, dims->Mm, dims->np_xi, dims->np_eta, dims->inode, dims->jnode, dims->ew_periodic,
                       dims->ns_periodic, 2 * P.s2d_k);
      wide.g.nx2 = b.nx2;
      wide.g.n2 = b.n2;
    }
    const int r = halo_setup(g.halo, (RomsComm*)comm, plan, 8 * (dims->N + 1), wide, kExchMax, g.err);
    if (r) return r;
    g.halo.ls = g.s;
    g.d.halo = &g.halo;
  }
  {
    const char* e = getenv("ROMS_GPU_HZ_UV");
    g.hzuv_env = e && e[0] == '1';
    g.hzuv_valid = true;
  }
  const char* env = getenv("ROMS_GPU_NO_GRAPH");
  g.use_graphs = !(env && env[0] == '1') && halo_graph_safe(g.d.halo);
  env = getenv("ROMS_GPU_RHO_REUSE");
  g.rho_reuse = !(env && env[0] == '0');
  g.rho_slot = 0;
  g.inited = true;
  return 0;
}

int roms_gpu_finalize(void) {
  if (g.inited) {
    (void)hipStreamSynchronize(g.s);
    free_all();
  }
  return 0;
}

long roms_gpu_field_size(int id) {
  if (!g.inited || id < 0 || id >= ROMS_NFIELDS) return -1;
  return g.f[id].hcount;
}

int roms_gpu_register(int id, double* host, long count) {
  REQUIRE_INIT();
  if (id < 0 || id >= ROMS_NFIELDS) { g.err = "roms_gpu_register: bad field id"; return -1; }
  if (count != g.f[id].hcount) { g.err = "roms_gpu_register: size mismatch for field"; return -1; }
  g.f[id].host = host;
  g.f[id].host_count = count;
  return 0;
}

// Hz_u/Hz_v after whole steps that did not store them (see Global::hzuv_valid)
static bool hzuv_readable(int id) {
  if ((id != ROMS_Hz_u && id != ROMS_Hz_v) || g.hzuv_valid) return true;
  g.err = "Hz_u/Hz_v are not maintained by whole steps unless registered for transfer or ROMS_GPU_HZ_UV=1 "
          "(extract_data inputs, set_depth.F:220,227)";
  return false;
}
static int xfer(int id, bool up) {
  if (id == ROMS_ALL) {
    for (int q = 0; q < ROMS_NFIELDS; q++)
      if (g.f[q].host) {
        const int r = xfer(q, up);
        if (r) return r;
      }
    return 0;
  }
  if (id < 0 || id >= ROMS_NFIELDS) { g.err = "bad field id"; return -1; }
  if (!g.f[id].host) { g.err = "field not registered"; return -1; }
  if (!up && !hzuv_readable(id)) return -5;
  if (up && (id == ROMS_Hz_u || id == ROMS_Hz_v)) g.hzuv_valid = true;
  CHECK_HIP(up ? field_h2d(id, g.f[id].d, g.f[id].host) : field_d2h(id, g.f[id].host, g.f[id].d));
  return 0;
}
int roms_gpu_upload(int id) { REQUIRE_INIT(); return xfer(id, true); }
int roms_gpu_download(int id) { REQUIRE_INIT_RO(); return xfer(id, false); }

int roms_gpu_copy_in(int id, const double* src, long count) {
  REQUIRE_INIT();
  if (id < 0 || id >= ROMS_NFIELDS || count != g.f[id].hcount) { g.err = "roms_gpu_copy_in: bad field/size"; return -1; }
  if (id == ROMS_Hz_u || id == ROMS_Hz_v) g.hzuv_valid = true;
  CHECK_HIP(field_h2d(id, g.f[id].d, src));
  return 0;
}
int roms_gpu_copy_out(int id, double* dst, long count) {
  REQUIRE_INIT_RO();
  if (id < 0 || id >= ROMS_NFIELDS || count != g.f[id].hcount) { g.err = "roms_gpu_copy_out: bad field/size"; return -1; }
  if (!hzuv_readable(id)) return -5;
  CHECK_HIP(field_d2h(id, dst, g.f[id].d));
  REQUIRE_HALO_OK();
  return 0;
}
int roms_gpu_sync(void) {
  REQUIRE_INIT_RO();
  CHECK_HIP(hipStreamSynchronize(g.s));
  REQUIRE_HALO_OK();
  return post_launch();
}

#define ROUTINE(name, call)           \
  int name(const roms_tlev* t) {      \
    REQUIRE_INIT();                   \
    const Tlev T = to_tlev(t);        \
    call;                             \
    return post_launch();             \
  }
ROUTINE(roms_gpu_set_huv, (launch_set_huv(g.d, g.s, T), g.hzuv_valid = true))
ROUTINE(roms_gpu_omega, launch_omega(g.d, g.s, T))
ROUTINE(roms_gpu_prsgrd, launch_prsgrd(g.d, g.s, T))
ROUTINE(roms_gpu_pre_step3d, launch_pre_step3d(g.d, g.s, T))
ROUTINE(roms_gpu_set_huv1, launch_set_huv1(g.d, g.s, T))
ROUTINE(roms_gpu_step3d_uv1, launch_step3d_uv1(g.d, g.s, T))
ROUTINE(roms_gpu_visc3d, launch_visc3d(g.d, g.s, T))
ROUTINE(roms_gpu_step3d_uv2, launch_step3d_uv2(g.d, g.s, T))
ROUTINE(roms_gpu_step3d_t, launch_step3d_t(g.d, g.s, T))
ROUTINE(roms_gpu_t3dmix, launch_t3dmix(g.d, g.s, T))
ROUTINE(roms_gpu_set_depth, launch_set_depth(g.d, g.s, T))
#undef ROUTINE

int roms_gpu_halo_transport(void) {
  REQUIRE_INIT_NOJOIN();
  return g.d.halo ? halo_transport(g.halo) : 0;
}

int roms_gpu_halo_overlap(void) {
  REQUIRE_INIT_NOJOIN();
  return g.d.halo && g.halo.xoverlap > 0 ? 1 : 0;
}

int roms_gpu_s2d_window(void) {
  REQUIRE_INIT_NOJOIN();
  return g.d.w2.base ? 1 : 0;
}

int roms_gpu_halo_exchanges(long* per_step, int* fast_interval) {
  REQUIRE_INIT_NOJOIN();
  if (per_step) *per_step = g.step_exch;
  if (fast_interval) *fast_interval = g.d.p.s2d_k;
  return 0;
}

int roms_gpu_step2d(const roms_tlev* t) {
  REQUIRE_INIT_NOJOIN();   // keeps the previous fast step's exchange in flight
  REQUIRE_HALO_OK();
  const Tlev T = to_tlev(t);
  launch_step2d(g.d, g.s, T, g.w1, g.w2);
  return post_launch();
}

int roms_gpu_rho_eos(int tidx, const roms_tlev* t) {
  REQUIRE_INIT();
  launch_rho_eos(g.d, g.s, to_tlev(t), tidx);
  return post_launch();
}
int roms_gpu_lmd_vmix(int tind, const roms_tlev* t) {
  REQUIRE_INIT();
  if (!g.cfg.lmd_mixing) { g.err = "roms_gpu_lmd_vmix: library initialised without lmd_mixing"; return -4; }
  if (tind < 1 || tind > 3) { g.err = "roms_gpu_lmd_vmix: bad time index"; return -1; }
  launch_lmd_vmix(g.d, g.s, to_tlev(t), tind);
  return post_launch();
}
int roms_gpu_swr_frac(const roms_tlev* t) {
  (void)t;
  REQUIRE_INIT();
  launch_swr_frac(g.d, g.s);
  g.have_swr = true;
  return post_launch();
}
int roms_gpu_set_pipe_frc(int npip, const int* pipe_idx, const double* pipe_flx, const double* pipe_prf,
                          const double* pipe_trc) {
  REQUIRE_INIT();
  const Bounds& b = g.d.b;
  Fields& F = g.d.f;
  if (npip < 0 || (npip > 0 && (!pipe_idx || !pipe_flx || !pipe_prf || !pipe_trc))) {
    g.err = "roms_gpu_set_pipe_frc: bad argument";
    return -1;
  }
  if (npip == 0) { g.d.p.npip = 0; return 0; }
  for (long q = 0; q < g.hb.n2; q++)
    if (pipe_idx[q] < 0 || pipe_idx[q] > npip) { g.err = "roms_gpu_set_pipe_frc: pipe_idx out of 0..npip"; return -1; }
  CHECK_HIP(hipStreamSynchronize(g.s));
  if (npip != g.d.p.npip || !F.pipe_idx) {
    // (re)allocate; captured graphs hold the old pointers
    for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
    g.graphs.clear();
    if (F.pipe_idx) (void)hipFree(F.pipe_idx);
    F.pipe_idx = nullptr;
    // free the previous pipe arrays (they are tracked in g.scratch)
    for (double** q : {&F.pipe_flx, &F.pipe_prf, &F.pipe_trc}) {
      if (!*q) continue;
      for (size_t k = 0; k < g.scratch.size(); k++)
        if (g.scratch[k] == *q) { g.scratch.erase(g.scratch.begin() + (long)k); break; }
      (void)hipFree(dev_base(*q));
      *q = nullptr;
    }
    g.d.p.npip = 0;
    CHECK_HIP(hipMalloc(&F.pipe_idx, (size_t)b.n2 * sizeof(int)));
    auto scratch = [&](double*& p, long n) -> int {
      CHECK_HIP(hipMalloc(&p, (size_t)n * sizeof(double)));
      g.scratch.push_back(p);
      return 0;
    };
    if (scratch(F.pipe_flx, b.n2) || scratch(F.pipe_prf, (long)npip * b.N) || scratch(F.pipe_trc, (long)npip * b.NT))
      return -2;
    g.d.p.npip = npip;
  }
  {
    const std::vector<int> di = to_dev_layout(pipe_idx, 1);
    const std::vector<double> df = to_dev_layout(pipe_flx, 1);
    CHECK_HIP(copy_on(F.pipe_idx, di.data(), (size_t)b.n2 * sizeof(int), hipMemcpyHostToDevice, g.s));
    CHECK_HIP(copy_on(F.pipe_flx, df.data(), (size_t)b.n2 * sizeof(double), hipMemcpyHostToDevice, g.s));
  }
  CHECK_HIP(copy_on(F.pipe_prf, pipe_prf, (size_t)npip * b.N * sizeof(double), hipMemcpyHostToDevice, g.s));
  CHECK_HIP(copy_on(F.pipe_trc, pipe_trc, (size_t)npip * b.NT * sizeof(double), hipMemcpyHostToDevice, g.s));
  return 0;
}

int roms_gpu_set_river_frc(int nriv, const double* riv_uflx, const double* riv_vflx, const double* riv_vol,
                           const double* riv_trc) {
  REQUIRE_INIT();
  const Bounds& b = g.d.b;
  Fields& F = g.d.f;
  if (nriv < 0 || nriv > 4096 || (nriv > 0 && (!riv_vol || !riv_trc)) || (!riv_uflx) != (!riv_vflx)) {
    g.err = "roms_gpu_set_river_frc: bad argument";
    return -1;
  }
  CHECK_HIP(hipStreamSynchronize(g.s));
  auto drop_graphs = [&]() {   // captured graphs hold the old Params / pointers
    for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
    g.graphs.clear();
  };
  if (nriv == 0) {
    if (g.d.p.nriv) drop_graphs();
    g.d.p.nriv = 0;
    return 0;
  }
  if (!riv_uflx && !F.riv_uflx) { g.err = "roms_gpu_set_river_frc: river faces never set"; return -1; }
  // faces kept from an earlier call index riv_vol/riv_trc up to riv_maxidx:
  // a smaller nriv without new faces would read past the new arrays
  if (!riv_uflx && nriv < g.riv_maxidx) {
    g.err = "roms_gpu_set_river_frc: nriv smaller than the largest river index of the faces on the device "
            "(pass riv_uflx/riv_vflx again)";
    return -1;
  }
  // faces of calc_river_flux: |riv_flx| > 1e-3 (step2d_FB.F:534), river index nint(riv_flx/10)
  std::vector<int> faces;
  long maxidx = 0;
  if (riv_uflx) {
    for (int dir = 0; dir < 2; dir++) {
      const double* a = dir == 0 ? riv_uflx : riv_vflx;
      for (int j = -1; j <= b.Mm + 2; j++)
        for (int i = -1; i <= b.Lm + 2; i++) {
          const double v = a[IJ(g.hb, i, j)];   // the host's layout
          if (!(std::fabs(v) > 1e-3)) continue;
          const long ir = std::lround(v / 10);
          if (ir < 1 || ir > nriv) { g.err = "roms_gpu_set_river_frc: river index nint(riv_flx/10) out of 1..nriv"; return -1; }
          faces.push_back(dir); faces.push_back(i); faces.push_back(j);
          if (ir > maxidx) maxidx = ir;
        }
    }
  }
  auto release = [&](double*& p) {
    if (!p) return;
    for (size_t k = 0; k < g.scratch.size(); k++)
      if (g.scratch[k] == p) { g.scratch.erase(g.scratch.begin() + (long)k); break; }
    (void)hipFree(dev_base(p));
    p = nullptr;
  };
  auto scratch = [&](double*& p, long n) -> int {
    CHECK_HIP(hipMalloc(&p, (size_t)n * sizeof(double)));
    g.scratch.push_back(p);
    return 0;
  };
  if (nriv != g.d.p.nriv || !F.riv_vol) {
    drop_graphs();
    release(F.riv_vol);
    release(F.riv_trc);
    if (scratch(F.riv_vol, nriv) || scratch(F.riv_trc, (long)nriv * b.NT)) return -2;
  }
  if (riv_uflx) {
    drop_graphs();
    if (!F.riv_uflx && (scratch(F.riv_uflx, b.n2) || scratch(F.riv_vflx, b.n2))) return -2;
    if (F.riv_face) { (void)hipFree(F.riv_face); F.riv_face = nullptr; }
    CHECK_HIP(hipMalloc(&F.riv_face, (faces.size() ? faces.size() : 1) * sizeof(int)));
    if (!faces.empty()) CHECK_HIP(copy_on(F.riv_face, faces.data(), faces.size() * sizeof(int), hipMemcpyHostToDevice, g.s));
    CHECK_HIP(rows_h2d(F.riv_uflx, riv_uflx, b.Mm + 4));
    CHECK_HIP(rows_h2d(F.riv_vflx, riv_vflx, b.Mm + 4));
    g.d.p.nrivf = (int)(faces.size() / 3);
    g.riv_maxidx = maxidx;
  }
  CHECK_HIP(copy_on(F.riv_vol, riv_vol, (size_t)nriv * sizeof(double), hipMemcpyHostToDevice, g.s));
  CHECK_HIP(copy_on(F.riv_trc, riv_trc, (size_t)nriv * b.NT * sizeof(double), hipMemcpyHostToDevice, g.s));
  g.d.p.nriv = nriv;
  return 0;
}

int roms_gpu_set_ub_tune(const double* ub_west, const double* ub_east, const double* ub_south, const double* ub_north) {
  REQUIRE_INIT();
  const double* src[4] = {ub_west, ub_east, ub_south, ub_north};
  const Bounds& b = g.d.b;
  // graphs captured with other ub pointers would keep using them
  for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
  g.graphs.clear();
  for (int q = 0; q < 4; q++) {
    double*& p = g.d.f.ub[q];
    if (!src[q]) {
      if (p) { CHECK_HIP(hipStreamSynchronize(g.s)); (void)hipFree(p); p = nullptr; }
      continue;
    }
    const long n = q < 2 ? b.Mm + 2 : b.Lm + 2;
    if (!p) CHECK_HIP(hipMalloc(&p, (size_t)n * sizeof(double)));
    CHECK_HIP(hipMemcpyAsync(p, src[q], (size_t)n * sizeof(double), hipMemcpyHostToDevice, g.s));
  }
  CHECK_HIP(hipStreamSynchronize(g.s));
  return 0;
}

int roms_gpu_bulk_flux(const roms_tlev* t) {
  REQUIRE_INIT();
  if (!g.d.p.bulk_frc) { g.err = "roms_gpu_bulk_flux: library initialised without bulk_frc"; return -4; }
  if (t->nrhs < 1 || t->nrhs > 3) { g.err = "roms_gpu_bulk_flux: bad time index"; return -1; }
  launch_bulk_flux(g.d, g.s, t->nrhs);
  return post_launch();
}

int roms_gpu_step(roms_tlev* t) {
  REQUIRE_INIT_RO();
  g.rho_slot = 0;
  t->iic = t->iic + 1;
  t->nstp = 1 + (t->iic - t->ntstart) % 2;
  t->nrhs = t->nstp;
  t->nnew = 3;
  t->nfast = g.cfg.nfast;
  const bool rho_current = g.rho_reuse && rho_keep_ == t->nrhs;
  {
    // in-step forcing weights of this step (roms_gpu_frc_clock), queued ahead of its kernels
    const int r = frc_step_prepare(g.s, g.d, g.cfg.dt, *t, g.err);
    if (r) return r;
    const long gen = frc_step_gen();
    if (gen != g.graph_frc_gen) {   // graphs captured with other forcing buffers / field lists
      CHECK_HIP(hipStreamSynchronize(g.s));
      for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
      g.graphs.clear();
      g.graph_frc_gen = gen;
    }
  }
  const bool first = (t->iic == t->forw_start);
  const bool store_huv = g.hzuv_env || g.f[ROMS_Hz_u].host != nullptr || g.f[ROMS_Hz_v].host != nullptr;
  g.hzuv_valid = store_huv;
  if (!g.use_graphs || first) {
    enqueue_step(t, rho_current, store_huv);
    return post_launch();
  }
  const long key = (long)t->nstp * 16 + t->knew + (rho_current ? 256 : 0) + (store_huv ? 512 : 0);
  auto it = g.graphs.find(key);
  roms_tlev t0 = *t;
  if (it == g.graphs.end()) {
    hipGraph_t graph;
    CHECK_HIP(hipStreamBeginCapture(g.s, hipStreamCaptureModeThreadLocal));
    enqueue_step(t, rho_current, store_huv);
    CHECK_HIP(hipStreamEndCapture(g.s, &graph));
    hipGraphExec_t exec;
    CHECK_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CHECK_HIP(hipGraphDestroy(graph));
    g.graphs[key] = exec;
    it = g.graphs.find(key);
    *t = t0;
  }
  // replay; advance the host-side indices exactly as enqueue_step would
  CHECK_HIP(hipGraphLaunch(it->second, g.s));
  t->nrhs = 3;
  t->nnew = 3 - t->nstp;
  g.rho_slot = t->nnew;   // the replayed step ended with rho_eos(nnew)
  for (int iif = 1; iif <= t->nfast; iif++) {
    t->iif = iif;
    t->kstp = t->knew;
    t->knew = t->kstp + 1;
    if (t->knew > 4) t->knew = 1;
  }
  return post_launch();
}

int roms_gpu_init_sequence(roms_tlev* t) {
  REQUIRE_INIT();
  const Tlev T = to_tlev(t);
  launch_set_depth(g.d, g.s, T);
  // main.F:217-220 (zeta at rest): at initialisation only, not after a
  // restart read (get_init leaves iic = ntstart - 1 > 0)
  if (g.cfg.lmd_mixing && t->iic == 0) {
    launch_swr_frac(g.d, g.s);
    g.have_swr = true;
  }
  if (g.cfg.lmd_mixing && !g.have_swr) {
    // after get_init the depths are no longer the rest state swr_frac is formed on
    g.err = "roms_gpu_init_sequence: swr_frac was never formed; call roms_gpu_swr_frac after set_depth at rest "
            "and before roms_gpu_get_init (main.F:216-220)";
    return -4;
  }
  launch_set_huv(g.d, g.s, T);
  g.hzuv_valid = true;
  launch_omega(g.d, g.s, T);
  launch_rho_eos(g.d, g.s, T, T.nrhs);
  return post_launch();
}

static int init_case_impl(const roms_case* c, int np_xi, int np_eta, void* comm, int device, roms_tlev* t) {
  if (!c || !t) { g.err = "roms_gpu_init_case: null argument"; return -1; }
  if (np_xi < 1 || np_eta < 1) { g.err = "roms_gpu_init_case: bad processor grid"; return -1; }
  const int rank = comm ? comm_rank((RomsComm*)comm) : 0;
  roms_dims D{};
  D.N = c->N; D.NT = c->NT; D.LLm = c->LLm; D.MMm = c->MMm;
  D.np_xi = np_xi; D.np_eta = np_eta;
  D.jnode = rank / np_xi;              // mpi_setup.F:60-61
  D.inode = rank - D.jnode * np_xi;
  rank_extent(c->LLm, np_xi, D.inode, D.Lm, D.iSW_corn);
  rank_extent(c->MMm, np_eta, D.jnode, D.Mm, D.jSW_corn);
  if (c->case_id < ROMS_CASE_FILAMENT || c->case_id > ROMS_CASE_RIVERS) { g.err = "roms_gpu_init_case: unknown case"; return -1; }
  const bool fil = c->case_id == ROMS_CASE_FILAMENT;
  // Rivers_ana shares Pipes_ana's physics and benchmark.in coefficients
  const bool pipes = c->case_id == ROMS_CASE_PIPES || c->case_id == ROMS_CASE_RIVERS;
  D.ew_periodic = D.ns_periodic = fil ? 1 : 0;
  if (!D.ew_periodic) { D.west_exchng = D.inode > 0; D.east_exchng = D.inode < np_xi - 1; }
  if (!D.ns_periodic) { D.south_exchng = D.jnode > 0; D.north_exchng = D.jnode < np_eta - 1; }
  roms_cfg C{};
  C.nonlin_eos = c->nonlin_eos; C.salinity = c->salinity; C.lmd_mixing = c->lmd_mixing;
  C.uv_vis2 = 1; C.ts_dif2 = 1;
  C.dt = c->dt; C.ndtfast = c->ndtfast;
  C.nfast = set_weights(c->ndtfast, C.weight);
  C.g = 9.81; C.rho0 = fil ? 1000.0 : 1027.5; C.gamma2 = 1.0;
  C.rdrg = 0.0; C.rdrg2 = 1.0e-3; C.Zob = 1.0e-2;
  C.Tcoef = 0.20; C.T0 = 1.0; C.Scoef = 0.822; C.S0 = 1.0;
  C.theta_s = 6.0; C.theta_b = pipes ? 6.0 : 2.0; C.hc = (fil || pipes) ? 25.0 : 250.0;
  // tests/Pipes_ana/benchmark.in has no vertical_mixing line: Akv_bak = Akt_bak = 0
  C.obc = c->case_id == ROMS_CASE_BASIN ? c->obc : 0;
  C.ubind = 0.1;  // Examples/Iceland/Iceland_parent/roms.in: ubind
  C.curvgrid = c->case_id == ROMS_CASE_BASIN ? c->curvgrid : 0;
  C.uv_adv = c->uv_adv; C.uv_cor = c->uv_cor;
  C.bulk_frc = c->case_id == ROMS_CASE_BASIN ? c->bulk_frc : 0;
  C.adv_isoneutral = c->adv_isoneutral;
  C.Akv_bak = (fil || pipes) ? 0.0 : 1.0e-4; C.Akt_bak[0] = (fil || pipes) ? 0.0 : 1.0e-5; C.Akt_bak[1] = C.Akt_bak[0];
  int r = roms_gpu_init(&D, &C, device, comm);
  if (r) return r;
  CaseSpec cs{};
  cs.case_id = c->case_id; cs.LLm = c->LLm; cs.MMm = c->MMm;
  cs.iSW_corn = D.iSW_corn; cs.jSW_corn = D.jSW_corn;
  cs.ew_periodic = D.ew_periodic; cs.ns_periodic = D.ns_periodic;
  cs.west_exchng = D.west_exchng; cs.east_exchng = D.east_exchng;
  cs.south_exchng = D.south_exchng; cs.north_exchng = D.north_exchng;
  cs.host_wrap = comm == nullptr;   // with a communicator the device exchange fills halos
  cs.salinity = c->salinity; cs.lmd = c->lmd_mixing != 0; cs.surf_flux = c->case_id == ROMS_CASE_BASIN ? c->surf_flux : 0; cs.theta_s = C.theta_s; cs.theta_b = C.theta_b; cs.hc = C.hc; cs.rho0 = C.rho0;
  cs.Tcoef = C.Tcoef; cs.visc2 = 0.0; cs.tnu2 = 0.0; cs.Akv_bak = C.Akv_bak;
  cs.Akt_bak[0] = C.Akt_bak[0]; cs.Akt_bak[1] = C.Akt_bak[1];
  cs.sizex = c->sizex; cs.sizey = c->sizey;
  cs.obc = C.obc; cs.island = c->case_id == ROMS_CASE_BASIN ? c->island : 0;
  cs.v_sponge = C.obc ? c->v_sponge : 0.0;
  cs.curvgrid = C.curvgrid;
  cs.bulk_frc = C.bulk_frc;
  HostState H(D.Lm, D.Mm, D.N, D.NT, C.salinity ? 2 : 1);
  double area = 0.0, volume = 0.0;
  build_case(cs, H, area, volume);
  // setup_grid2.F: per-rank pairwise sums, then the tree over ranks
  {
    const double loc[2] = {area, volume};
    std::vector<double> all(2 * (size_t)(np_xi * np_eta));
    if (halo_allgather(g.halo, g.s, loc, 2, all.data())) { g.err = "init_case: area/volume gather failed"; return -2; }
    std::vector<double> va, vv;
    for (int q = 0; q < np_xi * np_eta; q++) { va.push_back(all[2 * q]); vv.push_back(all[2 * q + 1]); }
    g.area = tree_sum(va);
    g.volume = tree_sum(vv);
    g.have_volume = true;
  }
  for (int id = 0; id < ROMS_NFIELDS; id++) {
    if (H.arr[id].empty()) continue;
    r = roms_gpu_copy_in(id, H.arr[id].data(), (long)H.arr[id].size());
    if (r) return r;
  }
  if (H.npip > 0) {
    r = roms_gpu_set_pipe_frc(H.npip, H.pipe_idx.data(), H.pipe_flx.data(), H.pipe_prf.data(), H.pipe_trc.data());
    if (r) return r;
  }
  if (H.nriv > 0) {
    r = roms_gpu_set_river_frc(H.nriv, H.riv_uflx.data(), H.riv_vflx.data(), H.riv_vol.data(), H.riv_trc.data());
    if (r) return r;
  }
  if (comm != nullptr) {
    // the exchanges of setup_grid1.F and ana_init (host wrap in the single-rank build)
    const Fields& F = g.d.f;
    const ExchList grid1{{F.dm_r, F.dn_r, F.dm_p, F.dn_p, F.dm_u, F.dn_u, F.dm_v, F.dn_v}, {1, 1, 1, 1, 1, 1, 1, 1}, 8};
    const ExchList grid2{{F.pmon_u, F.pnom_v, F.rmask, F.umask, F.vmask, F.pmask, F.dndx, F.dmde},
                         {1, 1, 1, 1, 1, 1, 1, 1}, 8};
    const ExchList st{{F.zeta, F.ubar, F.vbar, F.u, F.v}, {1, 1, 1, D.N, D.N}, 5};
    launch_exchange_list(g.d, g.s, grid1);
    launch_exchange_list(g.d, g.s, grid2);
    launch_exchange_list(g.d, g.s, st);
    launch_exchange_tracers(g.d, g.s, 1);
    CHECK_HIP(hipStreamSynchronize(g.s));
  }
  *t = roms_tlev{};
  t->iic = 0; t->ntstart = 1; t->forw_start = 1; t->iif = 1; t->nfast = C.nfast;
  t->kstp = 1; t->knew = 1; t->nstp = 1; t->nrhs = 1; t->nnew = 1;
  if (C.bulk_frc) launch_bulk_flux(g.d, g.s, 1);   // set_forces after ana_init (main.F:266)
  return roms_gpu_init_sequence(t);
}

int roms_gpu_init_case(const roms_case* c, int device, roms_tlev* t) { return init_case_impl(c, 1, 1, nullptr, device, t); }
int roms_gpu_init_case_comm(const roms_case* c, int np_xi, int np_eta, void* comm, int device, roms_tlev* t) {
  if (np_xi * np_eta > 1 && !comm) { g.err = "roms_gpu_init_case_comm: communicator required"; return -1; }
  return init_case_impl(c, np_xi, np_eta, comm, device, t);
}

// ---- communicators ----
int roms_gpu_comm_unique_id(void* id128) {
  if (!id128) return -1;
  if (comm_unique_id(id128)) { g.err = "ncclGetUniqueId failed"; return -5; }
  return 0;
}
int roms_gpu_comm_create(const void* id128, int nranks, int rank, int device, void** comm) {
  if (!id128 || !comm || nranks < 1 || rank < 0 || rank >= nranks) { g.err = "roms_gpu_comm_create: bad argument"; return -1; }
  CHECK_HIP(hipSetDevice(device));
  RomsComm* c = comm_create_rccl(id128, nranks, rank, g.err);
  if (!c) return -5;
  *comm = c;
  return 0;
}
int roms_gpu_comm_create_host(int nranks, int rank, int device, roms_host_allgather_fn allgather, void* ctx,
                              void** comm) {
  if (!allgather || !comm || nranks < 1 || rank < 0 || rank >= nranks) {
    g.err = "roms_gpu_comm_create_host: bad argument";
    return -1;
  }
  CHECK_HIP(hipSetDevice(device));
  *comm = comm_create_host(nranks, rank, allgather, ctx);
  return 0;
}
int roms_gpu_comm_create_local(int group, int nranks, int rank, void** comm) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) { g.err = "roms_gpu_comm_create_local: bad argument"; return -1; }
  *comm = comm_create_local(group, nranks, rank);
  return 0;
}
int roms_gpu_comm_destroy(void* comm) {
  comm_destroy((RomsComm*)comm);
  return 0;
}
long roms_gpu_halo_map(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic, int ns_periodic,
                       int dir, int unpack, int* iv, int* jv, long cap) {
  if (Lm < 2 || Mm < 2 || np_xi < 1 || np_eta < 1 || inode < 0 || inode >= np_xi || jnode < 0 || jnode >= np_eta ||
      dir < 0 || dir > 7)
    return -1;
  const HaloPlan P = halo_plan(Lm, Mm, np_xi, np_eta, inode, jnode, ew_periodic, ns_periodic);
  if (P.g.cnt[dir] > cap) return -1;
  return halo_map(P, dir, unpack, iv, jv);
}
long roms_gpu_halo_map_wide(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic,
                            int ns_periodic, int width, int dir, int unpack, int* iv, int* jv, long cap) {
  if (Lm < 2 || Mm < 2 || np_xi < 1 || np_eta < 1 || inode < 0 || inode >= np_xi || jnode < 0 || jnode >= np_eta ||
      dir < 0 || dir > 7 || width < 1 || width > Lm || width > Mm)
    return -1;
  const HaloPlan P = halo_plan(Lm, Mm, np_xi, np_eta, inode, jnode, ew_periodic, ns_periodic, width);
  if (P.g.cnt[dir] > cap) return -1;
  return halo_map(P, dir, unpack, iv, jv);
}
int roms_gpu_halo_plan(int Lm, int Mm, int np_xi, int np_eta, int inode, int jnode, int ew_periodic, int ns_periodic,
                       int peer[8], long count[8], int strip[4]) {
  if (Lm < 2 || Mm < 2 || np_xi < 1 || np_eta < 1 || inode < 0 || inode >= np_xi || jnode < 0 || jnode >= np_eta) return -1;
  const HaloPlan P = halo_plan(Lm, Mm, np_xi, np_eta, inode, jnode, ew_periodic, ns_periodic);
  for (int d = 0; d < 8; d++) { peer[d] = P.peer[d]; count[d] = P.g.cnt[d]; }
  strip[0] = P.g.i0; strip[1] = P.g.i1; strip[2] = P.g.j0; strip[3] = P.g.j1;
  return 0;
}

int roms_gpu_time_routine(int routine, int nsteps, roms_tlev* t, double* avg_ms, long* launches) {
  REQUIRE_INIT_RO();   // runs whole steps, as roms_gpu_step
  if (routine < 0 || routine >= ROMS_R_COUNT || nsteps < 1 || !avg_ms || !launches) {
    g.err = "roms_gpu_time_routine: bad argument";
    return -1;
  }
  const size_t need = (size_t)2 * (size_t)nsteps * (size_t)(g.cfg.nfast + 4);
  while (g.ev.size() < need) {
    hipEvent_t e;
    CHECK_HIP(hipEventCreate(&e));
    g.ev.push_back(e);
  }
  g.timed = routine;
  g.nev = 0;
  g.kcount = 0;
  // eager steps (no graph), same launches and stream as the graph replays
  for (int q = 0; q < nsteps; q++) {
    t->iic = t->iic + 1;
    t->nstp = 1 + (t->iic - t->ntstart) % 2;
    t->nrhs = t->nstp;
    t->nnew = 3;
    t->nfast = g.cfg.nfast;
    const int r = frc_step_prepare(g.s, g.d, g.cfg.dt, *t, g.err);   // in-step forcing, as roms_gpu_step
    if (r) { g.timed = -1; return r; }
    const bool store_huv = g.hzuv_env || g.f[ROMS_Hz_u].host != nullptr || g.f[ROMS_Hz_v].host != nullptr;
    g.hzuv_valid = store_huv;
    enqueue_step(t, g.rho_reuse && g.rho_slot == t->nrhs, store_huv);
  }
  g.timed = -1;
  CHECK_HIP(hipStreamSynchronize(g.s));
  double tot = 0.0;
  for (size_t q = 0; q + 1 < g.nev; q += 2) {
    float f = 0.f;
    CHECK_HIP(hipEventElapsedTime(&f, g.ev[q], g.ev[q + 1]));
    tot += (double)f;
  }
  *launches = (long)(g.nev / 2);
  *avg_ms = g.nev ? tot / (double)(g.nev / 2) : 0.0;
  if (g.kcount > 0) {   // kernel level: intervals span several launches
    *launches = g.kcount;
    *avg_ms = tot / (double)g.kcount;
  }
  return post_launch();
}

int roms_gpu_time_steps(roms_tlev* t, int n, double* ms) {
  REQUIRE_INIT_RO();
  hipEvent_t a, b;
  CHECK_HIP(hipEventCreate(&a));
  CHECK_HIP(hipEventCreate(&b));
  CHECK_HIP(hipEventRecord(a, g.s));
  for (int q = 0; q < n; q++) {
    const int r = roms_gpu_step(t);
    if (r) return r;
  }
  CHECK_HIP(hipEventRecord(b, g.s));
  CHECK_HIP(hipEventSynchronize(b));
  float f = 0.f;
  CHECK_HIP(hipEventElapsedTime(&f, a, b));
  *ms = (double)f;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 0;
}

// setup_grid2.F area/volume from the device grid (a host that registered its
// own arrays): per-rank pairwise sums, then the tree over ranks
static int grid_integrals() {
  const Bounds& b = g.d.b;
  HostState H(b.Lm, b.Mm, b.N, b.NT, b.nTS);
  std::vector<double> h(b.n2), pm(b.n2), pn(b.n2), rm(b.n2);
  CHECK_HIP(copy_on(h.data(), g.d.f.h, b.n2 * sizeof(double), hipMemcpyDeviceToHost, g.s));
  CHECK_HIP(copy_on(pm.data(), g.d.f.pm, b.n2 * sizeof(double), hipMemcpyDeviceToHost, g.s));
  CHECK_HIP(copy_on(pn.data(), g.d.f.pn, b.n2 * sizeof(double), hipMemcpyDeviceToHost, g.s));
  CHECK_HIP(copy_on(rm.data(), g.d.f.rmask, b.n2 * sizeof(double), hipMemcpyDeviceToHost, g.s));
  std::vector<double> dA(g.hb.n2, 0.0), dV(g.hb.n2, 0.0);   // the host layout pair_sum walks
  for (int j = 1; j <= b.Mm; j++)
    for (int i = 1; i <= b.Lm; i++) {
      const long o = IJ(b, i, j), q = IJ(g.hb, i, j);
      dA[q] = rm[o] / (pm[o] * pn[o]);
      dV[q] = dA[q] * h[o];
    }
  const double loc[2] = {pair_sum(H, dA), pair_sum(H, dV)};
  const int nr = g.halo.comm ? comm_size(g.halo.comm) : 1;
  std::vector<double> all(2 * (size_t)nr);
  if (halo_allgather(g.halo, g.s, loc, 2, all.data())) { g.err = "roms_gpu_diag: area/volume gather failed"; return -2; }
  std::vector<double> va, vv;
  for (int q = 0; q < nr; q++) { va.push_back(all[2 * q]); vv.push_back(all[2 * q + 1]); }
  g.area = tree_sum(va);
  g.volume = tree_sum(vv);
  g.have_volume = true;
  return 0;
}

int roms_gpu_set_weights(int ndtfast, double weight[2][ROMS_MAX_FAST]) {
  if (ndtfast < 1 || !weight) return -1;
  return set_weights(ndtfast, weight);
}

// diag.F code_check norms, all on the device (k_diag.hip: per-column terms,
// reduction by pairs, first-maximum Courant scan, blow-up flag); six numbers
// come back, ranks combine in the reference's tree order (diag.F:488-535).
int roms_gpu_diag(const roms_tlev* t, double norms[4]) {
  REQUIRE_INIT_RO();
  if (!g.have_volume) {
    CHECK_HIP(hipStreamSynchronize(g.s));
    const int r = grid_integrals();
    if (r) return r;
  }
  launch_diag(g.d, g.s, to_tlev(t), g.d_diag);
  CHECK_HIP(hipMemcpyAsync(g.h_diag, g.d_diag, 6 * sizeof(double), hipMemcpyDeviceToHost, g.s));
  CHECK_HIP(hipStreamSynchronize(g.s));
  const double avzeta = g.h_diag[0], kes = g.h_diag[1], ke2 = g.h_diag[2], Cu = g.h_diag[3], Cw = g.h_diag[4];
  const bool blowup = g.h_diag[5] != 0.0;
  if (g.halo.comm) {
    // per-rank partial sums / maxima combined in the reference's tree order (diag.F:488-535)
    const double loc[6] = {avzeta, kes, ke2, Cu, Cw, blowup ? 1.0 : 0.0};
    const int nr = comm_size(g.halo.comm);
    std::vector<double> all(6 * (size_t)nr);
    if (halo_allgather(g.halo, g.s, loc, 6, all.data())) { g.err = "roms_gpu_diag: gather failed"; return -2; }
    std::vector<double> a(nr), k1(nr), k2(nr), cu(nr), cw(nr);
    bool any = false;
    for (int q = 0; q < nr; q++) {
      a[q] = all[6 * q]; k1[q] = all[6 * q + 1]; k2[q] = all[6 * q + 2]; cu[q] = all[6 * q + 3]; cw[q] = all[6 * q + 4];
      any = any || all[6 * q + 5] != 0.0;
    }
    int size = nr;
    while (size > 1) {
      const int step = (size + 1) / 2;
      for (int r = 0; r < size - step; r++)
        if (cu[r + step] > cu[r]) { cu[r] = cu[r + step]; cw[r] = cw[r + step]; }
      size = step;
    }
    norms[0] = tree_sum(k1) / (g.volume + tree_sum(a));
    norms[1] = tree_sum(k2) / (g.volume + tree_sum(a));
    norms[2] = cu[0];
    norms[3] = cw[0];
    if (any) { g.err = "roms_gpu_diag: Abnormal termination: BLOWUP (non-finite norms, diag.F:621-633)"; return -7; }
    return post_launch();
  }
  norms[0] = kes / (g.volume + avzeta);
  norms[1] = ke2 / (g.volume + avzeta);
  norms[2] = Cu;
  norms[3] = Cw;
  if (blowup) { g.err = "roms_gpu_diag: Abnormal termination: BLOWUP (non-finite norms, diag.F:621-633)"; return -7; }
  return post_launch();
}

}  // extern "C"
