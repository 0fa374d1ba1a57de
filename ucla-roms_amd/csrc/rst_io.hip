// rst_io.hip -- partitioned netCDF restart and history files (SURVEY.md
// section 8(f)3): wrt_restart_file / wrt_his_ocean_vars (basic_output.F:
// 273-419, 568-682, def_vars_*: 736-1034), put_global_atts
// (roms_read_write.F:1544-1660) and get_init (get_init.F:28-620), one file
// per rank as the reference's PARALLEL_FILES build writes them.
//
// MI355X design: a write enqueues, on the library stream, one gather kernel
// per variable that packs the record's slabs (zeta(i0:i1,j0:j1,knew),
// u(1:i1,j0:j1,:,nnew), ...) into a device staging buffer -- a device-to-
// device snapshot at HBM speed, ordered before the next step's kernels -- and
// then returns.  A second stream drains the snapshot to pinned host memory
// over PCIe while the model keeps stepping, and a host writer thread waits for
// that copy and writes the big-endian netCDF record.  roms_gpu_io_wait()
// joins the writer; a new write joins the previous one first (one staging
// buffer).  Reads (get_init) are synchronous: host read, masking as the
// reference does it, upload of packed slabs, one scatter kernel per variable,
// and the reference's exchange_xxx after every field.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/roms_gpu.h"
#include "ncio.h"
#include "roms_dev.h"
#include "shim_state.h"

namespace roms {
namespace {

// one (i0:i1, j0:j1, 1:nk) block of a device field, packed i fastest
struct Slab {
  const double* src;   // element (i0, j0, level 1)
  int ni, nj, nk;
  long sj, sk;         // row and level strides
  int as_mask;         // riv_umask/riv_vmask: 1 where the river face array is non-zero
  // history omega (basic_output.F:374-384): pm*pn*(We+Wi) in m/s when src2
  // (Wi) is set; pm/pn are 2-D, element (i0, j0)
  const double* src2;
  const double *pm, *pn;
};

__global__ void __launch_bounds__(256) k_io_pack(Slab s, double* __restrict__ dst) {
  const long n = (long)s.ni * s.nj * s.nk;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) {
    const int i = (int)(q % s.ni);
    const long r = q / s.ni;
    const int j = (int)(r % s.nj), k = (int)(r / s.nj);
    const long o = i + j * s.sj;
    double v = s.src ? s.src[o + k * s.sk] : 0.0;
    if (s.src2) v = s.pm[o] * s.pn[o] * (v + s.src2[o + k * s.sk]);
    dst[q] = s.as_mask ? (v != 0.0 ? 1.0 : 0.0) : v;
  }
}
__global__ void __launch_bounds__(256) k_io_unpack(Slab s, double* __restrict__ dstf, const double* __restrict__ src) {
  const long n = (long)s.ni * s.nj * s.nk;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) {
    const int i = (int)(q % s.ni);
    const long r = q / s.ni;
    const int j = (int)(r % s.nj), k = (int)(r / s.nj);
    dstf[i + j * s.sj + k * s.sk] = src[q];
  }
}
unsigned blocks_for(long n) {
  const long b = (n + 255) / 256;
  return (unsigned)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

// the partition's write ranges (dimensions.F:40-45): rho points i0:i1, u points 1:i1
struct Part {
  int i0, i1, j0, j1;
  int xi_rho, xi_u, eta_rho, eta_v;
};
Part part_of(const roms_dims& D) {
  Part p;
  p.i0 = D.inode == 0 ? 0 : 1;
  p.i1 = D.inode == D.np_xi - 1 ? D.Lm + 1 : D.Lm;
  p.j0 = D.jnode == 0 ? 0 : 1;
  p.j1 = D.jnode == D.np_eta - 1 ? D.Mm + 1 : D.Mm;
  p.xi_rho = p.i1 - p.i0 + 1; p.xi_u = p.i1;
  p.eta_rho = p.j1 - p.j0 + 1; p.eta_v = p.j1;
  return p;
}

// grid type of a variable: 'r' rho, 'u', 'v'
Slab slab_of(const Bounds& b, const Part& p, const double* base, char g, int nk, long sk) {
  Slab s{};
  const int i0 = g == 'u' ? 1 : p.i0, j0 = g == 'v' ? 1 : p.j0;
  s.src = base ? base + IJ(b, i0, j0) : nullptr;
  s.ni = p.i1 - i0 + 1;
  s.nj = p.j1 - j0 + 1;
  s.nk = nk;
  s.sj = b.nx2;
  s.sk = sk;
  return s;
}

struct OutVar {
  std::string name, lname, units;
  char grid;      // 'r', 'u', 'v'
  int levels;     // 0: 2-D; N or N+1
  Slab slab;
  long off = 0;   // offset in the staging buffer (elements)
};

struct IoJob {
  std::thread th;
  bool running = false;
  int status = 0;
  std::string err;
};

struct IoCtx {
  double* stage = nullptr;      // device staging (snapshot)
  size_t stage_n = 0;
  double* pinned = nullptr;     // host staging
  size_t pinned_n = 0;
  hipStream_t drain = nullptr;  // D2H stream
  hipEvent_t packed = nullptr, landed = nullptr;
  IoJob job;
  std::vector<std::string> tname, tunits, tlname;
};
thread_local IoCtx io;

int io_join(std::string& err) {
  if (!io.job.running) return 0;
  io.job.th.join();
  io.job.running = false;
  if (io.job.status) { err = io.job.err; return io.job.status; }
  return 0;
}

// tracer names (tracers.F:296-301: temp, salt with SALINITY; passive tracers
// get trcNN unless the host named them with roms_gpu_io_tracer_name)
void tracer_meta(int NT, bool salinity, std::vector<std::string>& nm, std::vector<std::string>& un,
                 std::vector<std::string>& ln) {
  nm.assign(NT, ""); un.assign(NT, ""); ln.assign(NT, "");
  for (int q = 0; q < NT; q++) {
    if ((size_t)q < io.tname.size() && !io.tname[q].empty()) {
      nm[q] = io.tname[q]; un[q] = io.tunits[q]; ln[q] = io.tlname[q];
    } else if (q == 0) {
      nm[q] = "temp"; un[q] = "Celsius"; ln[q] = "potential temperature";
    } else if (q == 1 && salinity) {
      nm[q] = "salt"; un[q] = "PSU"; ln[q] = "salinity";
    } else {
      char b[32];
      snprintf(b, sizeof b, "trc%02d", q + 1);
      nm[q] = b; un[q] = "nondim"; ln[q] = std::string("passive tracer ") + b;
    }
  }
}

// put_global_atts (roms_read_write.F:1544-1660) + the 'type' attribute of the creator
void global_atts(nc::File& f, const ShimState& S, const char* type) {
  const roms_dims& D = *S.dims;
  const roms_cfg& C = *S.cfg;
  const Part p = part_of(D);
  const int mynode = D.inode + D.jnode * D.np_xi, nnodes = D.np_xi * D.np_eta;
  if (nnodes > 1) {   // PARALLEL_FILES: partition + the 4 main horizontal dimensions (for ncjoin)
    f.add_dim("xi_rho", p.xi_rho); f.add_dim("xi_u", p.xi_u);
    f.add_dim("eta_rho", p.eta_rho); f.add_dim("eta_v", p.eta_v);
    const int is = D.inode == 0 ? D.iSW_corn + 1 : D.iSW_corn + 2;
    const int js = D.jnode == 0 ? D.jSW_corn + 1 : D.jSW_corn + 2;
    f.gatts.push_back(nc::Att::i("partition", {mynode, nnodes, is, js}));
  }
  f.gatts.push_back(nc::Att::i("global_x", {D.LLm}));
  f.gatts.push_back(nc::Att::i("global_y", {D.MMm}));
  f.gatts.push_back(nc::Att::str("title", "roms_gpu (MI355X) run"));
  f.gatts.push_back(nc::Att::i("ndtfast", {C.ndtfast}));
  f.gatts.push_back(nc::Att::d("dt", {C.dt}));
  f.gatts.push_back(nc::Att::d("dtfast", {C.dt / C.ndtfast}));
  f.gatts.push_back(nc::Att::d("theta_s", {C.theta_s}));
  f.gatts.push_back(nc::Att::d("theta_b", {C.theta_b}));
  f.gatts.push_back(nc::Att::d("hc", {C.hc}));
  f.gatts.push_back(nc::Att::d("rho0", {C.rho0}));
  f.gatts.push_back(nc::Att::str("rho0_units", "kg/m^3"));
  if (!C.nonlin_eos) {
    f.gatts.push_back(nc::Att::d("Tcoef", {C.Tcoef}));
    f.gatts.push_back(nc::Att::d("T0", {C.T0}));
    if (C.salinity) { f.gatts.push_back(nc::Att::d("Scoef", {C.Scoef})); f.gatts.push_back(nc::Att::d("S0", {C.S0})); }
  }
  f.gatts.push_back(nc::Att::d("gamma2", {C.gamma2}));
  f.gatts.push_back(nc::Att::d("Akv_bak", {C.Akv_bak}));
  f.gatts.push_back(nc::Att::d("Akt_bak", {C.Akt_bak[0], C.Akt_bak[1]}));
  f.gatts.push_back(nc::Att::d("rdrg", {C.rdrg}));
  f.gatts.push_back(nc::Att::d("rdrg2", {C.rdrg2}));
  f.gatts.push_back(nc::Att::d("Zob", {C.Zob}));
  f.gatts.push_back(nc::Att::str("type", type));
}

// the variable list of a restart (def_vars_rst_ocean_vars) or history record
std::vector<OutVar> record_vars(const ShimState& S, const roms_tlev& t, bool rst, int mask) {
  const Bounds& b = S.d->b;
  const Fields& F = S.d->f;
  const Part p = part_of(*S.dims);
  const int N = b.N;
  std::vector<OutVar> v;
  auto add = [&](const char* name, const char* ln, const char* un, char g, int lev, const double* base, long sk) {
    OutVar o;
    o.name = name; o.lname = ln; o.units = un; o.grid = g; o.levels = lev;
    o.slab = slab_of(b, p, base, g, lev ? lev : 1, sk);
    v.push_back(o);
  };
  const long n2 = b.n2;
  const int knew = t.knew, nnew = t.nnew;
  if (rst || (mask & ROMS_WRT_Z)) add("zeta", "free-surface elevation", "meter", 'r', 0, F.zeta + (knew - 1) * n2, 0);
  if (rst || (mask & ROMS_WRT_UB))
    add("ubar", "vertically averaged u-momentum component", "meter second-1", 'u', 0, F.ubar + (knew - 1) * n2, 0);
  if (rst || (mask & ROMS_WRT_VB))
    add("vbar", "vertically averaged v-momentum component", "meter second-1", 'v', 0, F.vbar + (knew - 1) * n2, 0);
  if (rst || (mask & ROMS_WRT_U)) add("u", "u-momentum component", "meter second-1", 'u', N, F.u + (nnew - 1) * b.n3, n2);
  if (rst || (mask & ROMS_WRT_V)) add("v", "v-momentum component", "meter second-1", 'v', N, F.v + (nnew - 1) * b.n3, n2);
  if (rst || (mask & ROMS_WRT_T)) {
    std::vector<std::string> nm, un, ln;
    tracer_meta(b.NT, S.cfg->salinity != 0, nm, un, ln);
    for (int q = 0; q < b.NT; q++) {
      OutVar o;
      o.name = nm[q]; o.lname = ln[q]; o.units = un[q]; o.grid = 'r'; o.levels = N;
      o.slab = slab_of(b, p, F.t + (long)(nnew - 1) * b.n3 + (long)q * 3 * b.n3, 'r', N, n2);
      v.push_back(o);
    }
  }
  if (rst) {   // EXACT_RESTART + EXTRAP_BAR_FLUXES (basic_output.F:634-642)
    add("DU_avg1", "<<fast-time averaged uflx>>", "", 'u', 0, F.DU_avg1, 0);
    add("DV_avg1", "<<fast-time-averaged vflx>>", "", 'v', 0, F.DV_avg1, 0);
    add("DU_avg2", "<<fast-time averaged ubar(:,:,n+1/2)>>", "", 'u', 0, F.DU_avg2, 0);
    add("DV_avg2", "<<fast-time-averaged vbar(:,:,n+1/2)>>", "", 'v', 0, F.DV_avg2, 0);
    add("DU_avg_bak", "<back-step mixed fast-time-averaged ubar(:,:,n-1)>", "", 'u', 0, F.DU_avg_bak, 0);
    add("DV_avg_bak", "<back-step mixed fast-time-averaged vbar(:,:,n-1)>", "", 'v', 0, F.DV_avg_bak, 0);
  }
  if (!rst && (mask & ROMS_WRT_R)) {   // rho1 (SPLIT_EOS) or rho
    add("rho", "density anomaly", "kilogram meter-3", 'r', N, S.cfg->nonlin_eos ? F.rho1 : F.rho, n2);
  }
  if (!rst && (mask & ROMS_WRT_O)) {   // pm*pn*(We+Wi), m/s (basic_output.F:374-384)
    add("omega", "S-coordinate vertical momentum component", "meter second-1", 'r', N + 1, F.We, n2);
    Slab& o = v.back().slab;
    const long off = o.src - F.We;   // element (i0, j0)
    o.src2 = F.Wi + off;
    o.pm = F.pm + off;
    o.pn = F.pn + off;
  }
  if (!rst && (mask & ROMS_WRT_AKV)) add("AKv", "vertical viscosity coefficient", "meter2 second-1", 'r', N + 1, F.Akv, n2);
  if (!rst && (mask & ROMS_WRT_AKT))
    add("AKt", "temperature vertical diffusion coefficient", "meter2 second-1", 'r', N + 1, F.Akt, n2);
  if (!rst && (mask & ROMS_WRT_AKS) && S.cfg->salinity)
    add("AKs", "salinity vertical diffusion coefficient", "meter2 second-1", 'r', N + 1, F.Akt + b.n3w, n2);
  const bool kpp = S.cfg->lmd_mixing != 0;
  if (kpp && (rst || (mask & ROMS_WRT_HBLS))) add("hbls", "Thickness of KPP surface boundary layer", "meter", 'r', 0, F.hbls, 0);
  if (kpp && (rst || (mask & ROMS_WRT_HBBL))) add("hbbl", "Thickness of KPP bottom boundary layer", "meter", 'r', 0, F.hbbl, 0);
  if (rst) {
    add("riv_umask", "river mask at u points", "nondim", 'u', 0, F.riv_uflx, 0);
    v.back().slab.as_mask = 1;
    add("riv_vmask", "river mask at v points", "nondim", 'v', 0, F.riv_vflx, 0);
    v.back().slab.as_mask = 1;
  }
  return v;
}

void define_file(nc::File& f, const ShimState& S, const std::vector<OutVar>& vars, bool rst) {
  const Part p = part_of(*S.dims);
  const int N = S.d->b.N;
  // create_file (roms_read_write.F:1161-1208): ocean_time first, then the global attributes
  const int dtm = f.add_dim("time", 0);
  f.add_var("ocean_time", nc::NC_DOUBLE, {dtm},
            {nc::Att::str("long_name", "Time since 2000/01/01"), nc::Att::str("units", "second")});
  global_atts(f, S, rst ? "ROMS restart file" : "ROMS history file");
  const int daux = f.add_dim("auxil", 6);   // iaux
  f.add_var("time_step", nc::NC_INT, {dtm, daux},
            {nc::Att::str("long_name", "time step and record numbers from initialization")});
  const int dxr = f.add_dim("xi_rho", p.xi_rho), dxu = f.add_dim("xi_u", p.xi_u);
  const int dyr = f.add_dim("eta_rho", p.eta_rho), dyv = f.add_dim("eta_v", p.eta_v);
  int dzr = -1, dzw = -1;
  for (const OutVar& o : vars) {
    const int dx = o.grid == 'u' ? dxu : dxr, dy = o.grid == 'v' ? dyv : dyr;
    std::vector<int> dims{dtm};
    if (o.levels == N) { if (dzr < 0) dzr = f.add_dim("s_rho", N); dims.push_back(dzr); }
    if (o.levels == N + 1) { if (dzw < 0) dzw = f.add_dim("s_w", N + 1); dims.push_back(dzw); }
    dims.push_back(dy);
    dims.push_back(dx);
    std::vector<nc::Att> at{nc::Att::str("long_name", o.lname)};
    if (!o.units.empty()) at.push_back(nc::Att::str("units", o.units));
    f.add_var(o.name, nc::NC_DOUBLE, dims, at);
  }
}

int write_record(const char* path, int rec, int total_rec, double time, const roms_tlev* t, bool rst, int mask) {
  ShimState S;
  int r = shim_enter(S, true);
  if (r) return r;
  if (!path || rec < 1 || !t) { *S.err = "roms_gpu_wrt: bad path/record/time levels"; return -1; }
  if ((r = io_join(*S.err))) return r;
  std::vector<OutVar> vars = record_vars(S, *t, rst, mask);
  size_t n = 0;
  for (OutVar& o : vars) { o.off = (long)n; n += (size_t)o.slab.ni * o.slab.nj * o.slab.nk; }
  if (!io.drain) {
    if (hipStreamCreateWithFlags(&io.drain, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&io.packed, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&io.landed, hipEventDisableTiming) != hipSuccess) {
      *S.err = "roms_gpu_wrt: stream/event creation failed";
      return -2;
    }
  }
  if (io.stage_n < n) {
    if (io.stage) (void)hipFree(io.stage);
    io.stage = nullptr;
    if (hipMalloc(&io.stage, n * sizeof(double)) != hipSuccess) { *S.err = "roms_gpu_wrt: staging allocation failed"; return -2; }
    io.stage_n = n;
  }
  if (io.pinned_n < n) {
    if (io.pinned) (void)hipHostFree(io.pinned);
    io.pinned = nullptr;
    if (hipHostMalloc(&io.pinned, n * sizeof(double), hipHostMallocDefault) != hipSuccess) {
      *S.err = "roms_gpu_wrt: pinned staging allocation failed";
      return -2;
    }
    io.pinned_n = n;
  }
  // device snapshot on the library stream (ordered before the next step) ...
  for (const OutVar& o : vars) {
    const long m = (long)o.slab.ni * o.slab.nj * o.slab.nk;
    hipLaunchKernelGGL(k_io_pack, dim3(blocks_for(m)), dim3(256), 0, S.s, o.slab, io.stage + o.off);
  }
  if (hipEventRecord(io.packed, S.s) != hipSuccess || hipStreamWaitEvent(io.drain, io.packed, 0) != hipSuccess ||
      hipMemcpyAsync(io.pinned, io.stage, n * sizeof(double), hipMemcpyDeviceToHost, io.drain) != hipSuccess ||
      hipEventRecord(io.landed, io.drain) != hipSuccess) {
    *S.err = "roms_gpu_wrt: snapshot enqueue failed";
    return -2;
  }
  if (hipGetLastError() != hipSuccess) { *S.err = "roms_gpu_wrt: pack launch failed"; return -3; }
  // ... drained and written by a host thread while the model steps on
  const std::string fpath(path);
  const roms_tlev tl = *t;
  const bool create = rec == 1;
  nc::File* proto = new nc::File();
  if (create) define_file(*proto, S, vars, rst);
  io.job.status = 0;
  io.job.err.clear();
  io.job.running = true;
  hipEvent_t landed = io.landed;
  const double* host = io.pinned;
  IoJob* job = &io.job;   // io is thread_local: the writer reports through this pointer
  io.job.th = std::thread([=]() {
    std::unique_ptr<nc::File> f(proto);
    try {
      if (hipEventSynchronize(landed) != hipSuccess) throw std::runtime_error("snapshot copy failed");
      if (create) f->create(fpath);
      else f->open(fpath, true);
      const int64_t r0 = rec - 1;
      const int vt = f->find_var("ocean_time"), vs = f->find_var("time_step");
      if (vt < 0 || vs < 0) throw std::runtime_error(fpath + ": not a file of this writer (no ocean_time/time_step)");
      f->put_double(vt, r0, &time);
      const int ts[6] = {tl.iic, rec, total_rec, 0, 0, 0};   // write_time_step (basic_output.F:1120-1150)
      f->put_int(vs, r0, ts);
      for (const OutVar& o : vars) {
        const int id = f->find_var(o.name);
        if (id < 0) throw std::runtime_error(fpath + ": variable " + o.name + " not defined");
        if (f->vars[id].count() != (int64_t)o.slab.ni * o.slab.nj * o.slab.nk)
          throw std::runtime_error(fpath + ": variable " + o.name + " has another shape");
        f->put_double(id, r0, host + o.off);
      }
      f->close();
    } catch (const std::exception& e) {
      job->status = -7;
      job->err = std::string("roms_gpu_wrt: ") + e.what();
    }
  });
  return 0;
}

}  // namespace
}  // namespace roms

using namespace roms;

extern "C" {

int roms_gpu_wrt_rst(const char* path, int rec, int total_rec, double time, const roms_tlev* t) {
  return write_record(path, rec, total_rec, time, t, true, 0);
}
int roms_gpu_wrt_his(const char* path, int rec, int total_rec, double time, const roms_tlev* t, int wrt_mask) {
  return write_record(path, rec, total_rec, time, t, false, wrt_mask);
}
int roms_gpu_io_wait(void) {
  std::string err;
  const int r = io_join(err);
  if (r) shim_set_error(err);
  return r;
}
int roms_gpu_io_tracer_name(int itrc, const char* name, const char* units, const char* long_name) {
  if (itrc < 1 || itrc > 1024 || !name) return -1;
  if (io.tname.size() < (size_t)itrc) { io.tname.resize(itrc); io.tunits.resize(itrc); io.tlname.resize(itrc); }
  io.tname[itrc - 1] = name;
  io.tunits[itrc - 1] = units ? units : "";
  io.tlname[itrc - 1] = long_name ? long_name : name;
  return 0;
}

// get_init (get_init.F:28-620): fields of record req_rec (1-based; 0 = the
// last) into time slot tindx (u, v, t; zeta/ubar/vbar always into slot 1),
// masked and exchanged as the reference does.  With tindx = 2 it performs the
// EXACT_RESTART checks on records req_rec, req_rec+1 (ocean_time one dt apart,
// consecutive time_step) and reads nothing when they fail; tindx = 1 sets
// t->ntstart, t->iic (= ntstart-1) and t->forw_start (1 after a successful
// tindx = 2 call: exact restart; ntstart otherwise) and leaves the fast-time
// indices at knew = kstp = 1.  Returns 0 (read), 1 (tindx = 2: exact restart
// not possible, nothing read) or a negative error.
int roms_gpu_get_init(const char* path, int req_rec, int tindx, roms_tlev* t, double* start_time) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  if (!path || !t || (tindx != 1 && tindx != 2)) { *S.err = "roms_gpu_get_init: bad arguments"; return -1; }
  if ((r = io_join(*S.err))) return r;
  const Bounds& b = S.d->b;
  const Fields& F = S.d->f;
  const Part p = part_of(*S.dims);
  try {
    nc::File f;
    f.open(path, false);
    const int64_t max_rec = f.numrecs;
    int64_t record = req_rec > 0 ? req_rec : (max_rec > 0 ? max_rec : 1);
    if (record > max_rec) throw std::runtime_error("requested record exceeds the records in the file");
    int vt = f.find_var("ocean_time");
    if (vt < 0) vt = f.find_var("roms_time");
    if (vt < 0) vt = f.find_var("scrum_time");
    if (vt < 0) throw std::runtime_error("time variable not found");
    double tm = 0.0;
    f.get_double(vt, record - 1, &tm);
    const int vs = f.find_var("time_step");
    int ts[6] = {0, 0, 0, 0, 0, 0};
    if (tindx == 2) {
      // EXACT_RESTART checks (get_init.F:241-290, 333-357)
      if (record >= max_rec) return 1;
      double tm2 = 0.0;
      f.get_double(vt, record, &tm2);
      if (!(std::abs(tm2 - tm - S.cfg->dt) < 0.01 * S.cfg->dt)) return 1;
      if (vs < 0) return 1;
      int ts2[6];
      f.get_int(vs, record - 1, ts);
      f.get_int(vs, record, ts2);
      if (ts2[0] != ts[0] + 1) return 1;
      t->forw_start = 1;
    } else {
      if (vs >= 0) {
        f.get_int(vs, record - 1, ts);
        t->ntstart = ts[0] + 1;
        if (t->forw_start != 1) t->forw_start = t->ntstart;   // approximate restart: forward first step
      } else {
        t->ntstart = 1;
        t->forw_start = 1;
      }
      t->iic = t->ntstart - 1;
      t->kstp = t->knew = 1;
      t->nstp = t->nrhs = 1;
      t->nnew = 1;
      if (start_time) *start_time = tm;
    }
    // host copies of the masks for the partition's slabs
    const long n2 = b.n2;
    std::vector<double> rmask(n2), umask(n2), vmask(n2);
    if (copy_on(rmask.data(), F.rmask, n2 * 8, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
        copy_on(umask.data(), F.umask, n2 * 8, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
        copy_on(vmask.data(), F.vmask, n2 * 8, hipMemcpyDeviceToHost, S.s) != hipSuccess)
      throw std::runtime_error("mask download failed");
    auto read_slab = [&](const std::string& name, char g, int nk, std::vector<double>& buf) -> bool {
      const int id = f.find_var(name);
      if (id < 0) return false;
      const Slab s = slab_of(b, p, nullptr, g, nk, 0);
      const int64_t cnt = (int64_t)s.ni * s.nj * s.nk;
      if (f.vars[id].count() != cnt) throw std::runtime_error("variable " + name + " has another shape than this rank's partition");
      buf.resize((size_t)cnt);
      f.get_double(id, record - 1, buf.data());
      return true;
    };
    // mask(i,j) (+ river mask) on every level of a packed slab
    auto apply_mask = [&](std::vector<double>& buf, char g, int nk, const std::vector<double>& m,
                          const std::vector<double>* riv) {
      const Slab s = slab_of(b, p, nullptr, g, nk, 0);
      const int i0 = g == 'u' ? 1 : p.i0, j0 = g == 'v' ? 1 : p.j0;
      for (int k = 0; k < s.nk; k++)
        for (int j = 0; j < s.nj; j++)
          for (int i = 0; i < s.ni; i++) {
            const long q = i + (long)s.ni * (j + (long)s.nj * k), ij = IJ(b, i0 + i, j0 + j);
            const double rm = riv ? (*riv)[i + (size_t)s.ni * j] : 0.0;
            buf[q] = buf[q] * (m[ij] + rm);
          }
    };
    // upload staging, released on every exit (an error return included)
    struct DevBuf {
      double* p = nullptr;
      ~DevBuf() { if (p) (void)hipFree(p); }
    } stage;
    double*& dbuf = stage.p;
    auto upload = [&](const std::vector<double>& buf, double* base, char g, int nk, long sk) {
      Slab s = slab_of(b, p, base, g, nk, sk);
      if (dbuf) { (void)hipFree(dbuf); dbuf = nullptr; }
      if (hipMalloc(&dbuf, buf.size() * 8) != hipSuccess ||
          copy_on(dbuf, buf.data(), buf.size() * 8, hipMemcpyHostToDevice, S.s) != hipSuccess)
        throw std::runtime_error("upload failed");
      hipLaunchKernelGGL(k_io_unpack, dim3(blocks_for((long)buf.size())), dim3(256), 0, S.s, s, (double*)s.src, dbuf);
      if (hipStreamSynchronize(S.s) != hipSuccess) throw std::runtime_error("unpack failed");
    };
    auto exch = [&](double* a, int nlev) {
      ExchList L{};
      L.p[0] = a; L.nlev[0] = nlev; L.n = 1;
      launch_exchange_list(*S.d, S.s, L);
      if (hipStreamSynchronize(S.s) != hipSuccess) throw std::runtime_error("exchange failed");
    };
    std::vector<double> buf, rivu, rivv;
    const int N = b.N;
    const bool has_rivu = read_slab("riv_umask", 'u', 1, rivu), has_rivv = read_slab("riv_vmask", 'v', 1, rivv);
    if (!read_slab("zeta", 'r', 1, buf)) throw std::runtime_error("zeta not found");
    apply_mask(buf, 'r', 1, rmask, nullptr);
    upload(buf, F.zeta, 'r', 1, 0);
    exch(F.zeta, 1);
    if (!read_slab("ubar", 'u', 1, buf)) throw std::runtime_error("ubar not found");
    apply_mask(buf, 'u', 1, umask, has_rivu ? &rivu : nullptr);
    upload(buf, F.ubar, 'u', 1, 0);
    exch(F.ubar, 1);
    if (!read_slab("vbar", 'v', 1, buf)) throw std::runtime_error("vbar not found");
    apply_mask(buf, 'v', 1, vmask, has_rivv ? &rivv : nullptr);
    upload(buf, F.vbar, 'v', 1, 0);
    exch(F.vbar, 1);
    // EXACT_RESTART + EXTRAP_BAR_FLUXES barotropic flux averages (get_init.F:439-467)
    const char* bar[6] = {"DU_avg1", "DV_avg1", "DU_avg2", "DV_avg2", "DU_avg_bak", "DV_avg_bak"};
    double* bard[6] = {F.DU_avg1, F.DV_avg1, F.DU_avg2, F.DV_avg2, F.DU_avg_bak, F.DV_avg_bak};
    bool exact = true;
    for (int q = 0; q < 6; q++) exact = exact && f.find_var(bar[q]) >= 0;
    if (exact) {
      for (int q = 0; q < 6; q++) {
        const char g = (q % 2) ? 'v' : 'u';
        read_slab(bar[q], g, 1, buf);
        upload(buf, bard[q], g, 1, 0);
      }
    } else if (tindx == 1) {
      t->forw_start = t->ntstart;   // cancel exact restart
    }
    const long sk = n2;
    if (!read_slab("u", 'u', N, buf)) throw std::runtime_error("u not found");
    apply_mask(buf, 'u', N, umask, has_rivu ? &rivu : nullptr);
    upload(buf, F.u + (long)(tindx - 1) * b.n3, 'u', N, sk);
    exch(F.u + (long)(tindx - 1) * b.n3, N);
    if (!read_slab("v", 'v', N, buf)) throw std::runtime_error("v not found");
    apply_mask(buf, 'v', N, vmask, has_rivv ? &rivv : nullptr);
    upload(buf, F.v + (long)(tindx - 1) * b.n3, 'v', N, sk);
    exch(F.v + (long)(tindx - 1) * b.n3, N);
    std::vector<std::string> nm, un, ln;
    tracer_meta(b.NT, S.cfg->salinity != 0, nm, un, ln);
    const int nts = S.cfg->salinity ? 2 : 1;
    for (int q = 0; q < b.NT; q++) {
      double* base = F.t + (long)(tindx - 1) * b.n3 + (long)q * 3 * b.n3;
      if (read_slab(nm[q], 'r', N, buf)) {
        apply_mask(buf, 'r', N, rmask, nullptr);
        upload(buf, base, 'r', N, sk);
      } else if (q < nts) {
        throw std::runtime_error("tracer " + nm[q] + " not found");
      } else {
        buf.assign((size_t)(p.xi_rho) * p.eta_rho * N, 0.0);   // passive tracer absent: 0
        upload(buf, base, 'r', N, sk);
      }
      exch(base, N);
    }
    if (S.cfg->lmd_mixing) {
      const char* hb[2] = {"hbls", "hbbl"};
      double* hd[2] = {F.hbls, F.hbbl};
      for (int q = 0; q < 2; q++)
        if (read_slab(hb[q], 'r', 1, buf)) {
          apply_mask(buf, 'r', 1, rmask, nullptr);
          upload(buf, hd[q], 'r', 1, 0);
          exch(hd[q], 1);
        }
    }
  } catch (const std::exception& e) {
    *S.err = std::string("roms_gpu_get_init: ") + path + ": " + e.what();
    return -7;
  }
  return 0;
}

}  // extern "C"

namespace roms {
void io_free() {
  std::string err;
  (void)io_join(err);
  if (io.stage) (void)hipFree(io.stage);
  if (io.pinned) (void)hipHostFree(io.pinned);
  if (io.drain) (void)hipStreamDestroy(io.drain);
  if (io.packed) (void)hipEventDestroy(io.packed);
  if (io.landed) (void)hipEventDestroy(io.landed);
  std::vector<std::string> tn = io.tname, tu = io.tunits, tl = io.tlname;
  io = IoCtx{};
  io.tname = tn; io.tunits = tu; io.tlname = tl;
}
}  // namespace roms
