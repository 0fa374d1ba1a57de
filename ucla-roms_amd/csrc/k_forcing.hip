// k_forcing.hip -- forcing and boundary producers on the device (SURVEY.md
// section 8(f)1): the time interpolation of set_frc_data
// (roms_read_write.F:303-392, 394-...; set_forces.F, set_bry_all in
// boundary.F:227) and the tidal synthesis of set_tides (tides.F:86-254).
//
// The reference re-reads nothing per step: each forcing variable keeps two
// records (vdata(:,:,it1/it2)) and every step interpolates them linearly to
// the model time.  Here the two records of every registered field live in
// HBM; the host uploads a record only when the time window advances
// (roms_gpu_frc_record), and roms_gpu_frc_interp forms all interpolated
// fields with one streaming kernel per field -- no per-step host->device
// traffic.  set_tides sums the tidal constituents into the potential ptide and
// onto the open-boundary zeta/ubar/vbar data on the device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/roms_gpu.h"
#include "roms_dev.h"
#include "shim_state.h"

namespace roms {
namespace {

// up to three records of one field: the reference's pair (it1, it2) plus the
// next record, so that a refresh falling inside a step (set_frc_data moves
// to (it2, next) once times(it2) < modtime, roms_read_write.F:341-350) is
// reproduced at the phase where it happens
constexpr int kFrcSlots = 3;
struct FrcField {
  double* slot[kFrcSlots] = {nullptr, nullptr, nullptr};
  double time[kFrcSlots] = {0.0, 0.0, 0.0};
  bool have[kFrcSlots] = {false, false, false};
  long n = 0;
  int kind = 0;   // ROMS_FRC_SURFACE / ROMS_FRC_BRY
};
struct TideData {
  int ntides = 0;
  std::vector<double> ftide;
  double *pr = nullptr, *pi = nullptr;                       // pot_Re/pot_Im (ntides x n2)
  double *zr = nullptr, *zi = nullptr, *ur = nullptr, *ui = nullptr, *vr = nullptr, *vi = nullptr;
};
// the in-step schedule (roms_gpu_frc_clock)
struct FrcStep {
  bool on = false;
  double start = 0.0;        // start_time [s] (time = start + dt*(iic-ntstart), main.F:373)
  long gen = 1;              // bumped when captured graphs would go stale
  std::vector<int> ids;      // fields with two or more records: interpolated inside the step
  double* dev = nullptr;     // [4 points][ids][slot a, slot b, cff1, cff2], then cos/sin of the tides
  size_t dev_n = 0;
  double* pin[4] = {};       // pinned staging ring, one event each
  hipEvent_t ev[4] = {};
  size_t pin_n = 0;
  int ring = 0;
};
struct FrcCtx {
  std::vector<FrcField> f;
  TideData tide;
  FrcStep st;
};
thread_local FrcCtx fc;

__global__ void __launch_bounds__(256) k_frc_interp(double* __restrict__ out, const double* __restrict__ a,
                                                    const double* __restrict__ b, double cff1, double cff2, long n) {
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) out[q] = cff1 * a[q] + cff2 * b[q];
}

// pair and weights from device memory (the in-step schedule, formed per step
// on the host): out = cff1*rec(it1) + cff2*rec(it2) with it1 = slot c[0],
// it2 = slot c[1] -- the graph keeps the slot pointers, the step picks the pair
struct FrcSlots {
  const double* s[kFrcSlots];
};
__global__ void __launch_bounds__(256) k_frc_interp_dev(double* __restrict__ out, FrcSlots r,
                                                        const double* __restrict__ c, long n) {
  const double* __restrict__ a = r.s[(int)c[0]];
  const double* __restrict__ b = r.s[(int)c[1]];
  const double c0 = c[2], c1 = c[3];
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) out[q] = c0 * a[q] + c1 * b[q];
}

// set_tides_tile, pot_tides part: ptide over (istrR-1..iendR, jstrR-1..jendR)
__global__ void __launch_bounds__(256) k_tide_pot(Bounds b, double* __restrict__ ptide, const double* __restrict__ pr,
                                                  const double* __restrict__ pim, const double* __restrict__ cs,
                                                  const double* __restrict__ sn, int ntides) {
  const int i0 = b.istrR - 1, j0 = b.jstrR - 1;
  const int ni = b.iendR - i0 + 1, nj = b.jendR - j0 + 1;
  const long p = blockIdx.x * 256L + threadIdx.x;
  if (p >= (long)ni * nj) return;
  const int i = i0 + (int)(p % ni), j = j0 + (int)(p / ni);
  const long ij = IJ(b, i, j);
  double v = 0.0;
  for (int t = 0; t < ntides; t++) {
    const double a = pr[ij + t * b.n2] * cs[t], c = pim[ij + t * b.n2] * sn[t];
    v = t == 0 ? a - c : v + a - c;   // tides.F:236-247: the first constituent initialises
  }
  ptide[ij] = v;
}

// set_tides_tile, bry_tides part: the open edges' zeta/ubar/vbar data
struct TideBry {
  double* z[4];
  double* u[4];
  double* v[4];
  const double *zr, *zi, *ur, *ui, *vr, *vi;
  int obc;
};
__global__ void __launch_bounds__(256) k_tide_bry(Bounds b, TideBry T, const double* __restrict__ cs,
                                                  const double* __restrict__ sn, int ntides) {
  const int side = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (!(T.obc & (1 << side))) return;
  const bool edge = side == 0 ? b.west_edge : side == 1 ? b.east_edge : side == 2 ? b.south_edge : b.north_edge;
  if (!edge) return;
  auto add = [&](double* dst, long m, const double* re, const double* im, int i, int j) {
    const long ij = IJ(b, i, j);
    double v = dst[m];
    for (int t = 0; t < ntides; t++) v = v + re[ij + t * b.n2] * cs[t] - im[ij + t * b.n2] * sn[t];
    dst[m] = v;
  };
  if (side < 2) {   // west / east: index j (tides.F:131-180)
    const int j = b.jstrR + p;
    if (j > b.jendR) return;
    const int iz = side == 0 ? b.istr - 1 : b.iend + 1;
    const int iu = side == 0 ? b.istrU - 1 : b.iend + 1;
    add(T.z[side], j, T.zr, T.zi, iz, j);
    add(T.u[side], j, T.ur, T.ui, iu, j);
    if (j >= b.jstr) add(T.v[side], j, T.vr, T.vi, iz, j);
  } else {          // south / north: index i (tides.F:182-228)
    const int i = b.istrR + p;
    if (i > b.iendR) return;
    const int jz = side == 2 ? b.jstr - 1 : b.jend + 1;
    const int jv = side == 2 ? b.jstrV - 1 : b.jend + 1;
    add(T.z[side], i, T.zr, T.zi, i, jz);
    if (i >= b.istr) add(T.u[side], i, T.ur, T.ui, i, jz);
    add(T.v[side], i, T.vr, T.vi, i, jv);
  }
}

int field_kind(int id) {
  if (id >= ROMS_zeta_west && id <= ROMS_t_north) return ROMS_FRC_BRY;
  return ROMS_FRC_SURFACE;
}

// set_tides_tile on the device (tides.F:106-254) with cos/sin of omT in dcs
// (ntides each); bry: also the open-boundary sums
void launch_tides(const Dev& d, hipStream_t s, const double* dcs, bool pot, bool bry) {
  const TideData& T = fc.tide;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  if (T.pr && pot) {
    const long n = (long)(b.iendR - b.istrR + 2) * (b.jendR - b.jstrR + 2);
    hipLaunchKernelGGL(k_tide_pot, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, F.ptide, T.pr, T.pi, dcs,
                       dcs + T.ntides, T.ntides);
  }
  if (T.zr && d.p.obc && bry) {
    TideBry B{};
    for (int q = 0; q < 4; q++) { B.z[q] = F.bzeta[q]; B.u[q] = F.bubar[q]; B.v[q] = F.bvbar[q]; }
    B.zr = T.zr; B.zi = T.zi; B.ur = T.ur; B.ui = T.ui; B.vr = T.vr; B.vi = T.vi;
    B.obc = d.p.obc;
    const int n = (b.Lm > b.Mm ? b.Lm : b.Mm) + 4;
    hipLaunchKernelGGL(k_tide_bry, dim3((unsigned)((n + 255) / 256), 4), dim3(256), 0, s, b, B, dcs, dcs + T.ntides,
                       T.ntides);
  }
}

// The record pair and weights set_frc_data uses at modtime [days]
// (roms_read_write.F:338-381).  The reference keeps (it1, it2) and, whenever
// times(it2) < modtime, refreshes to (it2, next record) (:341-350); for model
// times that only grow this is the earliest consecutive pair of the loaded
// records (in time order) whose later time is >= modtime.  Returns 0 with
// slot ia = it1, ib = it2 and cff1/cff2 (:376-377); 1 when modtime is past
// every loaded record (the reference would read the next record here: the
// host must load it first); -1 for the out-of-window check (:381, dt as the
// reference has it); -2 for records with equal times.
int frc_pair(const FrcField& F, double modtime, double dt, int& ia, int& ib, double& cff1, double& cff2) {
  int ord[kFrcSlots], n = 0;
  for (int s = 0; s < kFrcSlots; s++)
    if (F.have[s]) {
      int k = n++;
      while (k > 0 && F.time[ord[k - 1]] > F.time[s]) { ord[k] = ord[k - 1]; k--; }
      ord[k] = s;
    }
  if (n < 2) return -1;
  for (int k = 0; k + 1 < n; k++)
    if (!(F.time[ord[k + 1]] > F.time[ord[k]])) return -2;
  int k = 0;
  while (k + 2 < n && F.time[ord[k + 1]] < modtime) k++;
  ia = ord[k];
  ib = ord[k + 1];
  const double t1 = F.time[ia], t2 = F.time[ib];
  if (t2 < modtime) return 1;
  if (t1 > modtime + dt || t2 < modtime - dt) return -1;
  cff1 = (t2 - modtime) / (t2 - t1);
  cff2 = (modtime - t1) / (t2 - t1);
  return 0;
}

int nrec(const FrcField& F) {
  int n = 0;
  for (int s = 0; s < kFrcSlots; s++) n += F.have[s] ? 1 : 0;
  return n;
}

std::string frc_pair_error(int rc, int id, double modtime, const char* where, const char* entry) {
  const std::string f = " of field " + std::to_string(id) + " at model time " + std::to_string(modtime) + " days (" +
                        where + ")";
  if (rc == 1)
    return std::string(entry) + ": model time past the last forcing record" + f +
           ": load the next record first (set_frc_data refresh, roms_read_write.F:341-350)";
  if (rc == -2) return std::string(entry) + ": two records have the same time" + f;
  return std::string(entry) + ": model time outside the forcing records" + f + " (set_frc_data, roms_read_write.F:381-388)";
}

}  // namespace

long frc_step_gen() { return fc.st.on ? fc.st.gen : 0; }

int frc_step_prepare(hipStream_t s, const Dev& d, double dt, const roms_tlev& t, std::string& err) {
  FrcStep& st = fc.st;
  if (!st.on) return 0;
  std::vector<int> ids;
  for (int id = 0; id < (int)fc.f.size(); id++)
    if (nrec(fc.f[id]) >= 2) ids.push_back(id);
  if (ids != st.ids) { st.ids = ids; st.gen++; }
  const int nid = (int)ids.size(), nt = fc.tide.ntides;
  // bry_tides adds the constituents onto every open side's zeta/ubar/vbar
  // data after each set_bry_all (main.F:389-394, 438-441), which re-sets
  // those arrays first: each of them must be interpolated in-step, or the
  // sums would pile up from step to step
  if (nt > 0 && fc.tide.zr && d.p.obc) {
    const int edge[4] = {d.b.west_edge, d.b.east_edge, d.b.south_edge, d.b.north_edge};
    for (int side = 0; side < 4; side++) {
      if (!(d.p.obc & (1 << side)) || !edge[side]) continue;
      for (int var = 0; var < 3; var++) {
        const int id = ROMS_zeta_west + 4 * var + side;
        if (id >= (int)fc.f.size() || nrec(fc.f[id]) < 2) {
          err = "roms_gpu_step: boundary tides need two records of every open side's zeta/ubar/vbar data "
                "(set_bry_all re-sets them before set_tides, main.F:389-394); field " + std::to_string(id) +
                " has fewer";
          return -1;
        }
      }
    }
  }
  const size_t n = (size_t)16 * nid + 2 * nt + 1;
  if (st.dev_n < n) {
    if (st.dev) { (void)hipStreamSynchronize(s); (void)hipFree(st.dev); st.dev = nullptr; }
    if (hipMalloc(&st.dev, n * sizeof(double)) != hipSuccess) { err = "frc_step: allocation failed"; st.dev_n = 0; return -2; }
    st.dev_n = n;
    st.gen++;
  }
  if (st.pin_n < n) {
    for (int r = 0; r < 4; r++) {
      if (st.ev[r]) (void)hipEventSynchronize(st.ev[r]);
      if (st.pin[r]) (void)hipHostFree(st.pin[r]);
      st.pin[r] = nullptr;
      if (hipHostMalloc((void**)&st.pin[r], n * sizeof(double), hipHostMallocDefault) != hipSuccess) {
        err = "frc_step: pinned allocation failed";
        st.pin_n = 0;
        return -2;
      }
      if (!st.ev[r] && hipEventCreateWithFlags(&st.ev[r], hipEventDisableTiming) != hipSuccess) {
        err = "frc_step: event creation failed";
        return -2;
      }
    }
    st.pin_n = n;
  }
  // main.F:373-441: time of step n, and the four set_frc_data model times
  const double sec2day = 1. / 86400.;
  const double time = st.start + dt * (double)(t.iic - t.ntstart);
  const double tdays = time * sec2day;
  const double mod[4] = {tdays,                                      // set_forces, frc_time 'current'
                         tdays + 0.5 * dt * sec2day,                 // set_bry_all, '1/2 fwd'
                         tdays + 0.5 * dt * sec2day,                 // set_forces, '1/2 fwd'
                         (time + 0.5 * dt) * sec2day + dt * sec2day};  // set_bry_all, 'forward'
  static const char* const where[4] = {"set_forces 'current'", "set_bry_all '1/2 fwd'", "set_forces '1/2 fwd'",
                                        "set_bry_all 'forward'"};
  const int r = st.ring;
  (void)hipEventSynchronize(st.ev[r]);   // its previous copy has landed
  double* h = st.pin[r];
  for (int p = 0; p < 4; p++)
    for (int q = 0; q < nid; q++) {
      const FrcField& F = fc.f[ids[q]];
      double* c = h + ((size_t)p * nid + q) * 4;
      c[0] = c[1] = c[2] = c[3] = 0.0;
      if ((p % 2 == 0) != (F.kind == ROMS_FRC_SURFACE)) continue;
      int ia = 0, ib = 0;
      const int rc = frc_pair(F, mod[p], dt, ia, ib, c[2], c[3]);
      if (rc) {
        err = frc_pair_error(rc, ids[q], mod[p], where[p], "roms_gpu_step");
        return rc == 1 ? -8 : -1;
      }
      c[0] = ia;
      c[1] = ib;
    }
  for (int q = 0; q < nt; q++) {   // omT = ftide*(time + 0.5*dt) (tides.F:129), both set_tides calls
    const double omT = fc.tide.ftide[q] * (time + 0.5 * dt);
    h[(size_t)16 * nid + q] = std::cos(omT);
    h[(size_t)16 * nid + nt + q] = std::sin(omT);
  }
  if (hipMemcpyAsync(st.dev, h, n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipEventRecord(st.ev[r], s) != hipSuccess) {
    err = "frc_step: weight upload failed";
    return -2;
  }
  st.ring = (r + 1) % 4;
  return 0;
}

void frc_step_phase(const Dev& d, hipStream_t s, int phase, bool pot_tides) {
  const FrcStep& st = fc.st;
  if (!st.on || !st.dev) return;
  const int nid = (int)st.ids.size();
  const int kind = phase % 2 == 0 ? ROMS_FRC_SURFACE : ROMS_FRC_BRY;
  bool bry = false;
  for (int q = 0; q < nid; q++) {
    const int id = st.ids[q];
    const FrcField& F = fc.f[id];
    if (F.kind != kind) continue;
    if (id >= ROMS_zeta_west && id <= ROMS_vbar_north) bry = true;
    const long nb = (F.n + 255) / 256;
    FrcSlots r{};
    for (int k = 0; k < kFrcSlots; k++) r.s[k] = F.slot[k] ? F.slot[k] : F.slot[0];
    hipLaunchKernelGGL(k_frc_interp_dev, dim3((unsigned)(nb < 8192 ? nb : 8192)), dim3(256), 0, s, shim_field(id), r,
                       st.dev + ((size_t)phase * nid + q) * 4, F.n);
  }
  // set_tides after each set_bry_all (main.F:394,441): the boundary sums go
  // onto freshly interpolated zeta/ubar/vbar data only (frc_step_prepare
  // requires two records of every open side's arrays when tides are on)
  if (kind == ROMS_FRC_BRY && fc.tide.ntides > 0) launch_tides(d, s, st.dev + (size_t)16 * nid, pot_tides, bry);
}

void frc_free() {
  for (FrcField& f : fc.f)
    for (double*& p : f.slot)
      if (p) { (void)hipFree(p); p = nullptr; }
  fc.f.clear();
  FrcStep& st = fc.st;
  if (st.dev) { (void)hipFree(st.dev); st.dev = nullptr; }
  for (int r = 0; r < 4; r++) {
    if (st.ev[r]) { (void)hipEventSynchronize(st.ev[r]); (void)hipEventDestroy(st.ev[r]); st.ev[r] = nullptr; }
    if (st.pin[r]) { (void)hipHostFree(st.pin[r]); st.pin[r] = nullptr; }
  }
  const long gen = st.gen + 1;
  st = FrcStep{};
  st.gen = gen;
  TideData& T = fc.tide;
  for (double** p : {&T.pr, &T.pi, &T.zr, &T.zi, &T.ur, &T.ui, &T.vr, &T.vi})
    if (*p) { (void)hipFree(*p); *p = nullptr; }
  T = TideData{};
}

}  // namespace roms

using namespace roms;

extern "C" {

int roms_gpu_frc_record(int field_id, int slot, double rec_time, const double* data) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  if (field_id < 0 || field_id >= ROMS_NFIELDS || slot < 0 || slot >= kFrcSlots || !data) {
    *S.err = "roms_gpu_frc_record: bad field/slot/data";
    return -1;
  }
  const long n = shim_field_dev_count(field_id);   // the record lives in the device layout, like the field
  if ((long)fc.f.size() < ROMS_NFIELDS) fc.f.resize(ROMS_NFIELDS);
  FrcField& F = fc.f[field_id];
  if (!F.slot[slot]) {
    if (hipMalloc(&F.slot[slot], (size_t)n * sizeof(double)) != hipSuccess) {
      *S.err = "roms_gpu_frc_record: allocation failed";
      return -2;
    }
    // the upload fills only the host layout's rows and columns: the row-pitch
    // padding and the wide-ghost frame, which the interpolation copies into
    // the field and aligned tiles read, stay zero as dev_alloc leaves them
    // (ADVICE r4), ordered on the library stream before the upload
    if (hipMemsetAsync(F.slot[slot], 0, (size_t)n * sizeof(double), S.s) != hipSuccess) {
      *S.err = "roms_gpu_frc_record: zero fill failed";
      return -2;
    }
    fc.st.gen++;   // a captured step graph does not know this buffer
  }
  F.n = n;
  F.kind = field_kind(field_id);
  // ordered after the kernels already queued (a slot may still be read by an
  // interpolation of the current step)
  if (shim_field_h2d(field_id, F.slot[slot], data) != hipSuccess) {
    *S.err = "roms_gpu_frc_record: upload failed";
    return -2;
  }
  F.time[slot] = rec_time;
  F.have[slot] = true;
  return 0;
}

int roms_gpu_frc_interp(double modtime, int kinds) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  // set_frc_data compares times in days with modtime +- dt, dt in seconds
  // (roms_read_write.F:381): kept as the reference has it
  const double dtw = S.cfg->dt;
  struct Job { int id, ia, ib; double c1, c2; };
  std::vector<Job> jobs;
  for (int id = 0; id < (int)fc.f.size(); id++) {   // every check before anything is queued
    const FrcField& F = fc.f[id];
    if (nrec(F) < 2 || !(kinds & F.kind)) continue;
    Job j{id, 0, 0, 0.0, 0.0};
    const int rc = frc_pair(F, modtime, dtw, j.ia, j.ib, j.c1, j.c2);
    if (rc) {
      *S.err = frc_pair_error(rc, id, modtime, "frc_interp", "roms_gpu_frc_interp");
      return rc == 1 ? -8 : -1;
    }
    jobs.push_back(j);
  }
  for (const Job& j : jobs) {
    const FrcField& F = fc.f[j.id];
    double* out = shim_field(j.id);   // the field's device array
    const long n = F.n;
    const long nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_frc_interp, dim3((unsigned)(nb < 8192 ? nb : 8192)), dim3(256), 0, S.s, out, F.slot[j.ia],
                       F.slot[j.ib], j.c1, j.c2, n);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int roms_gpu_frc_clock(double start_time, int on) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  fc.st.on = on != 0;
  fc.st.start = start_time;
  fc.st.gen++;
  return 0;
}

int roms_gpu_set_tide_data(int ntides, const double* ftide, const double* pot_re, const double* pot_im,
                           const double* ztide_re, const double* ztide_im, const double* utide_re,
                           const double* utide_im, const double* vtide_re, const double* vtide_im) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  if (ntides < 0 || ntides > 64 || (ntides > 0 && !ftide)) { *S.err = "roms_gpu_set_tide_data: bad arguments"; return -1; }
  if ((pot_re == nullptr) != (pot_im == nullptr) || (ztide_re == nullptr) != (ztide_im == nullptr) ||
      (ztide_re == nullptr) != (utide_re == nullptr) || (utide_re == nullptr) != (utide_im == nullptr) ||
      (utide_re == nullptr) != (vtide_re == nullptr) || (vtide_re == nullptr) != (vtide_im == nullptr)) {
    *S.err = "roms_gpu_set_tide_data: real and imaginary parts (and z/u/v) must come together";
    return -1;
  }
  TideData& T = fc.tide;
  (void)hipStreamSynchronize(S.s);   // a queued step may still read the old constituents
  for (double** p : {&T.pr, &T.pi, &T.zr, &T.zi, &T.ur, &T.ui, &T.vr, &T.vi})
    if (*p) { (void)hipFree(*p); *p = nullptr; }
  fc.st.gen++;
  T.ntides = ntides;
  T.ftide.assign(ftide, ftide + ntides);
  // ntides planes of the host layout into the device layout (rows of nx2)
  const size_t nb = (size_t)ntides * S.d->b.n2 * sizeof(double);
  const long rows = (long)ntides * (S.d->b.Mm + 4);
  auto up = [&](double*& d, const double* h) -> bool {
    if (!h || ntides == 0) return true;
    return hipMalloc(&d, nb) == hipSuccess && shim_rows_h2d(d, h, rows) == hipSuccess;
  };
  if (!up(T.pr, pot_re) || !up(T.pi, pot_im) || !up(T.zr, ztide_re) || !up(T.zi, ztide_im) || !up(T.ur, utide_re) ||
      !up(T.ui, utide_im) || !up(T.vr, vtide_re) || !up(T.vi, vtide_im)) {
    *S.err = "roms_gpu_set_tide_data: upload failed";
    return -2;
  }
  return 0;
}

int roms_gpu_set_tides(double time) {
  ShimState S;
  int r = shim_enter(S);
  if (r) return r;
  TideData& T = fc.tide;
  if (T.ntides == 0) return 0;
  // omT = ftide*(time + 0.5*dt) (tides.F:129); cos/sin once per constituent, on the host
  std::vector<double> cs(T.ntides), sn(T.ntides);
  for (int t = 0; t < T.ntides; t++) {
    const double omT = T.ftide[t] * (time + 0.5 * S.cfg->dt);
    cs[t] = std::cos(omT);
    sn[t] = std::sin(omT);
  }
  double* dcs = shim_scratch_small(2 * T.ntides);
  if (!dcs) { *S.err = "roms_gpu_set_tides: scratch"; return -2; }
  std::vector<double> h(2 * T.ntides);
  for (int t = 0; t < T.ntides; t++) { h[t] = cs[t]; h[T.ntides + t] = sn[t]; }
  if (hipMemcpyAsync(dcs, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, S.s) != hipSuccess) {
    *S.err = "roms_gpu_set_tides: upload failed";
    return -2;
  }
  launch_tides(*S.d, S.s, dcs, S.cfg->pot_tides != 0, true);
  // the cos/sin buffer is reused by the next call: keep the host in step
  if (hipStreamSynchronize(S.s) != hipSuccess) { *S.err = "roms_gpu_set_tides: kernel failed"; return -3; }
  return 0;
}

}  // extern "C"
