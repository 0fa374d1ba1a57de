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

struct FrcField {
  double* slot[2] = {nullptr, nullptr};
  double time[2] = {0.0, 0.0};
  bool have[2] = {false, false};
  long n = 0;
  int kind = 0;   // ROMS_FRC_SURFACE / ROMS_FRC_BRY
};
struct TideData {
  int ntides = 0;
  std::vector<double> ftide;
  double *pr = nullptr, *pi = nullptr;                       // pot_Re/pot_Im (ntides x n2)
  double *zr = nullptr, *zi = nullptr, *ur = nullptr, *ui = nullptr, *vr = nullptr, *vi = nullptr;
};
struct FrcCtx {
  std::vector<FrcField> f;
  TideData tide;
};
thread_local FrcCtx fc;

__global__ void __launch_bounds__(256) k_frc_interp(double* __restrict__ out, const double* __restrict__ a,
                                                    const double* __restrict__ b, double cff1, double cff2, long n) {
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256L) out[q] = cff1 * a[q] + cff2 * b[q];
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

}  // namespace

void frc_free() {
  for (FrcField& f : fc.f)
    for (double*& p : f.slot)
      if (p) { (void)hipFree(p); p = nullptr; }
  fc.f.clear();
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
  if (field_id < 0 || field_id >= ROMS_NFIELDS || slot < 0 || slot > 1 || !data) {
    *S.err = "roms_gpu_frc_record: bad field/slot/data";
    return -1;
  }
  const long n = roms_gpu_field_size(field_id);
  if ((long)fc.f.size() < ROMS_NFIELDS) fc.f.resize(ROMS_NFIELDS);
  FrcField& F = fc.f[field_id];
  if (!F.slot[slot]) {
    if (hipMalloc(&F.slot[slot], (size_t)n * sizeof(double)) != hipSuccess) {
      *S.err = "roms_gpu_frc_record: allocation failed";
      return -2;
    }
  }
  F.n = n;
  F.kind = field_kind(field_id);
  // ordered after the kernels already queued (a slot may still be read by an
  // interpolation of the current step)
  if (hipMemcpyAsync(F.slot[slot], data, (size_t)n * sizeof(double), hipMemcpyHostToDevice, S.s) != hipSuccess ||
      hipStreamSynchronize(S.s) != hipSuccess) {
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
  for (int id = 0; id < (int)fc.f.size(); id++) {
    FrcField& F = fc.f[id];
    if (!(F.have[0] && F.have[1]) || !(kinds & F.kind)) continue;
    const int it1 = F.time[0] <= F.time[1] ? 0 : 1, it2 = 1 - it1;
    const double t1 = F.time[it1], t2 = F.time[it2];
    if (!(t2 > t1)) { *S.err = "roms_gpu_frc_interp: the two records of a field have the same time"; return -1; }
    // set_frc_data's out-of-window check (roms_read_write.F:381-388)
    if (t1 > modtime + dtw || t2 < modtime - dtw) {
      *S.err = "roms_gpu_frc_interp: model time outside the records of field " + std::to_string(id);
      return -1;
    }
    const double cff1 = (t2 - modtime) / (t2 - t1), cff2 = (modtime - t1) / (t2 - t1);
    double* out = shim_field(id);   // the field's device array
    const long n = F.n;
    const long nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_frc_interp, dim3((unsigned)(nb < 8192 ? nb : 8192)), dim3(256), 0, S.s, out, F.slot[it1],
                       F.slot[it2], cff1, cff2, n);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
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
  for (double** p : {&T.pr, &T.pi, &T.zr, &T.zi, &T.ur, &T.ui, &T.vr, &T.vi})
    if (*p) { (void)hipFree(*p); *p = nullptr; }
  T.ntides = ntides;
  T.ftide.assign(ftide, ftide + ntides);
  const size_t nb = (size_t)ntides * S.d->b.n2 * sizeof(double);
  auto up = [&](double*& d, const double* h) -> bool {
    if (!h || ntides == 0) return true;
    return hipMalloc(&d, nb) == hipSuccess && copy_on(d, h, nb, hipMemcpyHostToDevice, S.s) == hipSuccess;
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
  const Bounds& b = S.d->b;
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
  const Fields& F = S.d->f;
  if (T.pr && S.cfg->pot_tides) {
    const long n = (long)(b.iendR - b.istrR + 2) * (b.jendR - b.jstrR + 2);
    hipLaunchKernelGGL(k_tide_pot, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S.s, b, F.ptide, T.pr, T.pi, dcs,
                       dcs + T.ntides, T.ntides);
  }
  if (T.zr && S.d->p.obc) {
    TideBry B{};
    for (int q = 0; q < 4; q++) { B.z[q] = F.bzeta[q]; B.u[q] = F.bubar[q]; B.v[q] = F.bvbar[q]; }
    B.zr = T.zr; B.zi = T.zi; B.ur = T.ur; B.ui = T.ui; B.vr = T.vr; B.vi = T.vi;
    B.obc = S.d->p.obc;
    const int n = (b.Lm > b.Mm ? b.Lm : b.Mm) + 4;
    hipLaunchKernelGGL(k_tide_bry, dim3((unsigned)((n + 255) / 256), 4), dim3(256), 0, S.s, b, B, dcs,
                       dcs + T.ntides, T.ntides);
  }
  // the cos/sin buffer is reused by the next call: keep the host in step
  if (hipStreamSynchronize(S.s) != hipSuccess) { *S.err = "roms_gpu_set_tides: kernel failed"; return -3; }
  return 0;
}

}  // extern "C"
