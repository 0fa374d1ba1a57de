// shim_state.h -- what the C-ABI modules outside roms_shim.cpp (rst_io.hip)
// see of the calling thread's library state.
#pragma once
#include <vector>
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/roms_gpu.h"
#include "roms_dev.h"

namespace roms {
struct ShimState {
  Dev* d = nullptr;
  hipStream_t s = nullptr;
  const roms_dims* dims = nullptr;
  const roms_cfg* cfg = nullptr;
  std::string* err = nullptr;
};
// The entry checks of every routine (initialised, no failed halo wait, fast-
// loop exchange joined); fills S.  Returns 0 or the negative error code.
int shim_enter(ShimState& S, bool read_only = false);   // read_only: the call changes no model field
void shim_set_error(const std::string& e);
void io_free();
// A blocking copy ordered on the library's stream.  The kernels run on
// non-blocking streams, which do not wait for null-stream work, so plain
// hipMemcpy/hipMemset can race with them (a pageable hipMemcpy may return
// before its DMA has landed).
inline hipError_t copy_on(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
  return e != hipSuccess ? e : hipStreamSynchronize(s);
}   // rst_io.hip: joins the writer, frees staging (roms_gpu_finalize)
void launch_fill_ones(double* p, long n, hipStream_t s);                               // k_diag.hip (self-test)
void launch_count_nonzero(const double* p, long n, unsigned long long* cnt, hipStream_t s, double v = 0.0);   // elements != v
void frc_free();  // k_forcing.hip: forcing records and tide data (roms_gpu_finalize)
// In-step forcing (roms_gpu_frc_clock, k_forcing.hip): the set_forces /
// set_bry_all / set_tides points of roms_step run inside roms_gpu_step.
// frc_step_prepare forms the step's interpolation weights on the host and
// queues them to the device before the step's kernels (0 or negative error);
// frc_step_phase enqueues the interpolations of one point (0: surface at
// 'current', 1: boundary at '1/2 fwd' + set_tides, 2: surface at '1/2 fwd',
// 3: boundary at 'forward' + set_tides), reading the weights from device
// memory so a captured step graph replays them; frc_step_gen changes
// whenever a captured graph would hold stale buffers or field lists.
int frc_step_prepare(hipStream_t s, const Dev& d, double dt, const roms_tlev& t, std::string& err);
void frc_step_phase(const Dev& d, hipStream_t s, int phase, bool pot_tides);
long frc_step_gen();
double* shim_field(int field_id);          // device array of a field (nullptr if absent)
long shim_field_dev_count(int field_id);   // elements of a field in the device layout (row pitch nx2)
// host-layout field data (the ABI's, rows of Lm+4) into a device-layout
// array of the field's shape, blocking on the library stream
hipError_t shim_field_h2d(int field_id, double* dev, const double* host);
hipError_t shim_rows_h2d(double* dev, const double* host, long rows);   // `rows` rows of Lm+4 (whole planes of Mm+4) -> device planes
// row r = p*prow + q: dst[p*dplane + q*dpitch + c] = src[p*splane + q*spitch + c], c < width (device arrays; k_diag.hip)
void launch_rows_copy(double* dst, long dpitch, long dplane, const double* src, long spitch, long splane, long width,
                      long rows, long prow, hipStream_t s);
double* shim_scratch_small(long n);        // small device scratch owned by the context (>= n doubles)
// step3d_uv2's closed-edge column lists (k_step3d_uv.hip): (dir, i, j) triples
void uv2_edge_lists(const Bounds& b, std::vector<int>& couple, std::vector<int>& flux);
}  // namespace roms
