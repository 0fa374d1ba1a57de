// k_bc_exchange.hip -- halo wrap for ranks that are their own periodic
// neighbour, and the closed-wall lateral boundary conditions.
//
// Periodic self-exchange reproduces mpi_exchanges.F:528-670 for NP=1 in a
// periodic direction (mpi_setup.F:65-67): the E/W message spans rows
// jl0..jl1 = 0..Mm+1, the N/S message columns 0..Lm+1, corners travel
// separately; since every message is packed from the pre-exchange array the
// final halo is the periodic wrap of the interior.  Closed-wall BCs restate
// u3dbc_im.F:4, v3dbc_im.F:4, t3dbc_im.F:4 with no OBC_* switch defined.
#include "halo.h"
#include "roms_dev.h"

namespace roms {

__global__ void __launch_bounds__(256) k_periodic_wrap(Bounds b, ExchList L) {
  const int Lm = b.Lm, Mm = b.Mm;
  const int W = Lm + 4;                 // i = -1..Lm+2 (not the row padding)
  const int nrow = 4 * W;               // rows j=-1,0,Mm+1,Mm+2, all i
  const int ncol = 4 * Mm;              // columns i=-1,0,Lm+1,Lm+2, j=1..Mm
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nrow + ncol) return;
  int i, j;
  if (p < nrow) {
    const int r = p / W;
    i = p - r * W - 1;
    j = r < 2 ? r - 1 : Mm - 1 + r;
  } else {
    // the four halo columns of one row j are neighbouring threads, so each
    // pair (-1,0) / (Lm+1,Lm+2) shares one line per access
    const int q = p - nrow;
    const int c = q & 3;
    j = (q >> 2) + 1;
    i = c < 2 ? c - 1 : Lm - 1 + c;
  }
  const bool xh = i < 1 || i > Lm, yh = j < 1 || j > Mm;
  const int wi = i < 1 ? i + Lm : (i > Lm ? i - Lm : i);
  const int wj = j < 1 ? j + Mm : (j > Mm ? j - Mm : j);
  int si, sj;
  if (xh && yh) {
    if (b.ew_periodic && b.ns_periodic) { si = wi; sj = wj; }
    else if (b.ew_periodic && j >= 0 && j <= Mm + 1) { si = wi; sj = j; }
    else if (b.ns_periodic && i >= 0 && i <= Lm + 1) { si = i; sj = wj; }
    else return;
  } else if (xh) {
    if (!b.ew_periodic) return;
    si = wi; sj = j;
  } else if (yh) {
    if (!b.ns_periodic) return;
    si = i; sj = wj;
  } else {
    return;
  }
  // grid.y enumerates the (array, level) pairs of the list: one copy per thread
  int lev = blockIdx.y, q = 0;
  while (q < L.n - 1 && lev >= L.nlev[q]) { lev -= L.nlev[q]; q++; }
  if (lev >= L.nlev[q]) return;
  const long off = (long)lev * b.n2;
  L.p[q][IJ(b, i, j) + off] = L.p[q][IJ(b, si, sj) + off];
}

void launch_exchange_list(const Dev& d, hipStream_t s, const ExchList& L) {
  const Bounds& b = d.b;
  if (d.halo && d.halo->comm) {
    Halo& H = *const_cast<Halo*>(d.halo);
    if (H.defer > 0) {   // a deferred producer's exchange (enqueue_step): onto the halo stream
      (void)halo_fork_exchange(H, s, L);
      return;
    }
    // one order on the transport: every exchange follows the forked ones
    halo_join(H, s);
    halo_exchange(H, s, L);
    return;
  }
  if (!b.ew_periodic && !b.ns_periodic) return;
  const int n = 4 * (b.Lm + 4) + 4 * b.Mm;
  int nl = 0;
  for (int q = 0; q < L.n; q++) nl += L.nlev[q];
  if (nl == 0) return;
  hipLaunchKernelGGL(k_periodic_wrap, dim3((n + 255) / 256, nl), dim3(256), 0, s, b, L);
}
bool rim_overlap_on(const Dev& d, const Range& R) {
  return d.halo && d.halo->comm && d.halo->overlap3d && R.i1 - R.i0 >= 7 && R.j1 - R.j0 >= 7;
}
void rim_fork(const Dev& d, hipStream_t s, const ExchList& L) { halo_fork_exchange(*const_cast<Halo*>(d.halo), s, L); }
void rim_join(const Dev& d, hipStream_t s) { halo_join(*const_cast<Halo*>(d.halo), s); }
bool tracer_exch_list(const Dev& d, int tlev, ExchList& L) {
  const Bounds& b = d.b;
  if (b.NT > 8) return false;
  L = ExchList{};
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    L.p[L.n] = d.f.t + (long)(tlev - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    L.nlev[L.n++] = b.N;
  }
  return true;
}
void launch_exchange_tracers(const Dev& d, hipStream_t s, int tlev) {
  const Bounds& b = d.b;
  ExchList L{};
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    L.p[L.n] = d.f.t + (long)(tlev - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    L.nlev[L.n++] = b.N;
    if (L.n == 8 || itrc == b.NT) {
      launch_exchange_list(d, s, L);
      L.n = 0;
    }
  }
}
void launch_exchange(const Dev& d, hipStream_t s, double* a, int nlev) {
  ExchList L{};
  L.p[0] = a; L.nlev[0] = nlev; L.n = 1;
  launch_exchange_list(d, s, L);
}

// ---- 3-D closed-wall BCs: one lane per (edge point, level k = 1 + blockIdx.y) ----
// phase 0 sets the wall-normal component, phase 1 the tangential one (which
// reads the former, as the sequential reference loop order implies)
__global__ void k_u3dbc(Bounds b, double gamma2, const double* __restrict__ umask, double* __restrict__ u,
                        int nnew, int phase) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int nj = b.jend - b.jstr + 1, ni = b.iendR - b.istr + 1;
  if (phase == 0) {
    if (p >= nj) return;
    const int j = b.jstr + p;
    if (b.west_edge) u[IJKL(b, b.istr, j, k, nnew)] = 0.0;
    if (b.east_edge) u[IJKL(b, b.iend + 1, j, k, nnew)] = 0.0;
  } else if (p < ni) {
    const int i = b.istr + p;
    if (b.south_edge)
      u[IJKL(b, i, b.jstr - 1, k, nnew)] = gamma2 * u[IJKL(b, i, b.jstr, k, nnew)] * umask[IJ(b, i, b.jstr - 1)];
    if (b.north_edge)
      u[IJKL(b, i, b.jend + 1, k, nnew)] = gamma2 * u[IJKL(b, i, b.jend, k, nnew)] * umask[IJ(b, i, b.jend + 1)];
  }
}
__global__ void k_v3dbc(Bounds b, double gamma2, const double* __restrict__ vmask, double* __restrict__ v,
                        int nnew, int phase) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int ni = b.iend - b.istr + 1, nj = b.jendR - b.jstr + 1;
  if (phase == 0) {
    if (p >= ni) return;
    const int i = b.istr + p;
    if (b.south_edge) v[IJKL(b, i, b.jstr, k, nnew)] = 0.0;
    if (b.north_edge) v[IJKL(b, i, b.jend + 1, k, nnew)] = 0.0;
  } else if (p < nj) {
    const int j = b.jstr + p;
    if (b.west_edge)
      v[IJKL(b, b.istr - 1, j, k, nnew)] = gamma2 * v[IJKL(b, b.istr, j, k, nnew)] * vmask[IJ(b, b.istr - 1, j)];
    if (b.east_edge)
      v[IJKL(b, b.iend + 1, j, k, nnew)] = gamma2 * v[IJKL(b, b.iend, j, k, nnew)] * vmask[IJ(b, b.iend + 1, j)];
  }
}
// t3dbc: edges first, corners in a second launch (they read edge values)
__global__ void k_t3dbc_edges(Bounds b, const double* __restrict__ rmask, double* __restrict__ t, int nnew, int itrc) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int nj = b.jend - b.jstr + 1, ni = b.iend - b.istr + 1;
  if (p < nj) {
    const int j = b.jstr + p;
    if (b.west_edge) t[TIDX(b, b.istr - 1, j, k, nnew, itrc)] = t[TIDX(b, b.istr, j, k, nnew, itrc)] * rmask[IJ(b, b.istr - 1, j)];
    if (b.east_edge) t[TIDX(b, b.iend + 1, j, k, nnew, itrc)] = t[TIDX(b, b.iend, j, k, nnew, itrc)] * rmask[IJ(b, b.iend + 1, j)];
  } else if (p < nj + ni) {
    const int i = b.istr + (p - nj);
    if (b.south_edge) t[TIDX(b, i, b.jstr - 1, k, nnew, itrc)] = t[TIDX(b, i, b.jstr, k, nnew, itrc)] * rmask[IJ(b, i, b.jstr - 1)];
    if (b.north_edge) t[TIDX(b, i, b.jend + 1, k, nnew, itrc)] = t[TIDX(b, i, b.jend, k, nnew, itrc)] * rmask[IJ(b, i, b.jend + 1)];
  }
}
__device__ void t_corner(const Bounds& b, const double* rm, double* t, int nnew, int itrc, int k, int ic, int jc,
                         int ia, int ja, int ib, int jb) {
  double cff = rm[IJ(b, ia, ja)] + rm[IJ(b, ib, jb)];
  if (cff > 0.0) {
    cff = 1.0 / cff;
    t[TIDX(b, ic, jc, k, nnew, itrc)] = cff * (rm[IJ(b, ia, ja)] * t[TIDX(b, ia, ja, k, nnew, itrc)] +
                                               rm[IJ(b, ib, jb)] * t[TIDX(b, ib, jb, k, nnew, itrc)]);
  } else {
    t[TIDX(b, ic, jc, k, nnew, itrc)] = 0.0;
  }
}
// one lane per (corner, level): corner c = lane & 3, k = 1 + lane / 4
__global__ void k_t3dbc_corners(Bounds b, const double* __restrict__ rm, double* __restrict__ t, int nnew, int itrc) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = p & 3, k = 1 + (p >> 2);
  if (k > b.N) return;
  const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
  if (c == 0 && b.south_edge && b.west_edge) t_corner(b, rm, t, nnew, itrc, k, is - 1, js - 1, is, js - 1, is - 1, js);
  if (c == 1 && b.south_edge && b.east_edge) t_corner(b, rm, t, nnew, itrc, k, ie + 1, js - 1, ie, js - 1, ie + 1, js);
  if (c == 2 && b.north_edge && b.west_edge) t_corner(b, rm, t, nnew, itrc, k, is - 1, je + 1, is, je + 1, is - 1, je);
  if (c == 3 && b.north_edge && b.east_edge) t_corner(b, rm, t, nnew, itrc, k, ie + 1, je + 1, ie, je + 1, ie + 1, je);
}

static inline bool closed_any(const Bounds& b) { return b.west_edge || b.east_edge || b.south_edge || b.north_edge; }

void launch_u3dbc_obc(const Dev& d, hipStream_t s, const Tlev& t);
void launch_v3dbc_obc(const Dev& d, hipStream_t s, const Tlev& t);
void launch_t3dbc_obc_edges(const Dev& d, hipStream_t s, const Tlev& t, int itrc);

void launch_u3dbc(const Dev& d, hipStream_t s, const Tlev& t) {
  if (!closed_any(d.b)) return;
  if (d.p.obc) { launch_u3dbc_obc(d, s, t); return; }
  const int n = (d.b.jend - d.b.jstr + 1) > (d.b.iendR - d.b.istr + 1) ? (d.b.jend - d.b.jstr + 1) : (d.b.iendR - d.b.istr + 1);
  for (int ph = 0; ph < 2; ph++)
    hipLaunchKernelGGL(k_u3dbc, dim3((n + 255) / 256, d.b.N), dim3(256), 0, s, d.b, d.p.gamma2, d.f.umask, d.f.u,
                       t.nnew, ph);
}
void launch_v3dbc(const Dev& d, hipStream_t s, const Tlev& t) {
  if (!closed_any(d.b)) return;
  if (d.p.obc) { launch_v3dbc_obc(d, s, t); return; }
  const int n = (d.b.iend - d.b.istr + 1) > (d.b.jendR - d.b.jstr + 1) ? (d.b.iend - d.b.istr + 1) : (d.b.jendR - d.b.jstr + 1);
  for (int ph = 0; ph < 2; ph++)
    hipLaunchKernelGGL(k_v3dbc, dim3((n + 255) / 256, d.b.N), dim3(256), 0, s, d.b, d.p.gamma2, d.f.vmask, d.f.v,
                       t.nnew, ph);
}
void launch_t3dbc(const Dev& d, hipStream_t s, const Tlev& t, int itrc) {
  if (!closed_any(d.b)) return;
  const int n = (d.b.jend - d.b.jstr + 1) + (d.b.iend - d.b.istr + 1);
  if (d.p.obc) launch_t3dbc_obc_edges(d, s, t, itrc);
  else hipLaunchKernelGGL(k_t3dbc_edges, dim3((n + 255) / 256, d.b.N), dim3(256), 0, s, d.b, d.f.rmask, d.f.t, t.nnew, itrc);
  hipLaunchKernelGGL(k_t3dbc_corners, dim3((4 * d.b.N + 255) / 256), dim3(256), 0, s, d.b, d.f.rmask, d.f.t, t.nnew,
                     itrc);
}

}  // namespace roms
