// k_obc.hip -- lateral boundary conditions with open edges: the Iceland switch
// set (Examples/Iceland/Iceland_parent/cppdefs.opt) OBC_M3ORLANSKI for u, v
// and OBC_TORLANSKI for tracers with M3_FRC_BRY / T_FRC_BRY boundary data and
// the binding velocity ubind; closed walls on the edges not flagged open.
// Restates u3dbc_im.F:4-424, v3dbc_im.F:4-433 and t3dbc_im.F:4-422 with the
// reference's arithmetic order (oracle/oracle_obc.c is the CPU twin).
//
// One lane per (edge point, level k = 1 + blockIdx.y).  A routine runs in the
// reference's dependency order: the wall-normal edges (phase 0), the
// tangential edges (phase 1, a closed tangential edge reads the normal value
// next to it), then the corners of adjacent open edges (phase 2).  Each lane
// forms the radiation gradients it needs from time level nstp itself, so the
// grad(:,:) scratch strips of the reference need no storage.
#include "roms_dev.h"

namespace roms {

namespace {
constexpr double kEps = 1.E-33;

__device__ __forceinline__ double fmx(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double fmn(double a, double b) { return a < b ? a : b; }

// u3dbc_im.F:50-110 (normal component, Orlanski radiation): bs = boundary
// value at nstp, i1s / i1n first interior point at nstp / nnew, i2n second
// interior at nnew; gb0/gb1 the boundary column's tangential differences at
// m, m+1, gi0/gi1 the first interior column's.
__device__ __forceinline__ double orl_normal(double bs, double i1s, double i1n, double i2n, double gb0, double gb1,
                                             double gi0, double gi1, bool& inflow) {
  const double dft = i1s - i1n, dfx = i1n - i2n;
  const double dfy = (dft * (gi0 + gi1) > 0.) ? gi0 : gi1;
  const double cff = fmx(dfx * dfx + dfy * dfy, kEps);
  double cy = fmn(cff, fmx(dft * dfy, -cff));
  double cx = dft * dfx;
  inflow = false;
  if (cx < 0.) { cx = 0.; cy = 0.; inflow = true; }
  return (cff * bs + cx * i1n - fmax0(cy) * gb0 - fmin0(cy) * gb1) / (cff + cx);
}
// tangential component (u3dbc_im.F:232-262): cx, cy advective Courant numbers
__device__ __forceinline__ double orl_tangential(double& cx, double cy, double bs, double is, double gb0, double gb1,
                                                 double gi0, double gi1, double& cext) {
  if (cx > 0.) cext = 0.;
  else { cext = -cx; cx = 0.; }
  return (1. - cx) * (bs - fmax0(cy) * gb0 - fmin0(cy) * gb1) + cx * (is - fmax0(cy) * gi0 - fmin0(cy) * gi1);
}
__device__ __forceinline__ bool obc_on(const Dev& d, int side) { return (d.p.obc >> side) & 1; }
// boundary data: west/east (index j, 0:Mm+1), south/north (index i, 0:Lm+1)
__device__ __forceinline__ int nbry(const Bounds& b, int side) { return side < 2 ? b.Mm + 2 : b.Lm + 2; }
}  // namespace

// ---- u3dbc: phase 0 western/eastern (normal), 1 southern/northern
// (tangential), 2 corners ----
__global__ void __launch_bounds__(256) k_u3dbc_obc(Dev d, int nnew, int nstp, int nrhs, double dtfwd, int phase) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
  const double* u = F.u;
  auto U = [&](int i, int j, int l) { return u[IJKL(b, i, j, k, l)]; };
  auto V = [&](int i, int j, int l) { return F.v[IJKL(b, i, j, k, l)]; };
  auto pm = [&](int i, int j) { return F.pm[IJ(b, i, j)]; };
  auto pn = [&](int i, int j) { return F.pn[IJ(b, i, j)]; };
  auto pmask = [&](int i, int j) { return F.pmask[IJ(b, i, j)]; };
  double* un = F.u;
  if (phase == 0) {
    const int j = js + p;
    if (j > je) return;
    if (b.west_edge) {
      double val = 0.0;
      if (obc_on(d, 0)) {
        auto gr = [&](int i, int jj) { return (U(i, jj, nstp) - U(i, jj - 1, nstp)) * pmask(i, jj); };
        bool inflow;
        const double ub = orl_normal(U(is, j, nstp), U(is + 1, j, nstp), U(is + 1, j, nnew), U(is + 2, j, nnew),
                                     gr(is, j), gr(is, j + 1), gr(is + 1, j), gr(is + 1, j + 1), inflow);
        const double bry = F.bu[0][j + (long)nbry(b, 0) * (k - 1)];
        double cext = 0.;
        if (inflow) {
          cext = bry > 0. ? bry : d.p.ubind;
          cext = cext * dtfwd * 0.5 * (pm(is - 1, j) + pm(is, j));
        }
        if (F.ub[0]) cext = fmax(cext, fmin(F.ub[0][j], 1.0));   // SPONGE_TUNE ub_west (u3dbc_im.F:101-103)
        val = (1. - cext) * ub + cext * bry;
        val = val * F.umask[IJ(b, is, j)];
      }
      un[IJKL(b, is, j, k, nnew)] = val;
    }
    if (b.east_edge) {
      double val = 0.0;
      if (obc_on(d, 1)) {
        auto gr = [&](int i, int jj) { return (U(i, jj, nstp) - U(i, jj - 1, nstp)) * pmask(i, jj); };
        bool inflow;
        const double ub = orl_normal(U(ie + 1, j, nstp), U(ie, j, nstp), U(ie, j, nnew), U(ie - 1, j, nnew),
                                     gr(ie + 1, j), gr(ie + 1, j + 1), gr(ie, j), gr(ie, j + 1), inflow);
        const double bry = F.bu[1][j + (long)nbry(b, 1) * (k - 1)];
        double cext = 0.;
        if (inflow) {
          cext = bry < 0. ? -bry : d.p.ubind;
          cext = cext * dtfwd * 0.5 * (pm(ie, j) + pm(ie + 1, j));
        }
        if (F.ub[1]) cext = fmax(cext, fmin(F.ub[1][j], 1.0));   // SPONGE_TUNE ub_east (u3dbc_im.F:190-192)
        val = (1. - cext) * ub + cext * bry;
        val = val * F.umask[IJ(b, ie + 1, j)];
      }
      un[IJKL(b, ie + 1, j, k, nnew)] = val;
    }
  } else if (phase == 1) {
    for (int side = 2; side <= 3; side++) {
      const bool edge = side == 2 ? b.south_edge : b.north_edge;
      if (!edge) continue;
      const int jb = side == 2 ? js - 1 : je + 1, ji = side == 2 ? js : je;
      if (obc_on(d, side)) {
        const int i = b.istrU + p;
        if (i > ie) continue;
        auto gr = [&](int ii, int jj) { return U(ii + 1, jj, nstp) - U(ii, jj, nstp); };
        double cx, cy;
        if (side == 2) {
          cx = -0.125 * dtfwd * (V(i, js, nrhs) + V(i - 1, js, nrhs)) * (pn(i, js - 1) + pn(i - 1, js - 1) + pn(i, js) + pn(i - 1, js));
          cy = 0.125 * dtfwd * (U(i, js - 1, nrhs) + U(i, js, nrhs)) * (pm(i, js - 1) + pm(i - 1, js - 1) + pm(i, js) + pm(i - 1, js));
        } else {
          cx = 0.125 * dtfwd * (V(i, je + 1, nrhs) + V(i - 1, je + 1, nrhs)) * (pn(i, je + 1) + pn(i - 1, je + 1) + pn(i, je) + pn(i - 1, je));
          cy = 0.125 * dtfwd * (U(i, je, nrhs) + U(i, je + 1, nrhs)) * (pm(i, je + 1) + pm(i - 1, je + 1) + pm(i, je) + pm(i - 1, je));
        }
        double cext;
        double val = orl_tangential(cx, cy, U(i, jb, nstp), U(i, ji, nstp), gr(i - 1, jb), gr(i, jb), gr(i - 1, ji),
                                    gr(i, ji), cext);
        if (F.ub[side]) cext = fmax(cext, fmin(F.ub[side][i], 1.0));   // ub_south/north (u3dbc_im.F:262-264,341-343)
        val = (1. - cext) * val + cext * F.bu[side][i + (long)nbry(b, side) * (k - 1)];
        un[IJKL(b, i, jb, k, nnew)] = val * F.umask[IJ(b, i, jb)];
      } else {
        const int i0 = b.ew_periodic ? b.istrU : is, i1 = b.ew_periodic ? ie : b.iendR;
        const int i = i0 + p;
        if (i > i1) continue;
        un[IJKL(b, i, jb, k, nnew)] = d.p.gamma2 * u[IJKL(b, i, ji, k, nnew)] * F.umask[IJ(b, i, jb)];
      }
    }
  } else if (p == 0) {
    const bool W = b.west_edge && obc_on(d, 0), E = b.east_edge && obc_on(d, 1);
    const bool S = b.south_edge && obc_on(d, 2), N = b.north_edge && obc_on(d, 3);
    auto Un = [&](int i, int j) -> double& { return un[IJKL(b, i, j, k, nnew)]; };
    if (S && W) Un(is, js - 1) = 0.5 * (Un(is + 1, js - 1) + Un(is, js));
    if (S && E) Un(ie + 1, js - 1) = 0.5 * (Un(ie, js - 1) + Un(ie + 1, js));
    if (N && W) Un(is, je + 1) = 0.5 * (Un(is + 1, je + 1) + Un(is, je));
    if (N && E) Un(ie + 1, je + 1) = 0.5 * (Un(ie, je + 1) + Un(ie + 1, je));
  }
}

// ---- v3dbc: phase 0 southern/northern (normal), 1 western/eastern
// (tangential), 2 corners ----
__global__ void __launch_bounds__(256) k_v3dbc_obc(Dev d, int nnew, int nstp, int nrhs, double dtfwd, int phase) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
  const double* v = F.v;
  auto U = [&](int i, int j, int l) { return F.u[IJKL(b, i, j, k, l)]; };
  auto V = [&](int i, int j, int l) { return v[IJKL(b, i, j, k, l)]; };
  auto pm = [&](int i, int j) { return F.pm[IJ(b, i, j)]; };
  auto pn = [&](int i, int j) { return F.pn[IJ(b, i, j)]; };
  auto pmask = [&](int i, int j) { return F.pmask[IJ(b, i, j)]; };
  double* vn = F.v;
  if (phase == 0) {
    const int i = is + p;
    if (i > ie) return;
    if (b.south_edge) {
      double val = 0.0;
      if (obc_on(d, 2)) {
        auto gr = [&](int ii, int jj) { return (V(ii, jj, nstp) - V(ii - 1, jj, nstp)) * pmask(ii, jj); };
        bool inflow;
        const double vb = orl_normal(V(i, js, nstp), V(i, js + 1, nstp), V(i, js + 1, nnew), V(i, js + 2, nnew),
                                     gr(i, js), gr(i + 1, js), gr(i, js + 1), gr(i + 1, js + 1), inflow);
        const double bry = F.bv[2][i + (long)nbry(b, 2) * (k - 1)];
        double cext = 0.;
        if (inflow) {
          cext = bry > 0. ? bry : d.p.ubind;
          cext = cext * dtfwd * 0.5 * (pn(i, js - 1) + pn(i, js));
        }
        if (F.ub[2]) cext = fmax(cext, fmin(F.ub[2][i], 1.0));   // SPONGE_TUNE ub_south (v3dbc_im.F:97-99)
        val = (1. - cext) * vb + cext * bry;
        val = val * F.vmask[IJ(b, i, js)];
      }
      vn[IJKL(b, i, js, k, nnew)] = val;
    }
    if (b.north_edge) {
      double val = 0.0;
      if (obc_on(d, 3)) {
        auto gr = [&](int ii, int jj) { return (V(ii, jj, nstp) - V(ii - 1, jj, nstp)) * pmask(ii, jj); };
        bool inflow;
        const double vb = orl_normal(V(i, je + 1, nstp), V(i, je, nstp), V(i, je, nnew), V(i, je - 1, nnew),
                                     gr(i, je + 1), gr(i + 1, je + 1), gr(i, je), gr(i + 1, je), inflow);
        const double bry = F.bv[3][i + (long)nbry(b, 3) * (k - 1)];
        double cext = 0.;
        if (inflow) {
          cext = bry < 0. ? -bry : d.p.ubind;
          cext = cext * dtfwd * 0.5 * (pn(i, je) + pn(i, je + 1));
        }
        if (F.ub[3]) cext = fmax(cext, fmin(F.ub[3][i], 1.0));   // SPONGE_TUNE ub_north (v3dbc_im.F:189-191)
        val = (1. - cext) * vb + cext * bry;
        val = val * F.vmask[IJ(b, i, je + 1)];
      }
      vn[IJKL(b, i, je + 1, k, nnew)] = val;
    }
  } else if (phase == 1) {
    for (int side = 0; side <= 1; side++) {
      const bool edge = side == 0 ? b.west_edge : b.east_edge;
      if (!edge) continue;
      const int ib = side == 0 ? is - 1 : ie + 1, ii = side == 0 ? is : ie;
      if (obc_on(d, side)) {
        const int j = b.jstrV + p;
        if (j > je) continue;
        auto gr = [&](int i, int jj) { return V(i, jj + 1, nstp) - V(i, jj, nstp); };
        double cx, cy;
        if (side == 0) {
          cx = -0.125 * dtfwd * (U(is, j, nrhs) + U(is, j - 1, nrhs)) * (pm(is - 1, j) + pm(is - 1, j - 1) + pm(is, j) + pm(is, j - 1));
          cy = 0.125 * dtfwd * (V(is - 1, j, nrhs) + V(is, j, nrhs)) * (pn(is - 1, j) + pn(is - 1, j - 1) + pn(is, j) + pn(is, j - 1));
        } else {
          cx = 0.125 * dtfwd * (U(ie + 1, j, nrhs) + U(ie + 1, j - 1, nrhs)) * (pm(ie + 1, j) + pm(ie + 1, j - 1) + pm(ie, j) + pm(ie, j - 1));
          cy = 0.125 * dtfwd * (V(ie, j, nrhs) + V(ie + 1, j, nrhs)) * (pn(ie + 1, j) + pn(ie + 1, j - 1) + pn(ie, j) + pn(ie, j - 1));
        }
        double cext;
        double val = orl_tangential(cx, cy, V(ib, j, nstp), V(ii, j, nstp), gr(ib, j - 1), gr(ib, j), gr(ii, j - 1),
                                    gr(ii, j), cext);
        if (F.ub[side]) cext = fmax(cext, fmin(F.ub[side][j], 1.0));   // ub_west/east (v3dbc_im.F:264-266,344-346)
        val = (1. - cext) * val + cext * F.bv[side][j + (long)nbry(b, side) * (k - 1)];
        vn[IJKL(b, ib, j, k, nnew)] = val * F.vmask[IJ(b, ib, j)];
      } else {
        const int j0 = b.ns_periodic ? b.jstrV : js, j1 = b.ns_periodic ? je : b.jendR;
        const int j = j0 + p;
        if (j > j1) continue;
        vn[IJKL(b, ib, j, k, nnew)] = d.p.gamma2 * v[IJKL(b, ii, j, k, nnew)] * F.vmask[IJ(b, ib, j)];
      }
    }
  } else if (p == 0) {
    const bool W = b.west_edge && obc_on(d, 0), E = b.east_edge && obc_on(d, 1);
    const bool S = b.south_edge && obc_on(d, 2), N = b.north_edge && obc_on(d, 3);
    auto Vn = [&](int i, int j) -> double& { return vn[IJKL(b, i, j, k, nnew)]; };
    if (S && W) Vn(is - 1, js) = 0.5 * (Vn(is - 1, js + 1) + Vn(is, js));
    if (S && E) Vn(ie + 1, js) = 0.5 * (Vn(ie + 1, js + 1) + Vn(ie, js));
    if (N && W) Vn(is - 1, je + 1) = 0.5 * (Vn(is - 1, je) + Vn(is, je + 1));
    if (N && E) Vn(ie + 1, je + 1) = 0.5 * (Vn(ie + 1, je) + Vn(ie, je + 1));
  }
}

// ---- t3dbc edges (phase 0; corners stay in k_t3dbc_corners) ----
__global__ void __launch_bounds__(256) k_t3dbc_obc(Dev d, int nnew, int nstp, int nrhs, double dtfwd, int itrc) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int p = blockIdx.x * blockDim.x + threadIdx.x, k = 1 + (int)blockIdx.y;
  const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
  double* t = F.t;
  auto T = [&](int i, int j, int l) { return t[TIDX(b, i, j, k, l, itrc)]; };
  auto U = [&](int i, int j) { return F.u[IJKL(b, i, j, k, nrhs)]; };
  auto V = [&](int i, int j) { return F.v[IJKL(b, i, j, k, nrhs)]; };
  auto rm = [&](int i, int j) { return F.rmask[IJ(b, i, j)]; };
  const int nj = je - js + 1, ni = ie - is + 1;
  const long nbk = (long)(k - 1) + (long)b.N * (itrc - 1);
  if (p < nj) {
    const int j = js + p;
    // western / eastern: gradients along j masked by vmask (t3dbc_im.F:40-48)
    auto gr = [&](int i, int jj) { return (T(i, jj, nstp) - T(i, jj - 1, nstp)) * F.vmask[IJ(b, i, jj)]; };
    if (b.west_edge) {
      double val;
      if (obc_on(d, 0)) {
        double cx = -dtfwd * U(is, j) * F.pm[IJ(b, is - 1, j)];
        const double cy = 0.5 * dtfwd * (V(is - 1, j) + V(is - 1, j + 1)) * F.pn[IJ(b, is - 1, j)];
        double cext;
        val = orl_tangential(cx, cy, T(is - 1, j, nstp), T(is, j, nstp), gr(is - 1, j), gr(is - 1, j + 1), gr(is, j),
                             gr(is, j + 1), cext);
        if (F.ub[0]) cext = fmax(cext, fmin(F.ub[0][j], 1.0));   // SPONGE_TUNE ub_west (t3dbc_im.F:73-74)
        val = (1. - cext) * val + cext * F.bt[0][j + (long)nbry(b, 0) * nbk];
        val = val * rm(is - 1, j);
      } else {
        val = T(is, j, nnew) * rm(is - 1, j);
      }
      t[TIDX(b, is - 1, j, k, nnew, itrc)] = val;
    }
    if (b.east_edge) {
      double val;
      if (obc_on(d, 1)) {
        double cx = dtfwd * U(ie + 1, j) * F.pm[IJ(b, ie + 1, j)];
        const double cy = 0.5 * dtfwd * (V(ie + 1, j) + V(ie + 1, j + 1)) * F.pn[IJ(b, ie + 1, j)];
        double cext;
        // the interior term reads t(iend,nnew) (t3dbc_im.F:133)
        val = orl_tangential(cx, cy, T(ie + 1, j, nstp), T(ie, j, nnew), gr(ie + 1, j), gr(ie + 1, j + 1), gr(ie, j),
                             gr(ie, j + 1), cext);
        if (F.ub[1]) cext = fmax(cext, fmin(F.ub[1][j], 1.0));   // SPONGE_TUNE ub_east (t3dbc_im.F:73-74)
        val = (1. - cext) * val + cext * F.bt[1][j + (long)nbry(b, 1) * nbk];
        val = val * rm(ie + 1, j);
      } else {
        val = T(ie, j, nnew) * rm(ie + 1, j);
      }
      t[TIDX(b, ie + 1, j, k, nnew, itrc)] = val;
    }
  } else if (p < nj + ni) {
    const int i = is + (p - nj);
    auto gr = [&](int ii, int jj) { return (T(ii, jj, nstp) - T(ii - 1, jj, nstp)) * F.umask[IJ(b, ii, jj)]; };
    if (b.south_edge) {
      double val;
      if (obc_on(d, 2)) {
        double cx = -dtfwd * V(i, js) * F.pn[IJ(b, i, js - 1)];
        const double cy = 0.5 * dtfwd * (U(i, js - 1) + U(i + 1, js - 1)) * F.pm[IJ(b, i, js - 1)];
        double cext;
        val = orl_tangential(cx, cy, T(i, js - 1, nstp), T(i, js, nstp), gr(i, js - 1), gr(i + 1, js - 1), gr(i, js),
                             gr(i + 1, js), cext);
        if (F.ub[2]) cext = fmax(cext, fmin(F.ub[2][i], 1.0));   // SPONGE_TUNE ub_south (t3dbc_im.F:73-74)
        val = (1. - cext) * val + cext * F.bt[2][i + (long)nbry(b, 2) * nbk];
        val = val * rm(i, js - 1);
      } else {
        val = T(i, js, nnew) * rm(i, js - 1);
      }
      t[TIDX(b, i, js - 1, k, nnew, itrc)] = val;
    }
    if (b.north_edge) {
      double val;
      if (obc_on(d, 3)) {
        double cx = dtfwd * V(i, je + 1) * F.pn[IJ(b, i, je + 1)];
        const double cy = 0.5 * dtfwd * (U(i, je + 1) + U(i + 1, je + 1)) * F.pm[IJ(b, i, je + 1)];
        double cext;
        // the interior term reads t(jend,nnew) (t3dbc_im.F:276)
        val = orl_tangential(cx, cy, T(i, je + 1, nstp), T(i, je, nnew), gr(i, je + 1), gr(i + 1, je + 1), gr(i, je),
                             gr(i + 1, je), cext);
        if (F.ub[3]) cext = fmax(cext, fmin(F.ub[3][i], 1.0));   // SPONGE_TUNE ub_north (t3dbc_im.F:73-74)
        val = (1. - cext) * val + cext * F.bt[3][i + (long)nbry(b, 3) * nbk];
        val = val * rm(i, je + 1);
      } else {
        val = T(i, je, nnew) * rm(i, je + 1);
      }
      t[TIDX(b, i, je + 1, k, nnew, itrc)] = val;
    }
  }
}

static double dtfwd_of(const Dev& d, const Tlev& t) { return t.nnew == 3 ? 0.5 * d.p.dt : d.p.dt; }  // PRED_STAGE

void launch_u3dbc_obc(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  const int n = (b.Mm > b.Lm ? b.Mm : b.Lm) + 4;
  const double dtw = dtfwd_of(d, t);
  for (int ph = 0; ph < 3; ph++)
    hipLaunchKernelGGL(k_u3dbc_obc, dim3(ph == 2 ? 1 : (n + 255) / 256, b.N), dim3(ph == 2 ? 64 : 256), 0, s, d, t.nnew,
                       t.nstp, t.nrhs, dtw, ph);
}
void launch_v3dbc_obc(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  const int n = (b.Mm > b.Lm ? b.Mm : b.Lm) + 4;
  const double dtw = dtfwd_of(d, t);
  for (int ph = 0; ph < 3; ph++)
    hipLaunchKernelGGL(k_v3dbc_obc, dim3(ph == 2 ? 1 : (n + 255) / 256, b.N), dim3(ph == 2 ? 64 : 256), 0, s, d, t.nnew,
                       t.nstp, t.nrhs, dtw, ph);
}
void launch_t3dbc_obc_edges(const Dev& d, hipStream_t s, const Tlev& t, int itrc) {
  const Bounds& b = d.b;
  const int n = (b.jend - b.jstr + 1) + (b.iend - b.istr + 1);
  hipLaunchKernelGGL(k_t3dbc_obc, dim3((n + 255) / 256, b.N), dim3(256), 0, s, d, t.nnew, t.nstp, t.nrhs,
                     dtfwd_of(d, t), itrc);
}

}  // namespace roms
