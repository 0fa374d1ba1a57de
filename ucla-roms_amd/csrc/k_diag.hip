// k_diag.hip -- per-column terms of diag_tile (diag.F:58-405): barotropic
// velocities ub,vb, kinetic energy, barotropic KE, free-surface volume and the
// advective/vertical Courant numbers.  The reduction-by-pairs and the
// first-maximum scan (diag.F loop order j, k=N..1, i) finish on the host.
#include "roms_dev.h"

namespace roms {

__device__ __forceinline__ double diag_ub(const Dev& d, int i, int j, int nstp) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  double ub = (F.Hz[ij + (N - 1) * n2] + F.Hz[ij - 1 + (N - 1) * n2]) * U[ij + (N - 1) * n2];
  for (int k = N - 1; k >= 2; k--) ub = ub + (F.Hz[ij + (k - 1) * n2] + F.Hz[ij - 1 + (k - 1) * n2]) * U[ij + (k - 1) * n2];
  return (ub + (F.Hz[ij] + F.Hz[ij - 1]) * U[ij]) /
         (F.z_w[ij + N * n2] + F.z_w[ij - 1 + N * n2] - F.z_w[ij] - F.z_w[ij - 1]);
}
__device__ __forceinline__ double diag_vb(const Dev& d, int i, int j, int nstp) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  double vb = (F.Hz[ij + (N - 1) * n2] + F.Hz[ij - sj + (N - 1) * n2]) * V[ij + (N - 1) * n2];
  for (int k = N - 1; k >= 2; k--) vb = vb + (F.Hz[ij + (k - 1) * n2] + F.Hz[ij - sj + (k - 1) * n2]) * V[ij + (k - 1) * n2];
  return (vb + (F.Hz[ij] + F.Hz[ij - sj]) * V[ij]) /
         (F.z_w[ij + N * n2] + F.z_w[ij - sj + N * n2] - F.z_w[ij] - F.z_w[ij - sj]);
}

__global__ void __launch_bounds__(256) k_diag(Dev d, Range R, int nstp) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const long ij = IJ(b, i, j), n2 = b.n2, sj = b.nx2;
  const double ub0 = diag_ub(d, i, j, nstp), ub1 = diag_ub(d, i + 1, j, nstp);
  const double vb0 = diag_vb(d, i, j, nstp), vb1 = diag_vb(d, i, j + 1, nstp);
  const double v2b = 0.5 * (ub0 * ub0 + ub1 * ub1 + vb0 * vb0 + vb1 * vb1);
  double ke = 0.0;
  double ke2b = 0.5 * (F.z_w[ij + N * n2] - F.z_w[ij]) * v2b;
  double cxm = 0.0, cwm = 0.0, km = -1.0;
  const double* U = F.u + (long)(nstp - 1) * b.n3;
  const double* V = F.v + (long)(nstp - 1) * b.n3;
  for (int k = N; k >= 1; k--) {
    const long o = ij + (long)(k - 1) * n2, w = ij + (long)k * n2;
    const double u0 = U[o], u1 = U[o + 1], v0 = V[o], v1 = V[o + sj];
    const double v2 = 0.5 * (u0 * u0 + u1 * u1 + v0 * v0 + v1 * v1);
    const double ciV = d.p.dt * F.rmask[ij] * F.pm[ij] * F.pn[ij] / F.Hz[o];
    const double cw = ciV * (fmax0(F.We[w] + F.Wi[w]) - fmin0(F.We[w - n2] + F.Wi[w - n2]));
    const double cx = cw + ciV * (fmax0(F.FlxU[o + 1]) - fmin0(F.FlxU[o]) + fmax0(F.FlxV[o + sj]) - fmin0(F.FlxV[o]));
    if (cx > cxm) { cxm = cx; cwm = cw; km = (double)k; }
    ke = ke + 0.5 * v2 * F.Hz[o];
  }
  const double dA = F.rmask[ij] / (F.pm[ij] * F.pn[ij]);
  F.s0[ij] = dA * F.z_w[ij + N * n2];
  F.s1[ij] = dA * ke;
  F.s2[ij] = dA * ke2b;
  F.s3[ij] = cxm;
  F.s4[ij] = cwm;
  F.s5[ij] = km;
}

void launch_diag(const Dev& d, hipStream_t s, const Tlev& t, double* partials) {
  (void)partials;
  const Bounds& b = d.b;
  (void)hipMemsetAsync(d.f.s0, 0, (size_t)b.n2 * sizeof(double), s);
  (void)hipMemsetAsync(d.f.s1, 0, (size_t)b.n2 * sizeof(double), s);
  (void)hipMemsetAsync(d.f.s2, 0, (size_t)b.n2 * sizeof(double), s);
  Range R{1, b.Lm, 1, b.Mm};
  hipLaunchKernelGGL(k_diag, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nstp);
}

}  // namespace roms
