// k_river.hip -- river sources (river_frc.F) in the hot path.
//
// calc_river_flux (river_frc.F:224-282) marks every face between a
// river-mouth cell and a wet neighbour with riv_flx = 10*iriver + the signed
// fraction of that river's volume flux through the face.  The hot path uses
// the faces in four places:
//   step2d_FB.F:531-554     ubar/vbar(knew) = river flux / (dn * mean depth),
//                           DU/DV_avg1 = river flux, after every fast step;
//   pre_step3d4S.F:493-522  u,v(nnew) = river velocity over the column;
//   step3d_uv2.F:689-717    the same after the corrector;
//   compute_horiz_tracer_fluxes.h:217-246
//                           the tracer flux through the face carries the
//                           river's tracer concentration (k_common.h,
//                           river_tracer_flux, inside the tracer kernels).
// The faces are few (a river mouth spans a handful of cells), so the first
// three run over the compact face list built by roms_gpu_set_river_frc, one
// thread per face, on the same stream and in the same place of the step as
// the reference's loops.
#include "k_common.h"

namespace roms {

// ---- step2d: after the fast step's momentum update and boundary fluxes ----
__global__ void __launch_bounds__(64) k_river_s2d(Dev d, int knew) {
  const int f = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= d.p.nrivf) return;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int dir = F.riv_face[3 * f], i = F.riv_face[3 * f + 1], j = F.riv_face[3 * f + 2];
  const long ij = IJ(b, i, j), kn = (long)(knew - 1) * b.n2;
  if (dir == 0) {
    if (!(j >= b.jstr && j <= b.jend && i >= b.istrU && i <= b.iend)) return;
    const double flx = F.riv_uflx[ij];
    const int iriver = (int)lround(flx / 10);
    const double river_flux = F.riv_vol[iriver - 1] * (flx - 10 * iriver);
    const double Dm = F.zeta[ij - 1 + kn] + F.h[ij - 1], D0 = F.zeta[ij + kn] + F.h[ij];   // Dnew(i-1), Dnew(i)
    F.ubar[ij + kn] = river_flux * 2 / (F.dn_u[ij] * (Dm + D0));
    F.DU_avg1[ij] = river_flux;
  } else {
    if (!(j >= b.jstrV && j <= b.jend && i >= b.istr && i <= b.iend)) return;
    const double flx = F.riv_vflx[ij];
    const int iriver = (int)lround(flx / 10);
    const double river_flux = F.riv_vol[iriver - 1] * (flx - 10 * iriver);
    const double Dm = F.zeta[ij - b.nx2 + kn] + F.h[ij - b.nx2], D0 = F.zeta[ij + kn] + F.h[ij];
    F.vbar[ij + kn] = river_flux * 2 / (F.dm_v[ij] * (Dm + D0));
    F.DV_avg1[ij] = river_flux;
  }
}

// ---- u,v(nnew) = river velocity over the whole column (pre_step3d: u at
// istrU.., v at jstrV..; step3d_uv2: istr.., jstr..) ----
__global__ void __launch_bounds__(64) k_river_uv(Dev d, int nnew, int pred) {
  const int f = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= d.p.nrivf) return;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const int dir = F.riv_face[3 * f], i = F.riv_face[3 * f + 1], j = F.riv_face[3 * f + 2];
  const long ij = IJ(b, i, j), n2 = b.n2;
  double vel;
  double* U;
  if (dir == 0) {
    if (!(j >= b.jstr && j <= b.jend && i >= (pred ? b.istrU : b.istr) && i <= b.iend)) return;
    vel = river_velocity(d, 0, ij, true);
    U = F.u + (long)(nnew - 1) * b.n3 + ij;
  } else {
    if (!(j >= (pred ? b.jstrV : b.jstr) && j <= b.jend && i >= b.istr && i <= b.iend)) return;
    vel = river_velocity(d, 1, ij, true);
    U = F.v + (long)(nnew - 1) * b.n3 + ij;
  }
  for (int k = 1; k <= N; k++) U[(long)(k - 1) * n2] = vel;
}

void launch_river_s2d(const Dev& d, hipStream_t s, int knew) {
  if (d.p.nriv <= 0 || d.p.nrivf <= 0) return;
  hipLaunchKernelGGL(k_river_s2d, dim3((d.p.nrivf + 63) / 64), dim3(64), 0, s, d, knew);
}

void launch_river_uv(const Dev& d, hipStream_t s, int nnew, int pred) {
  if (d.p.nriv <= 0 || d.p.nrivf <= 0) return;
  hipLaunchKernelGGL(k_river_uv, dim3((d.p.nrivf + 63) / 64), dim3(64), 0, s, d, nnew, pred);
}

}  // namespace roms
