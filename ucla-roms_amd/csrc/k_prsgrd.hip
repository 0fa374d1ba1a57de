// k_prsgrd.hip -- prsgrd_tile (prsgrd.F:25-510): Shchepetkin-McWilliams (2003)
// density-Jacobian pressure gradient with harmonic-mean cubic fits.
//
// Kernel 1 (per column over 0..nx x 0..ny): elementary vertical differences,
// harmonic averages dR,dZ and the top-down hydrostatic pressure P, all in
// registers (rolling window over k) -- no (N+1)-deep scratch.  For SPLIT_EOS it
// also materialises the in-situ density rho = rho1 + qp1*dpth*(1-qp2*dpth).
// Kernel 2 (per column): XI and ETA components ru, rv; each lane rebuilds the
// three u-point (v-point) elementary differences it needs, with the
// reference's one-sided extrapolation at closed edges expressed as a clamp.
#include "roms_dev.h"

namespace roms {

__device__ __forceinline__ double harm(double a, double b) {
  const double c = 2.0 * a * b;
  return c > 0.0 ? c / (a + b) : 0.0;
}

__global__ void __launch_bounds__(256) k_prsgrd_P(Dev d, Range R, int split) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double grho = g / rho0, HalfGRho = 0.5 * grho;
  const long ij = IJ(b, i, j), n2 = b.n2;
  const double* __restrict__ zr = F.z_r + ij;
  const double* __restrict__ rho = F.rho + ij;
  const double* __restrict__ rho1 = F.rho1 + ij;
  const double* __restrict__ qp1 = F.qp1 + ij;
  double* __restrict__ rhos = F.rhos + ij;
  double* __restrict__ Pp = F.P + ij;
  // in-situ density at rho-level k (SPLIT_EOS: rho1 + qp1*dpth*(1-qp2*dpth))
  auto rhoval = [&](long o) {
    if (split) {
      const double dpth = -zr[o];
      return rho1[o] + qp1[o] * dpth * (1.0 - qp2 * dpth);
    }
    return rho[o];
  };
  // elementary difference at w-level k in 1..N-1
  auto eZ = [&](int k) { const long o = (long)(k - 1) * n2; return zr[o + n2] - zr[o]; };
  auto eR = [&](int k) {
    const long o = (long)(k - 1) * n2;
    if (split) {
      const double dpth = -0.5 * (zr[o + n2] + zr[o]);
      return rho1[o + n2] - rho1[o] + (qp1[o + n2] - qp1[o]) * dpth * (1.0 - qp2 * dpth);
    }
    return rho[o + n2] - rho[o];
  };
  const bool doP = i >= b.istrU - 1 && i <= b.iend;
  // rolling: e(k), e(k-1) elementary; dZ/dR harmonic at k+1 (previous)
  double eZk = eZ(N - 1), eRk = eR(N - 1);   // e(N) = e(N-1)
  double dZ1 = 0.0, dR1 = 0.0, P1 = 0.0;       // values at k+1
#pragma unroll 8
  for (int k = N; k >= 1; k--) {
    const int km = k - 1;
    const double eZm = km >= 1 ? eZ(km) : eZ(1);   // e(0) = e(1)
    const double eRm = km >= 1 ? eR(km) : eR(1);
    const double dZk = [&] { const double c = 2.0 * eZk * eZm; return c / (eZk + eZm); }();
    double dRk = harm(eRk, eRm);
    const long o = (long)(k - 1) * n2;
    if (split) {
      const double dpth = -zr[o];
      dRk = dRk - qp1[o] * dZk * (1.0 - 2.0 * qp2 * dpth);
      rhos[o] = rhoval(o);
    }
    if (doP) {
      double Pk;
      if (k == N) {
        const double zw = F.z_w[ij + (long)N * n2], zr0 = zr[o], zrm = zr[o - n2];
        const double rN = rhoval(o), rNm = rhoval(o - n2);
        Pk = g * zw + grho * (rN + 0.5 * (rN - rNm) * (zw - zr0) / (zr0 - zrm)) * (zw - zr0);
      } else {
        const double zr1 = zr[o + n2], zr0 = zr[o];
        const double r1 = rhoval(o + n2), r0 = rhoval(o);
        Pk = P1 + HalfGRho * ((r1 + r0) * (zr1 - zr0) -
                              OneFifth * ((dR1 - dRk) * (zr1 - zr0 - OneTwelfth * (dZ1 + dZk)) -
                                          (dZ1 - dZk) * (r1 - r0 - OneTwelfth * (dR1 + dRk))));
      }
      Pp[o] = Pk;
      P1 = Pk;
    }
    dZ1 = dZk; dR1 = dRk;
    eZk = eZm; eRk = eRm;
  }
}

__global__ void __launch_bounds__(256) k_prsgrd_uv(Dev d, Range R, int split, int imin, int imax, int jmin, int jmax) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double HalfGRho = 0.5 * (g / rho0);
  const double* rho = split ? F.rhos : F.rho;
  const bool du = i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend;
  const bool dv = i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend;
  const long ij = IJ(b, i, j);
  {
    const int k = 1 + (int)blockIdx.z;
    const long kk = (long)(k - 1) * b.n2;
    if (du) {
      // FC(m), rx(m) at u-points m=i-1,i,i+1 (clamped = edge extrapolation)
      double FC[3], rx[3];
      for (int q = 0; q < 3; q++) {
        const int m = iclamp(i - 1 + q, imin, imax);
        const long om = IJ(b, m, j) + kk;
        const double um = F.umask[IJ(b, m, j)];
        FC[q] = (F.z_r[om] - F.z_r[om - 1]) * um;
        if (split) {
          const double dpth = -0.5 * (F.z_r[om] + F.z_r[om - 1]);
          rx[q] = (F.rho1[om] - F.rho1[om - 1] + (F.qp1[om] - F.qp1[om - 1]) * dpth * (1.0 - qp2 * dpth)) * um;
        } else {
          rx[q] = (F.rho[om] - F.rho[om - 1]) * um;
        }
      }
      double dZx[2], dRx[2];  // at i-1, i
      for (int q = 0; q < 2; q++) {
        dZx[q] = harm(FC[q], FC[q + 1]);
        dRx[q] = harm(rx[q], rx[q + 1]);
        if (split) {
          const long om = ij - 1 + q + kk;
          dRx[q] = dRx[q] - F.qp1[om] * dZx[q] * (1.0 + 2.0 * qp2 * F.z_r[om]);
        }
      }
      const long o = ij + kk;
      F.ru[o] = 0.5 * (F.Hz[o] + F.Hz[o - 1]) * F.dn_u[ij] *
                (F.P[o - 1] - F.P[o] -
                 HalfGRho * ((rho[o] + rho[o - 1]) * (F.z_r[o] - F.z_r[o - 1]) -
                             OneFifth * ((dRx[1] - dRx[0]) * (F.z_r[o] - F.z_r[o - 1] - OneTwelfth * (dZx[1] + dZx[0])) -
                                         (dZx[1] - dZx[0]) * (rho[o] - rho[o - 1] - OneTwelfth * (dRx[1] + dRx[0])))));
    }
    if (dv) {
      const long sj = b.nx2;
      double FC[3], rx[3];
      for (int q = 0; q < 3; q++) {
        const int m = iclamp(j - 1 + q, jmin, jmax);
        const long om = IJ(b, i, m) + kk;
        const double vm = F.vmask[IJ(b, i, m)];
        FC[q] = (F.z_r[om] - F.z_r[om - sj]) * vm;
        if (split) {
          const double dpth = -0.5 * (F.z_r[om] + F.z_r[om - sj]);
          rx[q] = (F.rho1[om] - F.rho1[om - sj] + (F.qp1[om] - F.qp1[om - sj]) * dpth * (1.0 - qp2 * dpth)) * vm;
        } else {
          rx[q] = (F.rho[om] - F.rho[om - sj]) * vm;
        }
      }
      double dZx[2], dRx[2];
      for (int q = 0; q < 2; q++) {
        dZx[q] = harm(FC[q], FC[q + 1]);
        dRx[q] = harm(rx[q], rx[q + 1]);
        if (split) {
          const long om = ij + (long)(q - 1) * sj + kk;
          dRx[q] = dRx[q] - F.qp1[om] * dZx[q] * (1.0 + 2.0 * qp2 * F.z_r[om]);
        }
      }
      const long o = ij + kk;
      F.rv[o] = 0.5 * (F.Hz[o] + F.Hz[o - sj]) * F.dm_v[ij] *
                (F.P[o - sj] - F.P[o] -
                 HalfGRho * ((rho[o] + rho[o - sj]) * (F.z_r[o] - F.z_r[o - sj]) -
                             OneFifth * ((dRx[1] - dRx[0]) * (F.z_r[o] - F.z_r[o - sj] - OneTwelfth * (dZx[1] + dZx[0])) -
                                         (dZx[1] - dZx[0]) * (rho[o] - rho[o - sj] - OneTwelfth * (dRx[1] + dRx[0])))));
    }
  }
}

void launch_prsgrd(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  const int split = d.p.nonlin_eos;
  int imin, imax, jmin, jmax;
  if (!b.ew_periodic) {
    imin = b.west_edge ? b.istrU : b.istrU - 1;
    imax = b.east_edge ? b.iend : b.iend + 1;
  } else { imin = b.istr - 1; imax = b.iend + 1; }
  if (!b.ns_periodic) {
    jmin = b.south_edge ? b.jstrV : b.jstrV - 1;
    jmax = b.north_edge ? b.jend : b.jend + 1;
  } else { jmin = b.jstr - 1; jmax = b.jend + 1; }
  Range R1{0, b.Lm, 0, b.Mm};
  hipLaunchKernelGGL(k_prsgrd_P, grid_of(R1), dim3(kBX, kBY), 0, s, d, R1, split);
  Range R2{b.istr, b.iend, b.jstr, b.jend};
  hipLaunchKernelGGL(k_prsgrd_uv, grid3_of(R2, b.N), dim3(kBX, kBY), 0, s, d, R2, split, imin, imax, jmin, jmax);
}

}  // namespace roms
