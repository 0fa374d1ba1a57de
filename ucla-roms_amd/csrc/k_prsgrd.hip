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
  // Top-down walk with a rolling register window: z_r, rho1, qp1 (or rho) of
  // each level are loaded once; the elementary differences, harmonic
  // averages and P keep the reference's expressions (prsgrd.F:200-330).
  auto rhov = [&](double r1, double q1, double z) {  // in-situ density at a rho level
    if (split) {
      const double dpth = -z;
      return r1 + q1 * dpth * (1.0 - qp2 * dpth);
    }
    return r1;
  };
  auto eRof = [&](double ru, double rl, double qu, double ql, double zu, double zl) {  // levels l+1 (u), l
    if (split) {
      const double dpth = -0.5 * (zu + zl);
      return ru - rl + (qu - ql) * dpth * (1.0 - qp2 * dpth);
    }
    return ru - rl;
  };
  const double* __restrict__ R1 = split ? rho1 : rho;
  auto ldz = [&](int k) { return zr[(long)(k - 1) * n2]; };
  auto ldr = [&](int k) { return R1[(long)(k - 1) * n2]; };
  auto ldq = [&](int k) { return split ? qp1[(long)(k - 1) * n2] : 0.0; };
  const bool doP = i >= b.istrU - 1 && i <= b.iend;
  double zC = ldz(N), rC = ldr(N), qC = ldq(N);              // level k
  double zM = ldz(N - 1), rM = ldr(N - 1), qM = ldq(N - 1);  // level k-1
  double eZk = zC - zM, eRk = eRof(rC, rM, qC, qM, zC, zM);  // e(N) = e(N-1)
  double dZ1 = 0.0, dR1 = 0.0, P1 = 0.0;                     // values at k+1
  double z1 = 0.0, v1 = 0.0;                                 // z_r, in-situ rho at k+1
#pragma unroll 4
  for (int k = N; k >= 1; k--) {
    double eZm, eRm;
    if (k >= 2) { eZm = zC - zM; eRm = eRof(rC, rM, qC, qM, zC, zM); }
    else { eZm = eZk; eRm = eRk; }                           // e(0) = e(1)
    const double dZk = [&] { const double c = 2.0 * eZk * eZm; return c / (eZk + eZm); }();
    double dRk = harm(eRk, eRm);
    const long o = (long)(k - 1) * n2;
    const double v0 = rhov(rC, qC, zC);
    if (split) {
      const double dpth = -zC;
      dRk = dRk - qC * dZk * (1.0 - 2.0 * qp2 * dpth);
      rhos[o] = v0;
    }
    if (doP) {
      double Pk;
      if (k == N) {
        const double zw = F.z_w[ij + (long)N * n2];
        const double rNm = rhov(rM, qM, zM);
        Pk = g * zw + grho * (v0 + 0.5 * (v0 - rNm) * (zw - zC) / (zC - zM)) * (zw - zC);
      } else {
        Pk = P1 + HalfGRho * ((v1 + v0) * (z1 - zC) -
                              OneFifth * ((dR1 - dRk) * (z1 - zC - OneTwelfth * (dZ1 + dZk)) -
                                          (dZ1 - dZk) * (v1 - v0 - OneTwelfth * (dR1 + dRk))));
      }
      Pp[o] = Pk;
      P1 = Pk;
    }
    dZ1 = dZk; dR1 = dRk;
    eZk = eZm; eRk = eRm;
    z1 = zC; v1 = v0;
    zC = zM; rC = rM; qC = qM;
    if (k >= 3) { zM = ldz(k - 2); rM = ldr(k - 2); qM = ldq(k - 2); }
  }
}

// ---- per cell (i,j,k): XI and ETA components ru, rv.  The block evaluates
// the clamped elementary differences FC, rx at the u-points (v-points) of its
// tile row (column) plus one on each side, then their harmonic averages
// dZ, dR (with the SPLIT_EOS compressibility term), once each, in LDS. ----
constexpr int kPXW = kBX + 2, kPXN = kPXW * kBY;          // u-points m = i0-1 .. i0+64, tile rows
constexpr int kPYH = kBY + 2, kPYN = kBX * kPYH;          // v-points m = j0-1 .. j0+4, tile columns
__global__ void __launch_bounds__(256) k_prsgrd_uv(Dev d, Range R, int split, int imin, int imax, int jmin, int jmax) {
  const uint3 bI = xcd_tile();
  __shared__ double sFCx[kPXN], sRx[kPXN], sFCy[kPYN], sRy[kPYN];
  __shared__ double sdZx[kPXN], sdRx[kPXN], sdZy[kPYN], sdRy[kPYN];
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double HalfGRho = 0.5 * (g / rho0);
  const double* rho = split ? F.rhos : F.rho;
  const int k = 1 + (int)bI.z;
  const long kk = (long)(k - 1) * b.n2, sj = b.nx2;
  const int i0 = R.i0 + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  // elementary differences at clamped u-points (xi) and v-points (eta)
  for (int q = tid; q < kPXN + kPYN; q += kBX * kBY) {
    if (q < kPXN) {
      const int j = j0 + q / kPXW;
      int m = i0 - 1 + q % kPXW;
      if (j > b.Mm + 1 || m > b.Lm + 2) { sFCx[q] = sRx[q] = 0.0; continue; }
      m = iclamp(m, imin, imax);
      const long om = IJ(b, m, j) + kk;
      const double um = F.umask[IJ(b, m, j)];
      sFCx[q] = (F.z_r[om] - F.z_r[om - 1]) * um;
      if (split) {
        const double dpth = -0.5 * (F.z_r[om] + F.z_r[om - 1]);
        sRx[q] = (F.rho1[om] - F.rho1[om - 1] + (F.qp1[om] - F.qp1[om - 1]) * dpth * (1.0 - qp2 * dpth)) * um;
      } else {
        sRx[q] = (F.rho[om] - F.rho[om - 1]) * um;
      }
    } else {
      const int qq = q - kPXN;
      const int i = i0 + qq % kBX;
      int m = j0 - 1 + qq / kBX;
      if (i > b.Lm + 1 || m > b.Mm + 2) { sFCy[qq] = sRy[qq] = 0.0; continue; }
      m = iclamp(m, jmin, jmax);
      const long om = IJ(b, i, m) + kk;
      const double vm = F.vmask[IJ(b, i, m)];
      sFCy[qq] = (F.z_r[om] - F.z_r[om - sj]) * vm;
      if (split) {
        const double dpth = -0.5 * (F.z_r[om] + F.z_r[om - sj]);
        sRy[qq] = (F.rho1[om] - F.rho1[om - sj] + (F.qp1[om] - F.qp1[om - sj]) * dpth * (1.0 - qp2 * dpth)) * vm;
      } else {
        sRy[qq] = (F.rho[om] - F.rho[om - sj]) * vm;
      }
    }
  }
  __syncthreads();
  // harmonic averages at rho points p = i-1, i (xi) and j-1, j (eta)
  for (int q = tid; q < kPXN + kPYN; q += kBX * kBY) {
    if (q < kPXN) {
      const int li = q % kPXW;
      if (li == kPXW - 1) continue;
      const int j = j0 + q / kPXW, p = i0 - 1 + li;
      double dz = harm(sFCx[q], sFCx[q + 1]), dr = harm(sRx[q], sRx[q + 1]);
      if (split && j <= b.Mm + 1 && p <= b.Lm + 1) {
        const long om = IJ(b, p, j) + kk;
        dr = dr - F.qp1[om] * dz * (1.0 + 2.0 * qp2 * F.z_r[om]);
      }
      sdZx[q] = dz;
      sdRx[q] = dr;
    } else {
      const int qq = q - kPXN;
      const int lj = qq / kBX;
      if (lj == kPYH - 1) continue;
      const int i = i0 + qq % kBX, p = j0 - 1 + lj;
      double dz = harm(sFCy[qq], sFCy[qq + kBX]), dr = harm(sRy[qq], sRy[qq + kBX]);
      if (split && i <= b.Lm + 1 && p <= b.Mm + 1) {
        const long om = IJ(b, i, p) + kk;
        dr = dr - F.qp1[om] * dz * (1.0 + 2.0 * qp2 * F.z_r[om]);
      }
      sdZy[qq] = dz;
      sdRy[qq] = dr;
    }
  }
  __syncthreads();
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  if (i > R.i1 || j > R.j1) return;
  const long ij = IJ(b, i, j), o = ij + kk;
  if (i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend) {
    const int q = threadIdx.x + threadIdx.y * kPXW;   // p = i-1 ; q+1: p = i
    const double dZ0 = sdZx[q], dZ1 = sdZx[q + 1], dR0 = sdRx[q], dR1 = sdRx[q + 1];
    F.ru[o] = 0.5 * (F.Hz[o] + F.Hz[o - 1]) * F.dn_u[ij] *
              (F.P[o - 1] - F.P[o] -
               HalfGRho * ((rho[o] + rho[o - 1]) * (F.z_r[o] - F.z_r[o - 1]) -
                           OneFifth * ((dR1 - dR0) * (F.z_r[o] - F.z_r[o - 1] - OneTwelfth * (dZ1 + dZ0)) -
                                       (dZ1 - dZ0) * (rho[o] - rho[o - 1] - OneTwelfth * (dR1 + dR0)))));
  }
  if (i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend) {
    const int q = threadIdx.x + threadIdx.y * kBX;    // p = j-1 ; q+kBX: p = j
    const double dZ0 = sdZy[q], dZ1 = sdZy[q + kBX], dR0 = sdRy[q], dR1 = sdRy[q + kBX];
    F.rv[o] = 0.5 * (F.Hz[o] + F.Hz[o - sj]) * F.dm_v[ij] *
              (F.P[o - sj] - F.P[o] -
               HalfGRho * ((rho[o] + rho[o - sj]) * (F.z_r[o] - F.z_r[o - sj]) -
                           OneFifth * ((dR1 - dR0) * (F.z_r[o] - F.z_r[o - sj] - OneTwelfth * (dZ1 + dZ0)) -
                                       (dZ1 - dZ0) * (rho[o] - rho[o - sj] - OneTwelfth * (dR1 + dR0)))));
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
