// k_step3d_t.hip -- tracer corrector step3d_t_iso_tile (step3d_t_ISO.F:45-1178,
// non-isoneutral branch: UPSTREAM_TS + SPLINE_TS) and the Laplacian tracer
// diffusion t3dmix_tile (t3dmix_S.F).  One lane per water column; all levels
// and the tridiagonal solve stay in the lane.
#include "k_common.h"

namespace roms {

__global__ void k_step3d_t(Dev d, Range R, int nnew, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const int N = b.N;
  const double dt = P.dt;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const double rm = F.rmask[ij];
  double* FCs = F.c0;
  double* CFs = F.c1;
  double* DCs = F.c2;
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    const double* Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    double* Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    const double stf = F.stflx[ij + (long)(itrc - 1) * n2];
    for (int k = 1; k <= N; k++) {
      const double FX0 = tracer_fx(d, Tr, i, j, k, true), FX1 = tracer_fx(d, Tr, i + 1, j, k, true);
      const double FE0 = tracer_fe(d, Tr, i, j, k, true), FE1 = tracer_fe(d, Tr, i, j + 1, k, true);
      const long o = ij + (long)(k - 1) * n2;
      Tn[o] = Tn[o] - dt * F.pm[ij] * F.pn[ij] * (FX1 - FX0 + FE1 - FE0);
    }
    tracer_spline_fc(d, Tr, ij, FCs, CFs);
    for (int k = 1; k <= N; k++) {
      const long o = ij + (long)(k - 1) * n2;
      Tn[o] = Tn[o] - dt * F.pm[ij] * F.pn[ij] * (FCs[ij + (long)k * n2] - FCs[ij + (long)(k - 1) * n2]);
    }
    const long oN = ij + (long)(N - 1) * n2;
    if (itrc == 1) Tn[oN] = Tn[oN] + dt * F.swflx[ij] * Tn[oN] / F.Hz[oN];
    Tn[oN] = Tn[oN] + dt * stf;
    if (P.lmd) {
      if (itrc == 1) {
        const double sr = F.srflx[ij];
        for (int k = N - 1; k >= 1; k--) {
          const long w = ij + (long)k * n2, o = ij + (long)(k - 1) * n2;
          const double cff = sr * F.swr_frac[w] - F.ghat[w] * (stf - sr);
          Tn[o + n2] = Tn[o + n2] - dt * cff;
          Tn[o] = Tn[o] + dt * cff;
        }
      } else if (itrc == 2 && P.salinity) {
        for (int k = N - 1; k >= 1; k--) {
          const long w = ij + (long)k * n2, o = ij + (long)(k - 1) * n2;
          const double cff = -dt * F.ghat[w] * stf;
          Tn[o + n2] = Tn[o + n2] - cff;
          Tn[o] = Tn[o] + cff;
        }
      }
    }
    const int iAkt = itrc < b.nTS ? itrc : b.nTS;
    const double* Akt = F.Akt + (long)(iAkt - 1) * b.n3w;
    const double DC0 = dt * F.pm[ij] * F.pn[ij];
    double FCk = 2.0 * dt * Akt[ij + n2] / (F.Hz[ij] + F.Hz[ij + n2]);
    double WCk = DC0 * F.Wi[ij + n2];
    double cff = 1.0 / (F.Hz[ij] + FCk + fmax0(WCk));
    double CFk = cff * (FCk - fmin0(WCk));
    double DCk = cff * Tn[ij];
    CFs[ij + n2] = CFk;
    DCs[ij + n2] = DCk;
    for (int k = 2; k <= N - 1; k++) {
      const long o = ij + (long)(k - 1) * n2;
      const double FCn = 2.0 * dt * Akt[ij + (long)k * n2] / (F.Hz[o] + F.Hz[o + n2]);
      const double WCn = F.Wi[ij + (long)k * n2] * DC0;
      cff = 1.0 / (F.Hz[o] + FCn + fmax0(WCn) + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
      const double CFn = cff * (FCn - fmin0(WCn));
      const double DCn = cff * (Tn[o] + DCk * (FCk + fmax0(WCk)));
      CFs[ij + (long)k * n2] = CFn;
      DCs[ij + (long)k * n2] = DCn;
      FCk = FCn; WCk = WCn; CFk = CFn; DCk = DCn;
    }
    double tk = (Tn[oN] + DCk * (FCk + fmax0(WCk))) / (F.Hz[oN] + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk))) * rm;
    Tn[oN] = tk;
    for (int k = N - 1; k >= 1; k--) {
      tk = (DCs[ij + (long)k * n2] + CFs[ij + (long)k * n2] * tk) * rm;
      Tn[ij + (long)(k - 1) * n2] = tk;
    }
  }
}

void launch_step3d_t(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  hipLaunchKernelGGL(k_step3d_t, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nnew, t.nrhs);
  for (int itrc = 1; itrc <= b.NT; itrc++) launch_t3dbc(d, s, t, itrc);
  for (int itrc = 1; itrc <= b.NT; itrc++)
    launch_exchange(d, s, d.f.t + (long)(t.nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3, b.N);
}

// ---- t3dmix: Laplacian diffusion along S, t(nnew) += dt*pm*pn*div(F)/Hz ----
__global__ void k_t3dmix(Dev d, Range R, int nnew, int nrhs, int itrc) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), sj = b.nx2, n2 = b.n2;
  const double* d2 = F.diff2 + (long)(itrc - 1) * n2;
  const double* Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
  double* Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
  auto FX = [&](long p, long kk) {
    return 0.25 * (d2[p] + d2[p - 1]) * F.pmon_u[p] * (F.Hz[p + kk] + F.Hz[p - 1 + kk]) * (Tr[p + kk] - Tr[p - 1 + kk]) *
           F.umask[p];
  };
  auto FE = [&](long p, long kk) {
    return 0.25 * (d2[p] + d2[p - sj]) * F.pnom_v[p] * (F.Hz[p + kk] + F.Hz[p - sj + kk]) *
           (Tr[p + kk] - Tr[p - sj + kk]) * F.vmask[p];
  };
  for (int k = 1; k <= b.N; k++) {
    const long kk = (long)(k - 1) * n2, o = ij + kk;
    Tn[o] = Tn[o] + d.p.dt * F.pm[ij] * F.pn[ij] * (FX(ij + 1, kk) - FX(ij, kk) + FE(ij + sj, kk) - FE(ij, kk)) / F.Hz[o];
  }
}

void launch_t3dmix(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    hipLaunchKernelGGL(k_t3dmix, grid_of(R), dim3(kBX, kBY), 0, s, d, R, t.nnew, t.nrhs, itrc);
    launch_exchange(d, s, d.f.t + (long)(t.nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3, b.N);
  }
}

}  // namespace roms
