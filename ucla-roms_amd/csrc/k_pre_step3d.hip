// k_pre_step3d.hip -- pre_step3d_tile (pre_step3d4S.F:23-742): LF-AM3
// predictor for tracers and momentum to n+1/2, and the bottom-drag
// coefficient r_D (compute_rd_bott_drag.h).  Also hosts the horizontal
// momentum r.h.s. kernel shared with step3d_uv1 (UPSTREAM_UV flag).
#include "k_common.h"

namespace roms {

struct PreCoef {
  double dtau, cf_stp, cf_bak;
};

// ---- tracers: horizontal 4th-order fluxes, vertical spline advection and the
// implicit vertical diffusion with Wi up-winding, one lane per column. ----
__global__ void k_pre_tracer(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, indx = 3 - nstp;
  const long n2 = b.n2, ij = IJ(b, i, j);
  double* FCs = F.c0;  // spline interface values / fluxes
  double* CFs = F.c1;
  double* DCs = F.c2;
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    const double* Tr = F.t + (long)(nrhs - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    double* Tn = F.t + (long)(nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    double* Ti = F.t + (long)(indx - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    const double* Ts = F.t + (long)(nstp - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3;
    for (int k = 1; k <= N; k++) {
      double hb, hf;
      hz_bak_fwd(d, i, j, k, 0.5 * c.dtau, hb, hf);
      const double FX0 = tracer_fx(d, Tr, i, j, k, false), FX1 = tracer_fx(d, Tr, i + 1, j, k, false);
      const double FE0 = tracer_fe(d, Tr, i, j, k, false), FE1 = tracer_fe(d, Tr, i, j + 1, k, false);
      const long o = ij + (long)(k - 1) * n2;
      const double tsk = Ts[o];
      Tn[o] = hb * (c.cf_stp * tsk + c.cf_bak * Ti[o]) - c.dtau * F.pm[ij] * F.pn[ij] * (FX1 - FX0 + FE1 - FE0);
      Ti[o] = F.Hz[o] * tsk;
    }
    // vertical advective fluxes (spline on t(nrhs)) -> Tn
    tracer_spline_fc(d, Tr, ij, FCs, CFs);
    for (int k = 1; k <= N; k++) {
      const long o = ij + (long)(k - 1) * n2;
      Tn[o] = Tn[o] - c.dtau * F.pm[ij] * F.pn[ij] * (FCs[ij + (long)k * n2] - FCs[ij + (long)(k - 1) * n2]);
    }
    // implicit vertical diffusion (Thomas, top-down elimination written bottom-up)
    const int iAkt = itrc < b.nTS ? itrc : b.nTS;
    const double* Akt = F.Akt + (long)(iAkt - 1) * b.n3w;
    double hf1, hf2, dummy;
    hz_bak_fwd(d, i, j, 1, 0.5 * c.dtau, dummy, hf1);
    hz_bak_fwd(d, i, j, 2, 0.5 * c.dtau, dummy, hf2);
    const double DC0 = c.dtau * F.pm[ij] * F.pn[ij];
    double FCk = 2.0 * c.dtau * Akt[ij + n2] / (hf2 + hf1);
    double WCk = DC0 * F.Wi[ij + n2];
    double cff = 1.0 / (hf1 + FCk + fmax0(WCk));
    double CFk = cff * (FCk - fmin0(WCk));
    double DCk = cff * Tn[ij];
    CFs[ij + n2] = CFk;
    DCs[ij + n2] = DCk;
    double hfk = hf2;
    for (int k = 2; k <= N - 1; k++) {
      double hfk1;
      hz_bak_fwd(d, i, j, k + 1, 0.5 * c.dtau, dummy, hfk1);
      const double FCn = 2.0 * c.dtau * Akt[ij + (long)k * n2] / (hfk1 + hfk);
      const double WCn = DC0 * F.Wi[ij + (long)k * n2];
      cff = 1.0 / (hfk + FCn + fmax0(WCn) + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
      const double CFn = cff * (FCn - fmin0(WCn));
      const double DCn = cff * (Tn[ij + (long)(k - 1) * n2] + DCk * (FCk + fmax0(WCk)));
      CFs[ij + (long)k * n2] = CFn;
      DCs[ij + (long)k * n2] = DCn;
      FCk = FCn; WCk = WCn; CFk = CFn; DCk = DCn; hfk = hfk1;
    }
    // hfk is Hz_fwd(N) here (N>=3); for N==2 it is hf2
    const long oN = ij + (long)(N - 1) * n2;
    double tk = (Tn[oN] + DCk * (FCk + fmax0(WCk))) / (hfk + FCk - fmin0(WCk) - CFk * (FCk + fmax0(WCk)));
    Tn[oN] = tk;
    for (int k = N - 1; k >= 1; k--) {
      const long o = ij + (long)(k - 1) * n2;
      tk = DCs[ij + (long)k * n2] + CFs[ij + (long)k * n2] * tk;
      Tn[o] = tk;
    }
  }
}

// ---- horizontal momentum r.h.s. for all levels (pre_step3d / step3d_uv1) ----
__global__ void k_uv_horiz(Dev d, Range R, int nrhs, UVBounds ub, int up) {
  ROMS_IJ_OR_RETURN(R)
  for (int k = 1; k <= d.b.N; k++) uv_horiz_rhs(d, i, j, k, nrhs, ub, up != 0);
}

void launch_uv_horiz(const Dev& d, hipStream_t s, int nrhs, int up) {
  const Bounds& b = d.b;
  Range R{b.istr, b.iend, b.jstr, b.jend};
  hipLaunchKernelGGL(k_uv_horiz, grid_of(R), dim3(kBX, kBY), 0, s, d, R, nrhs, uv_bounds(b), up);
}

// ---- bottom drag r_D (compute_rd_bott_drag.h), log-layer with Zob ----
__global__ void k_rd(Dev d, Range R, int nstp) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j);
  if (d.p.Zob > 0.0) {
    const double* U = F.u + (long)(nstp - 1) * b.n3;
    const double* V = F.v + (long)(nstp - 1) * b.n3;
    const double u0 = U[ij], u1 = U[ij + 1], v0 = V[ij], v1 = V[ij + b.nx2];
    const double cff = sqrt(0.333333333333 * (u0 * u0 + u1 * u1 + u0 * u1 + v0 * v0 + v1 * v1 + v0 * v1));
    const double q = d.p.vonKar / log(1.0 + 0.5 * F.Hz[ij] / d.p.Zob);
    F.r_D[ij] = cff * (q * q);
  } else {
    double rd = d.p.rdrg;
    F.r_D[ij] = dmin(rd, 0.8 * F.Hz[ij] / d.p.dt);
  }
}

// ---- momentum: vertical spline advection into ru/rv, then implicit
// viscosity with implicit no-slip bottom (IMPLCT_NO_SLIP_BTTM_BC) ----
__device__ void pre_uv_solve(const Dev& d, int i, int j, int dir, const PreCoef& c, int nstp, int nnew) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N, indx = 3 - nstp;
  const long n2 = b.n2, ij = IJ(b, i, j);
  const long s = dir == 0 ? 1 : b.nx2;
  double* Uall = dir == 0 ? F.u : F.v;
  const double* rr = dir == 0 ? F.ru : F.rv;
  const double* Ustp = Uall + (long)(nstp - 1) * b.n3;
  double* Uidx = Uall + (long)(indx - 1) * b.n3;
  double* Unew = Uall + (long)(nnew - 1) * b.n3;
  const double sstr = dir == 0 ? F.sustr[ij] : F.svstr[ij];
  double* CFs = F.c1;
  double* DCs = F.c2;
  const double hcf = 0.5 * c.dtau;
  auto hf = [&](int ii, int jj, int k) { double bb, ff; hz_bak_fwd(d, ii, jj, k, hcf, bb, ff); return ff; };
  auto hb = [&](int ii, int jj, int k) { double bb, ff; hz_bak_fwd(d, ii, jj, k, hcf, bb, ff); return bb; };
  const int im = dir == 0 ? i - 1 : i, jm = dir == 0 ? j : j - 1;
  const double DC0 = c.dtau * 0.25 * (F.pm[ij] + F.pm[ij - s]) * (F.pn[ij] + F.pn[ij - s]);
  // initial DC(k) (computed on the fly) and u(indx) = Hz*u(nstp)
  auto DCinit = [&](int k) {
    const long o = ij + (long)(k - 1) * n2;
    const double r = 0.5 * (hb(i, j, k) + hb(im, jm, k)) * (c.cf_stp * Ustp[o] + c.cf_bak * Uidx[o]) + DC0 * rr[o];
    Uidx[o] = 0.5 * (F.Hz[o] + F.Hz[o - s]) * Ustp[o];
    return r;
  };
  const double* Akv = F.Akv;
  double hfN = hf(i, j, N), hfNm = hf(im, jm, N);
  double hfK = hf(i, j, N - 1), hfKm = hf(im, jm, N - 1);
  double FCk = 2.0 * c.dtau * (Akv[ij + (long)(N - 1) * n2] + Akv[ij - s + (long)(N - 1) * n2]) / (hfN + hfNm + hfK + hfKm);
  double WCk = DC0 * 0.5 * (F.Wi[ij + (long)(N - 1) * n2] + F.Wi[ij - s + (long)(N - 1) * n2]);
  double cff = 1.0 / (0.5 * (hfN + hfNm) + FCk - fmin0(WCk));
  double CFk = cff * (FCk + fmax0(WCk));   // CF(N-1)
  double DCk1 = cff * (DCinit(N) + c.dtau * sstr);  // DC(N)
  DCs[ij + (long)N * n2] = DCk1;
  CFs[ij + (long)(N - 1) * n2] = CFk;
  // level k quantities: FCk=FC(k), WCk=WC(k), CFk=CF(k); hfK/hfKm = Hz_fwd(k)
  for (int k = N - 1; k >= 2; k--) {
    const double hfL = hf(i, j, k - 1), hfLm = hf(im, jm, k - 1);
    const double FCl = 2.0 * c.dtau * (Akv[ij + (long)(k - 1) * n2] + Akv[ij - s + (long)(k - 1) * n2]) / (hfK + hfKm + hfL + hfLm);
    const double WCl = DC0 * 0.5 * (F.Wi[ij + (long)(k - 1) * n2] + F.Wi[ij - s + (long)(k - 1) * n2]);
    cff = 1.0 / (0.5 * (hfK + hfKm) + FCl - fmin0(WCl) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
    const double CFl = cff * (FCl + fmax0(WCl));
    const double DCk = cff * (DCinit(k) + DCk1 * (FCk - fmin0(WCk)));
    CFs[ij + (long)(k - 1) * n2] = CFl;
    DCs[ij + (long)k * n2] = DCk;
    DCk1 = DCk; FCk = FCl; WCk = WCl; CFk = CFl; hfK = hfL; hfKm = hfLm;
  }
  // bottom: FCk=FC(1), WCk=WC(1), CFk=CF(1), DCk1=DC(2); hfK=Hz_fwd(1)
  const double rd = F.r_D[ij], rdm = F.r_D[ij - s];
  double un = (DCinit(1) + DCk1 * (FCk - fmin0(WCk))) /
              (0.5 * (hfK + hfKm) + 0.5 * c.dtau * (rd + rdm) + FCk + fmax0(WCk) - CFk * (FCk - fmin0(WCk)));
  Unew[ij] = un;
  for (int k = 2; k <= N; k++) {
    un = DCs[ij + (long)k * n2] + CFs[ij + (long)(k - 1) * n2] * un;
    Unew[ij + (long)(k - 1) * n2] = un;
  }
}

__global__ void k_pre_uv(Dev d, Range R, PreCoef c, int nstp, int nnew, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  if (i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend) {
    uv_vert_rhs(d, i, j, nrhs, 0, d.f.c0, d.f.c1);
    pre_uv_solve(d, i, j, 0, c, nstp, nnew);
  }
  if (i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend) {
    uv_vert_rhs(d, i, j, nrhs, 1, d.f.c0, d.f.c1);
    pre_uv_solve(d, i, j, 1, c, nstp, nnew);
  }
}

void launch_pre_step3d(const Dev& d, hipStream_t s, const Tlev& t) {
  const Bounds& b = d.b;
  PreCoef c;
  const double AM3_crv = 1.0 / 6.0;
  if (t.iic == t.forw_start) { c.dtau = 0.5 * d.p.dt; c.cf_stp = 1.0; c.cf_bak = 0.0; }
  else { c.dtau = d.p.dt * (1.0 - AM3_crv); c.cf_stp = 0.5 + AM3_crv; c.cf_bak = 0.5 - AM3_crv; }
  Range RI{b.istr, b.iend, b.jstr, b.jend};
  hipLaunchKernelGGL(k_pre_tracer, grid_of(RI), dim3(kBX, kBY), 0, s, d, RI, c, t.nstp, t.nnew, t.nrhs);
  launch_uv_horiz(d, s, t.nrhs, 0);
  Range Rd{b.istrU - 1, b.iend, b.jstrV - 1, b.jend};
  hipLaunchKernelGGL(k_rd, grid_of(Rd), dim3(kBX, kBY), 0, s, d, Rd, t.nstp);
  hipLaunchKernelGGL(k_pre_uv, grid_of(RI), dim3(kBX, kBY), 0, s, d, RI, c, t.nstp, t.nnew, t.nrhs);
  launch_u3dbc(d, s, t);
  launch_v3dbc(d, s, t);
  for (int itrc = 1; itrc <= b.NT; itrc++) {
    launch_t3dbc(d, s, t, itrc);
    launch_exchange(d, s, d.f.t + (long)(t.nnew - 1) * b.n3 + (long)(itrc - 1) * 3 * b.n3, b.N);
  }
}

}  // namespace roms
