// host_init.cpp -- host-side model setup for the analytic cases: the parts
// of roms_init (main.F:85-321) that the reference runs once on the CPU before
// time stepping -- set_weights (set_weights.F:7-235), set_scoord
// (set_scoord.F:4-66), ana_grid / ana_init (tests/Filament/ana_grid.h,
// ana_init.h; synthetic basin of SURVEY.md 8(d)), setup_grid1 metrics and the
// setup_grid2 area/volume sums.  Produces host arrays in the Fortran layout
// that the shim uploads; the time-stepping itself never touches the host.
#include "host_init.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace roms {

HostState::HostState(int Lm_, int Mm_, int N_, int NT_, int nTS_)
    : Lm(Lm_), Mm(Mm_), N(N_), NT(NT_), nTS(nTS_), nx2(Lm_ + 4), n2((long)(Lm_ + 4) * (Mm_ + 4)) {}

std::vector<double>& HostState::a(int id) { return arr[id]; }

// ---- set_weights (p=2, q=4, r=0.25) ----
int set_weights(int ndtfast, double w[2][kMaxFast]) {
  for (int i = 0; i < kMaxFast; i++) { w[0][i] = 0.0; w[1][i] = 0.0; }
  int nfast = 0;
  const double p = 2.0, q = 4.0, r = 0.25;
  double scale = (p + 1.0) * (p + q + 1.0) / ((p + 2.0) * (p + q + 2.0) * (double)ndtfast);
  double sum, shft, cff;
  for (int iter = 1; iter <= 16; iter++) {
    nfast = 0;
    for (int i = 1; i <= 2 * ndtfast; i++) {
      cff = scale * (double)i;
      w[0][i - 1] = std::pow(cff, p) - std::pow(cff, p + q) - r * cff;
      if (w[0][i - 1] > 0.0) nfast = i;
      if (nfast > 0 && w[0][i - 1] < 0.0) w[0][i - 1] = 0.0;
    }
    sum = 0.0; shft = 0.0;
    for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; shft = shft + w[0][i - 1] * (double)i; }
    scale = scale * shft / (sum * (double)ndtfast);
  }
  for (int iter = 1; iter <= ndtfast; iter++) {
    sum = 0.0; shft = 0.0;
    for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; shft = shft + (double)i * w[0][i - 1]; }
    shft = shft / sum;
    cff = (double)ndtfast - shft;
    if (cff > 1.0) {
      nfast = nfast + 1;
      for (int i = nfast; i >= 2; i--) w[0][i - 1] = w[0][i - 2];
      w[0][0] = 0.0;
    } else if (cff > 0.0) {
      sum = 1.0 - cff;
      for (int i = nfast; i >= 2; i--) w[0][i - 1] = sum * w[0][i - 1] + cff * w[0][i - 2];
      w[0][0] = sum * w[0][0];
    } else if (cff < -1.0) {
      nfast = nfast - 1;
      for (int i = 1; i <= nfast; i++) w[0][i - 1] = w[0][i];
      w[0][nfast] = 0.0;
    } else if (cff < 0.0) {
      sum = 1.0 + cff;
      for (int i = 1; i <= nfast - 1; i++) w[0][i - 1] = sum * w[0][i - 1] - cff * w[0][i];
      w[0][nfast - 1] = sum * w[0][nfast - 1];
    }
  }
  for (int j = 1; j <= nfast; j++) {
    cff = w[0][j - 1];
    for (int i = 1; i <= j; i++) w[1][i - 1] = w[1][i - 1] + cff;
  }
  sum = 0.0; cff = 0.0;
  for (int i = 1; i <= nfast; i++) { sum = sum + w[0][i - 1]; cff = cff + w[1][i - 1]; }
  sum = 1.0 / sum; cff = 1.0 / cff;
  for (int i = 1; i <= nfast; i++) { w[0][i - 1] = sum * w[0][i - 1]; w[1][i - 1] = cff * w[1][i - 1]; }
  return nfast;
}

// ---- set_scoord: SM09 stretching ----
static double CSF(double sc, double theta_s, double theta_b) {
  double csrf;
  if (theta_s > 0.0) csrf = (1.0 - std::cosh(theta_s * sc)) / (std::cosh(theta_s) - 1.0);
  else csrf = -(sc * sc);
  if (theta_b > 0.0) return (std::exp(theta_b * csrf) - 1.0) / (1.0 - std::exp(-theta_b));
  return csrf;
}
void set_scoord(int N, double theta_s, double theta_b, double* Cs_w, double* Cs_r) {
  const double ds = 1.0 / (double)N;
  Cs_w[N] = 0.0;
  for (int k = N - 1; k >= 1; k--) Cs_w[k] = CSF(ds * (double)(k - N), theta_s, theta_b);
  Cs_w[0] = -1.0;
  Cs_r[0] = 0.0;
  for (int k = 1; k <= N; k++) Cs_r[k] = CSF(ds * ((double)(k - N) - 0.5), theta_s, theta_b);
}

// periodic halo wrap on the host (same semantics as the device exchange)
static void wrap(const HostState& H, double* a, int nlev, bool ewp, bool nsp) {
  if (!H.wrap_on) return;
  const int Lm = H.Lm, Mm = H.Mm;
  auto at = [&](int i, int j, int k) -> double& { return a[(i + 1) + (long)(j + 1) * H.nx2 + (long)k * H.n2]; };
  for (int k = 0; k < nlev; k++) {
    if (ewp)
      for (int j = 0; j <= Mm + 1; j++) {
        at(-1, j, k) = at(Lm - 1, j, k); at(0, j, k) = at(Lm, j, k);
        at(Lm + 1, j, k) = at(1, j, k); at(Lm + 2, j, k) = at(2, j, k);
      }
    if (nsp)
      for (int i = 0; i <= Lm + 1; i++) {
        int is = i;
        if (ewp) { if (i == 0) is = Lm; if (i == Lm + 1) is = 1; }
        at(i, -1, k) = at(is, Mm - 1, k); at(i, 0, k) = at(is, Mm, k);
        at(i, Mm + 1, k) = at(is, 1, k); at(i, Mm + 2, k) = at(is, 2, k);
      }
    if (ewp && nsp)
      for (int dj = 0; dj < 2; dj++)
        for (int di = 0; di < 2; di++) {
          at(-1 + di, -1 + dj, k) = at(Lm - 1 + di, Mm - 1 + dj, k);
          at(Lm + 1 + di, -1 + dj, k) = at(1 + di, Mm - 1 + dj, k);
          at(-1 + di, Mm + 1 + dj, k) = at(Lm - 1 + di, 1 + dj, k);
          at(Lm + 1 + di, Mm + 1 + dj, k) = at(1 + di, 1 + dj, k);
        }
  }
}

static double pair_reduce(const HostState& H, std::vector<double> A, int istr, int iend, int jstr, int jend) {
  auto at = [&](int i, int j) -> double& { return A[(i + 1) + (long)(j + 1) * H.nx2]; };
  int isize = iend - istr, jsize = jend - jstr;
  while (isize > 0 || jsize > 0) {
    if (jsize > 0) {
      int js = (jsize + 1) / 2 - 1;
      for (int j = 0; j <= js; j++) {
        const int jtg = jstr + j;
        for (int i = istr; i <= istr + isize; i++) at(i, jtg) = at(i, jtg + j) + at(i, jtg + j + 1);
      }
      if (2 * js + 1 < jsize) {
        js = js + 1;
        const int jtg = jstr + js;
        for (int i = istr; i <= istr + isize; i++) at(i, jtg) = at(i, jtg + js);
      }
      jsize = js;
    }
    if (isize > 0) {
      int is = (isize + 1) / 2 - 1;
      for (int j = jstr; j <= jstr + jsize; j++)
        for (int i = 0; i <= is; i++) {
          const int itg = istr + i;
          at(itg, j) = at(itg + i, j) + at(itg + i + 1, j);
        }
      if (2 * is + 1 < isize) {
        is = is + 1;
        const int itg = istr + is;
        for (int j = jstr; j <= jstr + jsize; j++) at(itg, j) = at(itg + is, j);
      }
      isize = is;
    }
  }
  return at(istr, jstr);
}
double pair_sum(const HostState& H, const std::vector<double>& A) { return pair_reduce(H, A, 1, H.Lm, 1, H.Mm); }

// Build grid + initial state of an analytic case on the host.
void build_case(const CaseSpec& cs, HostState& H, double& area, double& volume) {
  const int Lm = H.Lm, Mm = H.Mm, N = H.N, NT = H.NT;
  const long n2 = H.n2, n3 = n2 * N, n3w = n2 * (N + 1);
  const bool ewp = cs.ew_periodic, nsp = cs.ns_periodic;
  auto alloc = [&](int id, long n) { H.arr[id].assign(n, 0.0); };
  for (int id : {kh, khinv, kf, kfomn, kpm, kpn, kdm_r, kdn_r, kdm_u, kdn_u, kdm_v, kdn_v, kdm_p, kdn_p, kpmon_u, kpnom_v,
                 krmask, kpmask, kumask, kvmask, kxr, kyr, kvisc2_r, kvisc2_p, ksustr, ksvstr, ksrflx, kswflx})
    alloc(id, n2);
  alloc(kzeta, 4 * n2); alloc(kubar, 4 * n2); alloc(kvbar, 4 * n2);
  alloc(ku, 3 * n3); alloc(kv, 3 * n3); alloc(kt, 3 * n3 * NT);
  alloc(kAkv, n3w); alloc(kAkt, n3w * H.nTS); alloc(kdiff2, n2 * NT); alloc(kstflx, n2 * NT);
  alloc(kz_r, n3); alloc(kz_w, n3w); alloc(kHz, n3);
  alloc(kCs_w, N + 1); alloc(kCs_r, N + 1);
  set_scoord(N, cs.theta_s, cs.theta_b, H.arr[kCs_w].data(), H.arr[kCs_r].data());
  auto A = [&](int id, int i, int j) -> double& { return H.arr[id][(i + 1) + (long)(j + 1) * H.nx2]; };
  auto A3 = [&](int id, int i, int j, int k) -> double& { return H.arr[id][(i + 1) + (long)(j + 1) * H.nx2 + (long)(k - 1) * n2]; };
  auto W3 = [&](int id, int i, int j, int k) -> double& { return H.arr[id][(i + 1) + (long)(j + 1) * H.nx2 + (long)k * n2]; };
  auto T = [&](int i, int j, int k, int l, int it) -> double& {
    return H.arr[kt][(i + 1) + (long)(j + 1) * H.nx2 + (long)(k - 1) * n2 + (long)(l - 1) * n3 + (long)(it - 1) * 3 * n3];
  };
  H.wrap_on = cs.host_wrap != 0;
  // ---- ana_grid ----
  if (cs.case_id == 0) {
    const double SizeX = cs.sizex, SizeY = cs.sizey;
    const double f0 = 2 * 7.81e-5, beta = 0;
    const double dx = SizeX / cs.LLm, dy = SizeY / cs.MMm, x_mid = SizeX / 2.0;
    const double x0 = dx * (double)cs.iSW_corn, y0 = dy * (double)cs.jSW_corn;
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) {
        A(kxr, i, j) = x0 + dx * ((double)i - 0.5) - x_mid;
        A(kyr, i, j) = y0 + dy * ((double)j - 0.5);
        A(kpm, i, j) = 1.0 / dx;
        A(kpn, i, j) = 1.0 / dy;
        A(kf, i, j) = f0 + beta * (A(kyr, i, j) - SizeY / 2.0);
        A(kh, i, j) = 1000;
        A(krmask, i, j) = 1;
      }
  } else if (cs.case_id == ROMS_CASE_PIPES) {
    // tests/Pipes_ana/ana_grid.h:19-131: shelf + slope, land strip with a river gap, one pipe
    const double SizeX = cs.sizex, SizeY = cs.sizey, f0 = 1.0e-4, beta = 0;
    const double dx = SizeX / cs.LLm, dy = SizeY / cs.MMm;
    const double x0 = dx * (double)cs.iSW_corn, y0 = dy * (double)cs.jSW_corn;
    const double depth = 10, max_depth = 100, shelf = SizeY / 5, slope = (max_depth - depth) / (SizeY * 4 / 5);
    const double land = SizeY * 0.1, coast = SizeY * 0.02, riv_west = SizeX * 0.4, riv_east = SizeX * 0.6;
    const double psz = SizeX * 0.02, px = SizeX * .5, py = SizeY * .5;
    const long pc = std::lround(psz / dx);
    const double pipe_cells = (double)(pc * pc);
    H.npip = 1;
    H.pipe_idx.assign(n2, 0);
    H.pipe_flx.assign(n2, 0.0);
    H.pipe_prf.assign((size_t)N, 0.0);
    H.pipe_prf[0] = 0.5; H.pipe_prf[1] = 0.5;             // ana_pipe_frc.h: pipe_prf(1,1:2)
    H.pipe_trc.assign((size_t)NT, 0.0);
    H.pipe_trc[0] = 24.0; if (NT > 1) H.pipe_trc[1] = 1.0;  // pipe_trc(1,1:2)
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) {
        const double x = x0 + dx * ((double)i - 0.5), y = y0 + dy * ((double)j - 0.5);
        A(kxr, i, j) = x; A(kyr, i, j) = y;
        A(kpm, i, j) = 1. / dx; A(kpn, i, j) = 1. / dy;
        A(kf, i, j) = f0 + beta * (y - SizeY / 2.);
        A(kh, i, j) = y < shelf ? depth : depth + (y - shelf) * slope;
        double rm = 1;
        if (y < land && (x < riv_west || x > riv_east)) rm = 0.0;
        if (y < coast) rm = 0.0;
        A(krmask, i, j) = rm;
        if (x > px - 0.5 * psz && x < px + 0.5 * psz && y > py - 0.5 * psz && y < py + 0.5 * psz) {
          const long o = (i + 1) + (long)(j + 1) * H.nx2;
          H.pipe_idx[o] = 1;
          H.pipe_flx[o] = 1.0 / pipe_cells * 5e2;  // pipe_fraction * pipe_vol(1)
        }
      }
  } else if (cs.case_id == ROMS_CASE_RIVERS) {
    // tests/Rivers_ana/ana_grid.h:1-101: 10 km shelf (5..100 m), f = 0, land
    // strip with the river channel; the reference fills 0..nx+1, 0..ny+1 of
    // each rank (the outer halo ring keeps the allocation values: 0, rmask 1)
    const double Size_XI = 1.0e4, Size_ETA = 1.0e4, depth = 5., max_depth = 100.0, f0 = 0.0e-4, beta = 0.;
    const double xl = Size_XI, el = Size_ETA;
    const double dx = Size_XI / (double)cs.LLm, dy = Size_ETA / (double)cs.MMm;
    const double x0 = dx * (double)cs.iSW_corn, y0 = dy * (double)cs.jSW_corn;
    const double shelf = Size_ETA / 5, slope = (max_depth - depth) / (Size_ETA * 4 / 5);
    const double land = el * 0.1, coast = el * 0.02, riv_west = xl * 0.4, riv_east = xl * 0.6;
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) A(krmask, i, j) = 1;
    for (int j = 0; j <= Mm + 1; j++)
      for (int i = 0; i <= Lm + 1; i++) {
        const double x = x0 + dx * ((double)i - 0.5), y = y0 + dy * ((double)j - 0.5);
        A(kxr, i, j) = x; A(kyr, i, j) = y;
        A(kpm, i, j) = 1. / dx; A(kpn, i, j) = 1. / dy;
        A(kf, i, j) = f0 + beta * (y - Size_ETA / 2.);
        A(kh, i, j) = y < shelf ? depth : depth + (y - shelf) * slope;
        double rm = 1;
        if (y < land && (x < riv_west || x > riv_east)) rm = 0.0;
        if (y < coast) rm = 0.0;
        A(krmask, i, j) = rm;
      }
    // river_frc.F init_river_frc (analytical, :118-135) and calc_river_flux
    // (:228-282) over this rank's 0..nx+1, 0..ny+1; ana_frc_river.h:
    // riv_vol(1) = 5e2 m3/s, riv_trc(1,1:2) = (24, 1)
    H.nriv = 1;
    H.riv_uflx.assign(n2, 0.0);
    H.riv_vflx.assign(n2, 0.0);
    H.riv_vol.assign(1, 5e2);
    H.riv_trc.assign((size_t)NT, 0.0);
    H.riv_trc[0] = 24.0; if (NT > 1) H.riv_trc[1] = 1.0;
    const double riv_cells = (double)std::lround((riv_east - riv_west) * A(kpm, 1, 1));
    auto RU = [&](int i, int j) -> double& { return H.riv_uflx[(i + 1) + (long)(j + 1) * H.nx2]; };
    auto RV = [&](int i, int j) -> double& { return H.riv_vflx[(i + 1) + (long)(j + 1) * H.nx2]; };
    for (int j = 0; j <= Mm + 1; j++)
      for (int i = 0; i <= Lm + 1; i++) {
        if (!(A(kxr, i, j) > riv_west && A(kxr, i, j) < riv_east)) continue;
        if (!(A(krmask, i, j) == 0 && A(krmask, i, j + 1) == 1)) continue;
        const double rfrc = 1 / riv_cells;
        const int ridx = 1;
        const int faces = (int)(A(krmask, i - 1, j) + A(krmask, i + 1, j) + A(krmask, i, j - 1) + A(krmask, i, j + 1));
        if (A(krmask, i - 1, j) > 0) RU(i, j) = -(rfrc) / faces + 10 * ridx;
        if (A(krmask, i + 1, j) > 0) RU(i + 1, j) = (rfrc) / faces + 10 * ridx;
        if (A(krmask, i, j - 1) > 0) RV(i, j) = -(rfrc) / faces + 10 * ridx;
        if (A(krmask, i, j + 1) > 0) RV(i, j + 1) = (rfrc) / faces + 10 * ridx;
      }
  } else {
    const double dx = cs.sizex / cs.LLm, dy = cs.sizey / cs.MMm;
    const double R = 0.5 * (cs.sizex < cs.sizey ? cs.sizex : cs.sizey);
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) {
        const double x = dx * ((double)(i + cs.iSW_corn) - 0.5), y = dy * ((double)(j + cs.jSW_corn) - 0.5);
        A(kxr, i, j) = x; A(kyr, i, j) = y;
        A(kpm, i, j) = 1.0 / dx; A(kpn, i, j) = 1.0 / dy;
        if (cs.curvgrid) {  // non-uniform metrics (oracle_main.c or_ana_grid): m varies along eta, n along xi
          const double pi = 3.14159265358979323;
          A(kpm, i, j) = (1.0 + 0.1 * std::sin(2.0 * pi * ((double)(j + cs.jSW_corn) - 0.5) / (double)cs.MMm)) / dx;
          A(kpn, i, j) = (1.0 + 0.1 * std::cos(2.0 * pi * ((double)(i + cs.iSW_corn) - 0.5) / (double)cs.LLm)) / dy;
        }
        A(kf, i, j) = 1.0e-4;
        const double rx = x - 0.5 * cs.sizex, ry = y - 0.5 * cs.sizey;
        double s = 1.0 - (rx * rx + ry * ry) / (R * R);
        if (s < 0.0) s = 0.0;
        A(kh, i, j) = 200.0 + 3800.0 * s;
        A(krmask, i, j) = 1.0;
        if (cs.island) {  // circular island of radius 0.1 min(Lx,Ly) at (0.35 Lx, 0.6 Ly)
          const double ix = x - 0.35 * cs.sizex, iy = y - 0.6 * cs.sizey, ir = 0.2 * R;
          if (ix * ix + iy * iy < ir * ir) A(krmask, i, j) = 0.0;
        }
      }
  }
  // ---- setup_grid1 (setup_grid1.F): metric combinations and masks ----
  const int istr = 1, iend = Lm, jstr = 1, jend = Mm;
  const bool we = !ewp && !cs.west_exchng, ee = !ewp && !cs.east_exchng;
  const bool se = !nsp && !cs.south_exchng, ne = !nsp && !cs.north_exchng;
  const int istrR = we ? istr - 1 : istr, iendR = ee ? iend + 1 : iend;
  const int jstrR = se ? jstr - 1 : jstr, jendR = ne ? jend + 1 : jend;
  const int istrE = (ewp || cs.west_exchng) ? istr - 2 : istr - 1, iendE = (ewp || cs.east_exchng) ? iend + 2 : iend + 1;
  const int jstrE = (nsp || cs.south_exchng) ? jstr - 2 : jstr - 1, jendE = (nsp || cs.north_exchng) ? jend + 2 : jend + 1;
  for (int j = jstrE; j <= jendE; j++)
    for (int i = istrE; i <= iendE; i++) A(kfomn, i, j) = A(kf, i, j) / (A(kpm, i, j) * A(kpn, i, j));
  for (int j = jstrR; j <= jendR; j++)
    for (int i = istrR; i <= iendR; i++) { A(kdm_r, i, j) = 1.0 / A(kpm, i, j); A(kdn_r, i, j) = 1.0 / A(kpn, i, j); }
  for (int j = jstrR; j <= jendR; j++)
    for (int i = istr; i <= iendR; i++) {
      A(kpmon_u, i, j) = (A(kpm, i, j) + A(kpm, i - 1, j)) / (A(kpn, i, j) + A(kpn, i - 1, j));
      A(kdm_u, i, j) = 2.0 / (A(kpm, i, j) + A(kpm, i - 1, j));
      A(kdn_u, i, j) = 2.0 / (A(kpn, i, j) + A(kpn, i - 1, j));
      A(kumask, i, j) = A(krmask, i, j) * A(krmask, i - 1, j);
    }
  for (int j = jstr; j <= jendR; j++)
    for (int i = istrR; i <= iendR; i++) {
      A(kpnom_v, i, j) = (A(kpn, i, j) + A(kpn, i, j - 1)) / (A(kpm, i, j) + A(kpm, i, j - 1));
      A(kdm_v, i, j) = 2.0 / (A(kpm, i, j) + A(kpm, i, j - 1));
      A(kdn_v, i, j) = 2.0 / (A(kpn, i, j) + A(kpn, i, j - 1));
      A(kvmask, i, j) = A(krmask, i, j) * A(krmask, i, j - 1);
    }
  for (int j = jstr; j <= jendR; j++)
    for (int i = istr; i <= iendR; i++) {
      A(kdm_p, i, j) = 4.0 / (A(kpm, i, j) + A(kpm, i, j - 1) + A(kpm, i - 1, j) + A(kpm, i - 1, j - 1));
      A(kdn_p, i, j) = 4.0 / (A(kpn, i, j) + A(kpn, i, j - 1) + A(kpn, i - 1, j) + A(kpn, i - 1, j - 1));
      const int a = A(krmask, i - 1, j) > 0.5, b = A(krmask, i, j) > 0.5, c = A(krmask, i - 1, j - 1) > 0.5,
                d = A(krmask, i, j - 1) > 0.5;
      const int n = a + b + c + d;
      double pmk = 0.0;
      if (n >= 3) pmk = 1.0;
      else if (n == 2 && ((a && c) || (b && d) || (a && b) || (c && d))) pmk = 2.0;
      A(kpmask, i, j) = pmk;
    }
  alloc(kdndx, n2); alloc(kdmde, n2);
  if (cs.curvgrid) {  // setup_grid1.F:89-103 (exchanged below / by the device exchange)
    for (int j = jstrR; j <= jendR; j++)
      for (int i = istr; i <= iend; i++) A(kdndx, i, j) = 0.5 / A(kpn, i + 1, j) - 0.5 / A(kpn, i - 1, j);
    for (int j = jstr; j <= jend; j++)
      for (int i = istrR; i <= iendR; i++) A(kdmde, i, j) = 0.5 / A(kpm, i, j + 1) - 0.5 / A(kpm, i, j - 1);
  }
  for (int id : {kdm_r, kdn_r, kdm_p, kdn_p, kdm_u, kdn_u, kdm_v, kdn_v, kpmon_u, kpnom_v, krmask, kumask, kvmask, kpmask,
                 kdndx, kdmde})
    wrap(H, H.arr[id].data(), 1, ewp, nsp);
  // setup_grid2: area/volume (single-rank pairwise sums)
  {
    std::vector<double> dA(n2, 0.0), dV(n2, 0.0);
    for (int j = 1; j <= Mm; j++)
      for (int i = 1; i <= Lm; i++) {
        const long o = (i + 1) + (long)(j + 1) * H.nx2;
        dA[o] = A(krmask, i, j) / (A(kpm, i, j) * A(kpn, i, j));
        dV[o] = dA[o] * A(kh, i, j);
      }
    area = pair_sum(H, dA);
    volume = pair_sum(H, dV);
  }
  // mixing.F:156-162
  for (long q = 0; q < n2; q++) { H.arr[kvisc2_r][q] = cs.visc2; H.arr[kvisc2_p][q] = cs.visc2; }
  for (long q = 0; q < n2 * NT; q++) H.arr[kdiff2][q] = cs.tnu2;
  // set_nudgcof.F:42-111 sponge bands along open edges, on this rank's own
  // points only (the reference exchanges nothing afterwards, main.F:299)
  if (cs.obc) {
    const int isp = 15 + 1;
    std::vector<double> wrk(n2, 0.0);
    auto Wk = [&](int i, int j) -> double& { return wrk[(i + 1) + (long)(j + 1) * H.nx2]; };
    for (int j = std::max(-1, jstrR - 1); j <= jendR; j++)
      for (int i = std::max(-1, istrR - 1); i <= iendR; i++) {
        const int ig = i + cs.iSW_corn, jg = j + cs.jSW_corn;
        int ibnd = isp;
        if (cs.obc & 1) ibnd = std::min(ibnd, ig);
        if (cs.obc & 2) ibnd = std::min(ibnd, cs.LLm + 1 - ig);
        if (cs.obc & 4) ibnd = std::min(ibnd, jg);
        if (cs.obc & 8) ibnd = std::min(ibnd, cs.MMm + 1 - jg);
        Wk(i, j) = (double)(isp - ibnd) / (double)isp;
      }
    const double vs = cs.v_sponge;
    for (int j = jstrR; j <= jendR; j++)
      for (int i = istrR; i <= iendR; i++) A(kvisc2_r, i, j) = A(kvisc2_r, i, j) + vs * Wk(i, j);
    for (int j = jstr; j <= jendR; j++)
      for (int i = istr; i <= iendR; i++)
        A(kvisc2_p, i, j) = A(kvisc2_p, i, j) + 0.25 * vs * (Wk(i, j) + Wk(i - 1, j) + Wk(i, j - 1) + Wk(i - 1, j - 1));
    for (int it = 1; it <= NT; it++)
      for (int j = jstrR; j <= jendR; j++)
        for (int i = istrR; i <= iendR; i++) {
          double& d2 = H.arr[kdiff2][(i + 1) + (long)(j + 1) * H.nx2 + (long)(it - 1) * n2];
          d2 = d2 + vs * Wk(i, j);
        }
  }
  // ---- set_depth at rest (zeta=0) for ana_init: set_depth.F:65-90 ----
  const double hc = cs.hc, ds = 1.0 / (double)N;
  const double* Cs_w = H.arr[kCs_w].data();
  const double* Cs_r = H.arr[kCs_r].data();
  // istrR..iendR plus the halo the exchange fills (set_depth.F:72-90 and its
  // exchange): on a physical non-periodic edge the outer ghost stays zero
  for (int j = se ? jstrR : -1; j <= (ne ? jendR : Mm + 2); j++)
    for (int i = we ? istrR : -1; i <= (ee ? iendR : Lm + 2); i++) {
      const double hh = A(kh, i, j), hi = 1.0 / (hh + hc), z = 0.0;
      W3(kz_w, i, j, 0) = -hh;
      for (int k = 1; k <= N; k++) {
        const double cff_w = hc * ds * (double)(k - N), cff_r = hc * ds * ((double)(k - N) - 0.5);
        W3(kz_w, i, j, k) = z + (z + hh) * (cff_w + Cs_w[k] * hh) * hi;
        A3(kz_r, i, j, k) = z + (z + hh) * (cff_r + Cs_r[k] * hh) * hi;
        A3(kHz, i, j, k) = W3(kz_w, i, j, k) - W3(kz_w, i, j, k - 1);
      }
    }
  // ---- ana_init ----
  const double g = 9.81;
  if (cs.case_id == 0) {
    const double b0 = 5.0e-2, B_cff = 0.025, lambda_inv = 8.0, Nb = 1.0e-7, N0 = 3.0e-5, h0 = 60.0, dh0 = 15.,
                 L = 2000.0, HD = 1000;
    const double alpha = cs.Tcoef / cs.rho0;
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) {
        const double xl = A(kxr, i, j) / L;
        const double h_sbl = h0 + dh0 * std::exp(-(xl * xl));
        for (int k = 1; k <= N; k++) {
          const double zr = A3(kz_r, i, j, k);
          const double b = b0 + Nb * (zr + HD) +
                           0.5 * N0 * ((1 + B_cff) * zr - (1 - B_cff) * (h_sbl + lambda_inv * std::log(std::cosh((1. / lambda_inv) * (zr + h_sbl)))));
          T(i, j, k, 1, 1) = b / (g * alpha);
        }
      }
    double bf_int = 0;
    for (int k = 1; k <= N; k++) {
      const double zr = A3(kz_r, 1, 1, k);
      bf_int = bf_int + A3(kHz, 1, 1, k) *
                            (b0 + Nb * (zr + HD) +
                             0.5 * N0 * ((1 + B_cff) * zr - (1 - B_cff) * (h0 + lambda_inv * std::log(std::cosh((1. / lambda_inv) * (zr + h0)))))) /
                            g;
    }
    for (int k = 1; k <= N; k++)
      for (int j = -1; j <= Mm + 2; j++)
        for (int i = -1; i <= Lm + 2; i++) {
          T(i, j, k, 2, 1) = T(i, j, k, 1, 1);
          if (cs.salinity) { T(i, j, k, 1, 2) = 36.; T(i, j, k, 2, 2) = T(i, j, k, 1, 2); }
        }
    auto Z = [&](int i, int j, int l) -> double& { return H.arr[kzeta][(i + 1) + (long)(j + 1) * H.nx2 + (long)(l - 1) * n2]; };
    auto VB = [&](int i, int j, int l) -> double& { return H.arr[kvbar][(i + 1) + (long)(j + 1) * H.nx2 + (long)(l - 1) * n2]; };
    auto V = [&](int i, int j, int k, int l) -> double& {
      return H.arr[kv][(i + 1) + (long)(j + 1) * H.nx2 + (long)(k - 1) * n2 + (long)(l - 1) * n3];
    };
    for (int k = 1; k <= N; k++)
      for (int j = -1; j <= Mm + 2; j++)
        for (int i = -1; i <= Lm + 2; i++) Z(i, j, 1) = Z(i, j, 1) + T(i, j, k, 1, 1) * alpha * A3(kHz, i, j, k);
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) Z(i, j, 1) = (Z(i, j, 1) - bf_int);
    for (int j = 0; j <= Mm + 1; j++)
      for (int i = 0; i <= Lm + 1; i++) {
        const double dzdx = 0.5 * A(kpm, i, j) * (Z(i + 1, j, 1) - Z(i - 1, j, 1));
        V(i, j, N, 1) = g * dzdx / A(kf, i, j);
      }
    for (int k = N - 1; k >= 1; k--)
      for (int j = 0; j <= Mm + 1; j++)
        for (int i = 0; i <= Lm + 1; i++) {
          const double dbdx = 0.25 * A(kpm, i, j) * g * alpha *
                              (T(i + 1, j, k, 1, 1) - T(i - 1, j, k, 1, 1) + T(i + 1, j, k + 1, 1, 1) - T(i - 1, j, k + 1, 1, 1));
          V(i, j, k, 1) = V(i, j, k + 1, 1) - dbdx * (A3(kz_r, i, j, k + 1) - A3(kz_r, i, j, k)) / A(kf, i, j);
        }
    for (int k = N - 1; k >= 1; k--)
      for (int j = 0; j <= Mm + 1; j++)
        for (int i = 0; i <= Lm + 1; i++) VB(i, j, 1) = VB(i, j, 1) + V(i, j, k, 1) * A3(kHz, i, j, k) / HD;
    for (int j = 1; j <= Mm; j++)
      for (int i = 1; i <= Lm; i++) {
        VB(i, j, 2) = VB(i, j, 1);
        Z(i, j, 2) = Z(i, j, 1);
        for (int k = 1; k <= N; k++) V(i, j, k, 2) = V(i, j, k, 1);
      }
  } else if (cs.case_id == ROMS_CASE_PIPES || cs.case_id == ROMS_CASE_RIVERS) {
    // tests/Pipes_ana/ana_init.h:14-52, tests/Rivers_ana/ana_init.h:10-40:
    // at rest, T = 4 + 10 e^{z/50}, S = 36 (LMD: Akv = Akt = 0)
    for (int k = 1; k <= N; k++)
      for (int j = 0; j <= Mm + 1; j++)
        for (int i = 0; i <= Lm + 1; i++) {
          T(i, j, k, 1, 1) = 4. + 10. * std::exp(A3(kz_r, i, j, k) / 50.);
          T(i, j, k, 2, 1) = T(i, j, k, 1, 1);
          if (cs.salinity) { T(i, j, k, 1, 2) = 36.; T(i, j, k, 2, 2) = T(i, j, k, 1, 2); }
        }
  } else {
    const double Lx = cs.sizex, Ly = cs.sizey, pi = 3.14159265358979323;
    for (int k = 1; k <= N; k++)
      for (int j = -1; j <= Mm + 2; j++)
        for (int i = -1; i <= Lm + 2; i++) {
          const double x = A(kxr, i, j), y = A(kyr, i, j), ez = std::exp(A3(kz_r, i, j, k) / 500.0);
          T(i, j, k, 1, 1) = 4.0 + 10.0 * ez + 0.5 * std::sin(2.0 * pi * x / Lx) * std::sin(2.0 * pi * y / Ly) * ez;
          T(i, j, k, 2, 1) = T(i, j, k, 1, 1);
          if (cs.salinity) {
            T(i, j, k, 1, 2) = 35.0 + 0.25 * std::cos(2.0 * pi * x / Lx);
            T(i, j, k, 2, 2) = T(i, j, k, 1, 2);
          }
          for (int it = 3; it <= NT; it++) {
            const double rx = (x - 0.3 * Lx) / (0.1 * Lx), ry = (y - 0.5 * Ly) / (0.1 * Ly);
            T(i, j, k, 1, it) = std::exp(-(rx * rx + ry * ry)) * ez * (double)(it - 2);
            T(i, j, k, 2, it) = T(i, j, k, 1, it);
          }
        }
    if (!cs.lmd) {  // mixing.F:163-181: LMD_MIXING starts from Akv = Akt = 0
      for (long q = 0; q < n3w; q++) H.arr[kAkv][q] = cs.Akv_bak;
      for (int it = 1; it <= H.nTS; it++)
        for (long q = 0; q < n3w; q++) H.arr[kAkt][q + (long)(it - 1) * n3w] = cs.Akt_bak[it - 1];
    }
    const double piy = 3.14159265358979323;
    if (cs.bulk_frc) {  // analytic atmosphere for BULK_FRC (oracle_main.c or_ana_forces); the
                        // device computes the fluxes (k_bulk.hip) at init and in every step
      for (int id : {kuwnd, kvwnd, ktair, kqair, kprate, kswrad, klwrad}) alloc(id, n2);
      for (int j = -1; j <= Mm + 2; j++)
        for (int i = -1; i <= Lm + 2; i++) {
          const double x = A(kxr, i, j), y = A(kyr, i, j);
          A(kuwnd, i, j) = 8.0 * std::sin(piy * y / cs.sizey);
          A(kvwnd, i, j) = 2.0 * std::cos(piy * x / cs.sizex);
          A(ktair, i, j) = 10.0 + 3.0 * std::cos(2.0 * piy * x / cs.sizex);
          A(kqair, i, j) = 0.007 + 0.001 * std::sin(2.0 * piy * y / cs.sizey);
          A(kprate, i, j) = 0.3;
          A(kswrad, i, j) = 150.0 + 50.0 * std::sin(piy * y / cs.sizey);
          A(klwrad, i, j) = 320.0;
        }
    }
    for (int j = -1; j <= Mm + 2; j++)
      for (int i = -1; i <= Lm + 2; i++) {
        if (cs.bulk_frc) continue;
        A(ksustr, i, j) = 1.0e-4 * std::sin(piy * A(kyr, i, j) / cs.sizey);
        if (cs.surf_flux) {  // synthetic ana_stflux/ana_srflux (oracle_main.c or_ana_forces)
          const double x = A(kxr, i, j), y = A(kyr, i, j);
          H.arr[kstflx][(i + 1) + (long)(j + 1) * H.nx2] = -1.0e-4 * (1.0 + 0.5 * std::cos(2.0 * piy * x / cs.sizex));
          A(ksrflx, i, j) = 4.0e-5 * (1.0 + 0.5 * std::sin(piy * y / cs.sizey));
          if (cs.salinity) H.arr[kstflx][(i + 1) + (long)(j + 1) * H.nx2 + n2] = 1.0e-7 * std::cos(piy * y / cs.sizey);
        }
      }
  }
  // ana_init_generic exchanges
  wrap(H, H.arr[kzeta].data(), 1, ewp, nsp);
  wrap(H, H.arr[kubar].data(), 1, ewp, nsp);
  wrap(H, H.arr[kvbar].data(), 1, ewp, nsp);
  wrap(H, H.arr[ku].data(), N, ewp, nsp);
  wrap(H, H.arr[kv].data(), N, ewp, nsp);
  for (int it = 1; it <= NT; it++) wrap(H, H.arr[kt].data() + (long)(it - 1) * 3 * n3, N, ewp, nsp);
  // analytic open-boundary data (oracle_main.c or_ana_bry): smooth along-edge
  // profiles of zeta/ubar/vbar/u/v, tracers = initial edge state + 0.05
  if (cs.obc) {
    const double pi = 3.14159265358979323;
    for (int q = 0; q < 4; q++) {
      const int nb = q < 2 ? Mm + 2 : Lm + 2;
      const int off = q < 2 ? cs.jSW_corn : cs.iSW_corn;
      std::vector<double>& bz = H.arr[ROMS_zeta_west + q];
      std::vector<double>& bub = H.arr[ROMS_ubar_west + q];
      std::vector<double>& bvb = H.arr[ROMS_vbar_west + q];
      std::vector<double>& bu = H.arr[ROMS_u_west + q];
      std::vector<double>& bv = H.arr[ROMS_v_west + q];
      std::vector<double>& bt = H.arr[ROMS_t_west + q];
      bz.assign(nb, 0.0); bub.assign(nb, 0.0); bvb.assign(nb, 0.0);
      bu.assign((size_t)nb * N, 0.0); bv.assign((size_t)nb * N, 0.0); bt.assign((size_t)nb * N * NT, 0.0);
      for (int m = 0; m < nb; m++) {
        const int mg = m + off;
        const double s = q < 2 ? ((double)mg - 0.5) / (double)cs.MMm : ((double)mg - 0.5) / (double)cs.LLm;
        const double sgn = (q == 0 || q == 2) ? 1.0 : -1.0;
        bz[m] = sgn * (q < 2 ? 0.05 : 0.03) * std::sin(pi * s);
        bub[m] = q < 2 ? 0.02 * std::sin(pi * s) : 0.01;
        bvb[m] = q < 2 ? -0.01 : 0.015 * std::sin(pi * s);
        for (int k = 1; k <= N; k++) {
          const double fk = 1.0 + 0.2 * ((double)k - 0.5) / (double)N;
          bu[m + (size_t)nb * (k - 1)] = bub[m] * fk;
          bv[m + (size_t)nb * (k - 1)] = bvb[m] * fk;
          const int i = q == 0 ? 0 : q == 1 ? Lm + 1 : m, j = q == 2 ? 0 : q == 3 ? Mm + 1 : m;
          for (int it = 1; it <= NT; it++) bt[m + (size_t)nb * ((k - 1) + (size_t)N * (it - 1))] = T(i, j, k, 1, it) + 0.05;
        }
      }
    }
  }
}

}  // namespace roms
