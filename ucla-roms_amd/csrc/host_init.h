// host_init.h -- host-side setup of analytic cases (see host_init.cpp).
#pragma once
#include <vector>

#include "roms_dev.h"
#include "../../include/roms_gpu.h"

namespace roms {

enum HostId : int {
  kh = ROMS_h, khinv = ROMS_hinv, kf = ROMS_f, kfomn = ROMS_fomn, kpm = ROMS_pm, kpn = ROMS_pn, kdm_r = ROMS_dm_r,
  kdn_r = ROMS_dn_r, kdm_u = ROMS_dm_u, kdn_u = ROMS_dn_u, kdm_v = ROMS_dm_v, kdn_v = ROMS_dn_v, kdm_p = ROMS_dm_p,
  kdn_p = ROMS_dn_p, kpmon_u = ROMS_pmon_u, kpnom_v = ROMS_pnom_v, krmask = ROMS_rmask, kpmask = ROMS_pmask,
  kumask = ROMS_umask, kvmask = ROMS_vmask, kCs_w = ROMS_Cs_w, kCs_r = ROMS_Cs_r, kzeta = ROMS_zeta,
  kubar = ROMS_ubar, kvbar = ROMS_vbar, ku = ROMS_u, kv = ROMS_v, kt = ROMS_t, kHz = ROMS_Hz, kz_r = ROMS_z_r,
  kz_w = ROMS_z_w, kAkv = ROMS_Akv, kAkt = ROMS_Akt, kvisc2_r = ROMS_visc2_r, kvisc2_p = ROMS_visc2_p,
  kdiff2 = ROMS_diff2, ksustr = ROMS_sustr, ksvstr = ROMS_svstr, kstflx = ROMS_stflx, ksrflx = ROMS_srflx,
  kswflx = ROMS_swflx, kdndx = ROMS_dndx, kdmde = ROMS_dmde,
  kuwnd = ROMS_uwnd, kvwnd = ROMS_vwnd, ktair = ROMS_tair, kqair = ROMS_qair, kprate = ROMS_prate,
  kswrad = ROMS_swrad, klwrad = ROMS_lwrad,
  kxr = ROMS_NFIELDS, kyr, kNHost
};

struct HostState {
  int Lm, Mm, N, NT, nTS, nx2;
  long n2;
  std::vector<double> arr[kNHost];
  bool wrap_on = true;
  // pipe_frc.F (analytic pipes): npip = 0 when pipe_source is off
  int npip = 0;
  std::vector<int> pipe_idx;
  std::vector<double> pipe_flx, pipe_prf, pipe_trc;
  // river_frc.F (analytic river): nriv = 0 when river_source is off
  int nriv = 0;
  std::vector<double> riv_uflx, riv_vflx, riv_vol, riv_trc;
  HostState(int Lm_, int Mm_, int N_, int NT_, int nTS_);
  std::vector<double>& a(int id);
};

struct CaseSpec {
  int case_id, LLm, MMm;
  int iSW_corn, jSW_corn;
  int ew_periodic, ns_periodic, west_exchng, east_exchng, south_exchng, north_exchng;
  int salinity, lmd, surf_flux;
  int obc, island;   // open edges (bitmask), circular land mask
  int curvgrid;      // non-uniform metrics + dndx/dmde
  int bulk_frc;      // BULK_FRC analytic atmosphere (basin)
  double v_sponge;   // set_nudgcof.F sponge
  int host_wrap;  // apply periodic halo wraps on the host (single rank)
  double theta_s, theta_b, hc, rho0, Tcoef, visc2, tnu2, Akv_bak, Akt_bak[2];
  double sizex, sizey;
};

int set_weights(int ndtfast, double w[2][kMaxFast]);
void set_scoord(int N, double theta_s, double theta_b, double* Cs_w, double* Cs_r);
void build_case(const CaseSpec& cs, HostState& H, double& area, double& volume);
double pair_sum(const HostState& H, const std::vector<double>& A);

}  // namespace roms
