// k_bulk.hip -- BULK_FRC surface forcing on the device: calc_all_bulk_forces
// (bulk_frc.F:143-913), the COARE 3.0 bulk parameterisation of the air-sea
// momentum, heat and fresh-water fluxes, with the surface-current feedback
// on the stress (CFB) and the rho- to u/v-point stress averages.
//
// Inputs (host uploads, the set_frc_data results of bulk_frc.F:85-141 for
// the current time, all at rho points): uwnd, vwnd [m/s], tair [degC],
// qair = Q [kg/kg], prate [cm/day], swrad (the short-wave data, W/m2, which
// the reference reads into srflx before converting it in place) and lwrad
// (downward long-wave, W/m2); the model's surface t(N,nrhs), u,v(N,nrhs).
// Outputs: srflx [degC m/s], stflx(:,:,itemp), swflx, sustr_r, svstr_r
// (rho points, used by lmd_kpp.F:174 for u*) and sustr, svstr (u/v points).
// Without QCORRECTION / SFLX_CORR / TAU_CORRECTION / SEA_ICE_NOFLUX /
// DIURNAL_SRFLUX (not defined by Examples/Iceland; stflx(isalt) is left as
// the host set it).  One thread per rho point; FP64 with the reference's
// operation order.
#include "roms_dev.h"

namespace roms {

namespace {

// bulk_frc.F:916-976 (Grachev et al. 2000 convective, Beljaars-Holtslag stable)
__device__ double bulk_psiu(double ZoL, double pi) {
  const double r3 = 1.0 / 3.0;
  double Fw, cff, psic, psik, x, y;
  if (ZoL < 0.0) {
    x = pow(1.0 - 15.0 * ZoL, 0.25);
    psik = 2.0 * log(0.5 * (1.0 + x)) + log(0.5 * (1.0 + x * x)) - 2.0 * atan(x) + 0.5 * pi;
    cff = sqrt(3.0);
    y = pow(1.0 - 10.15 * ZoL, r3);
    psic = 1.5 * log(r3 * (1.0 + y + y * y)) - cff * atan((1.0 + 2.0 * y) / cff) + pi / cff;
    cff = ZoL * ZoL;
    Fw = cff / (1.0 + cff);
    return (1.0 - Fw) * psik + Fw * psic;
  }
  cff = fmin(50.0, 0.35 * ZoL);
  return -((1.0 + ZoL) + 0.6667 * (ZoL - 14.28) / exp(cff) + 8.525);
}
// bulk_frc.F:978-1036
__device__ double bulk_psit(double ZoL, double pi) {
  const double r3 = 1.0 / 3.0;
  double Fw, cff, psic, psik, x, y;
  if (ZoL < 0.0) {
    x = pow(1.0 - 15.0 * ZoL, 0.5);
    psik = 2.0 * log(0.5 * (1.0 + x));
    cff = sqrt(3.0);
    y = pow(1.0 - 34.15 * ZoL, r3);
    psic = 1.5 * log(r3 * (1.0 + y + y * y)) - cff * atan((1.0 + 2.0 * y) / cff) + pi / cff;
    cff = ZoL * ZoL;
    Fw = cff / (1.0 + cff);
    return (1.0 - Fw) * psik + Fw * psic;
  }
  cff = fmin(50.0, 0.35 * ZoL);
  return -(pow(1.0 + 2.0 * ZoL, 1.5) + 0.6667 * (ZoL - 14.28) / exp(cff) + 8.525);
}

constexpr double kCp = 3985.0;              // scalars.F:128
constexpr double kPi = 3.14159265358979323846;
constexpr double kCmday2ms = 0.01 / 86400.0;   // scalars.F:129 (day2sec = 86400)

// ---- the COARE flux loop over rho points (bulk_frc.F:409-800) ----
__global__ void __launch_bounds__(256) k_bulk_flux(Dev d, Range R, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const Params& P = d.p;
  const long ij = IJ(b, i, j);
  const double g = P.g, vonKar = P.vonKar, rho0 = P.rho0;
  const double blk_Rgas = 287.1, blk_ZW = 10.0, blk_ZT = 10.0, blk_ZQ = 10.0, blk_Zabl = 600.0, blk_beta = 1.2,
               blk_Cpa = 1004.67;
  const double emiss_lw = 0.985, SigmaSB = 5.6697E-8, patm = 1010.0, eps = 1.e-20, r3 = 1.0 / 3.0;
  const double cpi = 1. / kCp;
  const double rho0i = 1.0 / rho0;
  // srflx: [W/m2] -> kinematic [degC m/s] (the set_srflux part, bulk_frc.F:409)
  const double srflx = F.swrad[ij] / (rho0 * kCp);
  F.srflx[ij] = srflx;
  const double uw = F.uwnd[ij], vw = F.vwnd[ij];
  const double wspd_used = sqrt(uw * uw + vw * vw);
  const double radlw = F.lwrad[ij] / (rho0 * kCp);
  double wspd0 = wspd_used;
  const double TairC = F.tair[ij];
  const double TairK = TairC + 273.16;
  const double TseaC = F.t[ij + (long)(b.N - 1) * b.n2 + (long)(nrhs - 1) * b.n3];
  const double TseaK = TseaC + 273.16;
  const double Q = F.qair[ij];
  const double hflw = radlw - emiss_lw * rho0i * cpi * SigmaSB * TseaK * TseaK * TseaK * TseaK;
  double cff = (1.0007 + 3.46e-6 * patm) * 6.1121 * exp(17.502 * TseaC / (240.97 + TseaC));
  cff = cff * 0.98;
  const double Qsea = 0.62197 * (cff / (patm - 0.378 * cff));
  const double rhoAir = patm * 100.0 / (blk_Rgas * TairK * (1.0 + 0.61 * Q));
  const double VisAir = 1.326E-5 * (1.0 + TairC * (6.542E-3 + TairC * (8.301e-6 - 4.84e-9 * TairC)));
  const double Hlv = (2.501 - 0.00237 * TseaC) * 1.0e+6;
  double Wgus = 0.5;
  double delW = sqrt(wspd0 * wspd0 + Wgus * Wgus);
  const double delQ = Qsea - Q;
  const double delT = TseaC - TairC;
  double ZoW = 0.0001;
  const double u10 = delW * log(10.0 / ZoW) / log(blk_ZW / ZoW);
  double Wstar = 0.035 * u10;
  const double Zo10 = 0.011 * Wstar * Wstar / g + 0.11 * VisAir / Wstar;
  const double c10 = vonKar / log(10.0 / Zo10), Cd10 = c10 * c10;   // **2
  const double Ch10 = 0.00115;
  const double Ct10 = Ch10 / sqrt(Cd10);
  const double ZoT10 = 10.0 / exp(vonKar / Ct10);
  const double cW = vonKar / log(blk_ZW / Zo10);
  double Cd = cW * cW;
  const double Ct = vonKar / log(blk_ZT / ZoT10);
  const double CC = vonKar * Ct / Cd;
  const double Ribcu = -blk_ZW / (blk_Zabl * 0.004 * (blk_beta * blk_beta * blk_beta));   // **3
  const double Ri = -g * blk_ZW * (delT + 0.61 * TairK * delQ) / (TairK * delW * delW);
  double Zetu;
  if (Ri < 0.0) Zetu = CC * Ri / (1.0 + Ri / Ribcu);
  else Zetu = CC * Ri / (1.0 + 3.0 * Ri / CC);
  const double L10 = blk_ZW / Zetu;
  const int IterMax = Zetu > 50.0 ? 1 : 3;
  Wstar = delW * vonKar / (log(blk_ZW / Zo10) - bulk_psiu(blk_ZW / L10, kPi));
  double Tstar = -delT * vonKar / (log(blk_ZT / ZoT10) - bulk_psit(blk_ZT / L10, kPi));
  double Qstar = -delQ * vonKar / (log(blk_ZQ / ZoT10) - bulk_psit(blk_ZQ / L10, kPi));
  double charn;
  if (delW > 18.0) charn = 0.018;
  else if ((10.0 < delW) && (delW <= 18.0)) charn = 0.011 + 0.125 * (0.018 - 0.011) * (delW - 10.);
  else charn = 0.011;
  for (int iter = 1; iter <= IterMax; iter++) {
    ZoW = charn * Wstar * Wstar / g + 0.11 * VisAir / (Wstar + eps);
    const double Rr = ZoW * Wstar / VisAir;
    const double ZoQ = fmin(1.15e-4, 5.5e-5 / pow(Rr, 0.6));
    const double ZoT = ZoQ;
    const double ZoL = vonKar * g * blk_ZW * (Tstar * (1.0 + 0.61 * Q) + 0.61 * TairK * Qstar) /
                       (TairK * Wstar * Wstar * (1.0 + 0.61 * Q) + eps);
    const double L = blk_ZW / (ZoL + eps);
    const double Wpsi = bulk_psiu(ZoL, kPi);
    const double Tpsi = bulk_psit(blk_ZT / L, kPi);
    const double Qpsi = bulk_psit(blk_ZQ / L, kPi);
    Wstar = fmax(eps, delW * vonKar / (log(blk_ZW / ZoW) - Wpsi));
    Tstar = -delT * vonKar / (log(blk_ZT / ZoT) - Tpsi);
    Qstar = -delQ * vonKar / (log(blk_ZQ / ZoQ) - Qpsi);
    const double Bff = -g / TairK * Wstar * (Tstar + 0.61 * TairK * Qstar);
    if (Bff > 0.0) Wgus = blk_beta * pow(Bff * blk_Zabl, r3);
    else Wgus = 0.2;
    delW = sqrt(wspd0 * wspd0 + Wgus * Wgus);
  }
  wspd0 = sqrt(wspd0 * wspd0 + Wgus * Wgus);
  Cd = Wstar * Wstar / (wspd0 * wspd0 + eps);
  double hfsen = -blk_Cpa * rhoAir * Wstar * Tstar;
  double hflat = -Hlv * rhoAir * Wstar * Qstar;
  const double upvel = -1.61 * Wstar * Qstar - (1.0 + 1.61 * Q) * Wstar * Tstar / TairK;
  hflat = hflat + rhoAir * Hlv * upvel * Q;
  hflat = -hflat * rho0i * cpi;
  hfsen = -hfsen * rho0i * cpi;
  const double rm = F.rmask[ij];
  double stT = srflx + hflw + hflat + hfsen;
  if (P.salinity) {
    const double evap = -kCp * hflat / Hlv;
    F.swflx[ij] = F.prate[ij] * kCmday2ms - evap;
  }
  F.stflx[ij] = stT * rm;   // MASKING (stflx(isalt) * rmask: the host's value, masked as the reference)
  if (P.salinity) F.stflx[ij + b.n2] = F.stflx[ij + b.n2] * rm;
  const double aer = rhoAir * wspd0 * rho0i, cer = Cd;
  F.sustr_r[ij] = aer * cer * uw * rm;
  F.svstr_r[ij] = aer * cer * vw * rm;
}

// ---- surface-current feedback on the rho-point stresses (bulk_frc.F:823-895):
// sustr_r on istrR..iend+1 x jstrR..jendR, svstr_r on istrR..iendR x jstrR..jend+1 ----
__global__ void __launch_bounds__(256) k_bulk_cfb(Dev d, Range R, int nrhs) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), oN = ij + (long)(b.N - 1) * b.n2 + (long)(nrhs - 1) * b.n3;
  const double Wspd_min = 3., stau_ref = -0.0027, cfb_slope = -0.0029, cfb_offset = 0.008;
  const double rho0 = d.p.rho0;
  const double uw = F.uwnd[ij], vw = F.vwnd[ij];
  const double wspd = sqrt(uw * uw + vw * vw);
  const double cff = wspd > Wspd_min ? cfb_slope * wspd + cfb_offset : stau_ref;
  if (i <= b.iend + 1) F.sustr_r[ij] = F.sustr_r[ij] + cff * 0.5 * (F.u[oN] + F.u[oN + 1]) / rho0;
  if (j <= b.jend + 1) F.svstr_r[ij] = F.svstr_r[ij] + cff * 0.5 * (F.v[oN] + F.v[oN + b.nx2]) / rho0;
}

// ---- rho -> u/v points (bulk_frc.F:866-873, 903-910) ----
__global__ void __launch_bounds__(256) k_bulk_uv(Dev d, Range R) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j);
  if (i >= R.i0 + 1 && i <= b.iend + 1) F.sustr[ij] = (F.sustr_r[ij - 1] + F.sustr_r[ij]) / 2 * F.umask[ij];
  if (j >= R.j0 + 1 && j <= b.jend + 1) F.svstr[ij] = (F.svstr_r[ij - b.nx2] + F.svstr_r[ij]) / 2 * F.vmask[ij];
}

}  // namespace

void launch_bulk_flux(const Dev& d, hipStream_t s, int nrhs) {
  if (!d.p.bulk_frc) return;
  const Bounds& b = d.b;
  const Range RE{b.istrE, b.iendE, b.jstrE, b.jendE};   // compute_extended_bounds.h
  hipLaunchKernelGGL(k_bulk_flux, grid_of(RE), dim3(kBX, kBY), 0, s, d, RE, nrhs);
  hipLaunchKernelGGL(k_bulk_cfb, grid_of(RE), dim3(kBX, kBY), 0, s, d, RE, nrhs);
  hipLaunchKernelGGL(k_bulk_uv, grid_of(RE), dim3(kBX, kBY), 0, s, d, RE);
}

}  // namespace roms
