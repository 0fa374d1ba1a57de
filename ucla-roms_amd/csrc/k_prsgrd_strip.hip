// k_prsgrd_strip.hip -- prsgrd's ru/rv (prsgrd.F:229-305 XI, 345-421 ETA)
// together with the horizontal momentum r.h.s. of the following pre_step3d /
// step3d_uv1 (compute_horiz_rhs_uv_terms.h:1-291, UV_COR + UV_ADV), in
// strips that march along j.
//
// One wavefront is one strip of 64 consecutive columns c0..c0+63 at one
// level; it owns the 60 columns c0+2..c0+61 and marches its rows j one after
// the other.  Every value a cell needs from its i-neighbours comes from the
// neighbouring lane through a DPP wave shift (v_mov_b32_dpp wave_shr:1 /
// wave_shl:1, two per double), and every value it needs from its
// j-neighbours stays in registers from the rows before, so each elementary
// difference, harmonic mean and advective flux is evaluated once per face
// (k_prsgrd_uv evaluates each momentum flux twice and stages every
// intermediate through LDS).  The two lanes on each side only feed their
// neighbours: a cell at lane l reads lanes l-2..l+2.
//
// Only rows no closed-edge extrapolation reaches take this path (jA..jB,
// launch_prsgrd); the strips at a closed west/east edge apply the
// reference's one-sided extrapolations (FC(istrU-1) = FC(istrU), ...) as a
// lane shuffle to the clamped column.  The rows of the south and north bands
// go through k_prsgrd_uv.  Every value is formed with k_prsgrd_uv's and
// uv_horiz_rhs_pre's expressions in their order: bit-identical.
#include "k_common.h"

namespace roms {

namespace {
// lane l gets lane l-1's value (wave_shr:1) / lane l+1's (wave_shl:1); the
// lane without a source gets 0 (it feeds nothing an owned cell uses)
__device__ __forceinline__ double dpp_shr(double x) {
  const long long v = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double dpp_shl(double x) {
  const long long v = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double harm2(double a, double b) {   // k_prsgrd.hip harm()
  const double c = 2.0 * a * b;
  return c > 0.0 ? c / (a + b) : 0.0;
}
}  // namespace

constexpr int kStripOwn = 60;   // owned columns per strip (lanes 2..61)
#ifndef ROMS_PRS_STRIP_PF
#define ROMS_PRS_STRIP_PF 1   // 1: the next row's inputs are loaded before this row's stores
#endif
#ifndef ROMS_PRS_STRIP_J
#define ROMS_PRS_STRIP_J 8    // rows per wavefront
#endif
#ifndef ROMS_PRS_STRIP_WAVES
#define ROMS_PRS_STRIP_WAVES 1   // __launch_bounds__ minimum waves per SIMD
#endif

// geometry of one launch (launch_prsgrd)
struct StripGeom {
  int c00;           // column of lane 0 of strip 0
  int ilast;         // last owned column (iend)
  int jA, jB;        // rows of the launch
  int imin, imax;    // FC / rx extrapolation (prsgrd.F:229-240)
  int uimin, uimax;  // uxx, Huxx (compute_horiz_rhs_uv_terms.h:55-75)
  int ximin, ximax;  // vxx (compute_horiz_rhs_uv_terms.h:160-172)
  int xlo, xhi;      // strips whose used columns all lie in [xlo, xhi] need no extrapolation
};

template <bool SPLIT, bool UP, int J>
__global__ void __launch_bounds__(64, ROMS_PRS_STRIP_WAVES) k_prsgrd_strip(Dev d, StripGeom G, int nrhs) {
  const uint3 bI = xcd_tile();
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double HalfGRho = 0.5 * (g / rho0);
  const double delta = 0.1666666666666667, gamma = 0.3333333333333333;
  const int lane = (int)threadIdx.x;
  const int c0 = G.c00 + (int)bI.x * kStripOwn;
  const int i = c0 + lane;
  const int ja = G.jA + (int)bI.y * J;
  const int nrow = min(J, G.jB - ja + 1);   // rows of this wave (uniform)
  const int k = 1 + (int)bI.z;
  // loads: the lane's column clamped into the array (the lanes past Lm+2 of
  // the last strip feed nothing an owned cell uses); row r at vo + (r-ja)*rb
  const int il = min(i, b.Lm + 2);
  const unsigned rb = (unsigned)b.nx2 * 8u;
  const unsigned vo = (unsigned)IJ(b, il, ja) * 8u;
  const unsigned sk = (unsigned)((long)(k - 1) * b.n2) * 8u;
  const BufF64 bZ(F.z_r), bR(SPLIT ? F.rho1 : F.rho), bQ(F.qp1), bHz(F.Hz), bP(F.P);
  const BufF64 bU(F.u + (long)(nrhs - 1) * b.n3), bV(F.v + (long)(nrhs - 1) * b.n3), bFU(F.FlxU), bFV(F.FlxV);
  const BufF64 bum(F.umask), bvm(F.vmask), bdn(F.dn_u), bdm(F.dm_v), bfo(F.fomn);
  const BufF64 bru(F.ru), brv(F.rv);
  auto L3 = [&](const BufF64& B, int r) { return B.ld(vo + (unsigned)(r - ja) * rb, sk); };
  auto L2 = [&](const BufF64& B, int r) { return B.ld(vo + (unsigned)(r - ja) * rb, 0u); };
  // owned cells and their ru / rv predicates (prsgrd.F:229 / 345 loop bounds)
  const bool own = lane >= 2 && lane <= 61 && i <= G.ilast;
  const bool du = own && i >= b.istrU && i <= b.iend;
  const bool dv = own && i >= b.istr && i <= b.iend;
  // closed-edge extrapolation: the clamped column's value, as a lane shuffle
  const bool xedge = c0 + 1 < G.xlo || c0 + 62 > G.xhi;   // uniform
  const int lpg = iclamp(i, G.imin, G.imax) - c0, lu = iclamp(i, G.uimin, G.uimax) - c0,
            lx = iclamp(i, G.ximin, G.ximax) - c0;
  auto rhov = [&](double r1, double q1, double z) {   // in-situ density (k_prsgrd_uv rhov)
    if (SPLIT) {
      const double dpth = -z;
      return r1 + q1 * dpth * (1.0 - qp2 * dpth);
    }
    return r1;
  };
  // elementary differences between two points (k_prsgrd_uv's stage 2): point
  // 1 east / north of point 0, mask at the u- / v-point
  auto efc = [&](double z1, double z0, double mk) { return (z1 - z0) * mk; };
  auto erx = [&](double r1, double r0, double q1, double q0, double z1, double z0, double mk) {
    if (SPLIT) {
      const double dpth = -0.5 * (z1 + z0);
      return (r1 - r0 + (q1 - q0) * dpth * (1.0 - qp2 * dpth)) * mk;
    }
    return (r1 - r0) * mk;
  };
  // harmonic means at a rho point (stage 3), with SPLIT_EOS's compressibility term
  auto hdr = [&](double rxa, double rxb, double dz, double q, double z) {
    double dr = harm2(rxa, rxb);
    if (SPLIT) dr = dr - q * dz * (1.0 + 2.0 * qp2 * z);
    return dr;
  };
  auto sec = [](double m1, double c, double p1) { return m1 - 2.0 * c + p1; };   // uxx_at / vee_at ... form
  // the four advective fluxes (adv_UFx, adv_VFe, adv_UFe, adv_VFx of k_common.h)
  auto fUFx = [&](double u0, double u1, double ux0, double ux1, double f0, double f1, double Hx0, double Hx1) {
    if (UP) {
      const double cff = f0 + f1 - delta * (Hx0 + Hx1);
      return 0.25 * (cff * (u0 + u1) - gamma * (fmax0(cff) * ux0 + fmin0(cff) * ux1));
    }
    return 0.25 * (u0 + u1 - delta * (ux0 + ux1)) * (f0 + f1 - delta * (Hx0 + Hx1));
  };
  auto fVFe = [&](double v0, double v1, double ve0, double ve1, double f0, double f1, double He0, double He1) {
    if (UP) {
      const double cff = f0 + f1 - delta * (He0 + He1);
      return 0.25 * (cff * (v0 + v1) - gamma * (fmax0(cff) * ve0 + fmin0(cff) * ve1));
    }
    return 0.25 * (v0 + v1 - delta * (ve0 + ve1)) * (f0 + f1 - delta * (He0 + He1));
  };
  // UFe at psi (i,m): u(i,m), u(i,m-1), uee(m-1), uee(m), fv(i,m), fv(i-1,m), Hvxx(i,m), Hvxx(i-1,m)
  auto fUFe = [&](double um, double umm, double um1, double u0, double fv0, double fvm, double Hv0, double Hvm) {
    if (UP) {
      const double cff = fv0 + fvm - delta * (Hv0 + Hvm);
      return 0.25 * (cff * (um + umm) - gamma * (fmax0(cff) * um1 + fmin0(cff) * u0));
    }
    return 0.25 * (um + umm - delta * (u0 + um1)) * (fv0 + fvm - delta * (Hv0 + Hvm));
  };
  // VFx at psi (m,j): v(m,j), v(m-1,j), vxx(m-1), vxx(m), fu(m,j), fu(m,j-1), Huee(m,j), Huee(m,j-1)
  auto fVFx = [&](double vm, double vmm, double vm1, double v0, double fu0, double fum, double Hu0, double Hum) {
    if (UP) {
      const double cff = fu0 + fum - delta * (Hu0 + Hum);
      return 0.25 * (cff * (vm + vmm) - gamma * (fmax0(cff) * vm1 + fmin0(cff) * v0));
    }
    return 0.25 * (vm + vmm - delta * (v0 + vm1)) * (fu0 + fum - delta * (Hu0 + Hum));
  };

  // ---- prologue: the rows above ja the march carries ----
  const int j = ja;
  double Um2 = L3(bU, j - 2), Um1 = L3(bU, j - 1), U0 = L3(bU, j), U1 = L3(bU, j + 1);
  double Vm2 = L3(bV, j - 2), Vm1 = L3(bV, j - 1), V0 = L3(bV, j), V1 = L3(bV, j + 1);
  double FVm2 = L3(bFV, j - 2), FVm1 = L3(bFV, j - 1), FV0 = L3(bFV, j), FV1 = L3(bFV, j + 1);
  double FUm2 = L3(bFU, j - 2), FUm1 = L3(bFU, j - 1), FU0 = L3(bFU, j);
  double Zm2 = L3(bZ, j - 2), Zm1 = L3(bZ, j - 1), Z0 = L3(bZ, j);
  double Rm2 = L3(bR, j - 2), Rm1 = L3(bR, j - 1), R0 = L3(bR, j);
  double Qm2 = SPLIT ? L3(bQ, j - 2) : 0.0, Qm1 = SPLIT ? L3(bQ, j - 1) : 0.0, Q0 = SPLIT ? L3(bQ, j) : 0.0;
  double vmm1 = L2(bvm, j - 1), vm0 = L2(bvm, j);
  double HZm1 = L3(bHz, j - 1), PPm1 = L3(bP, j - 1), fom1 = L2(bfo, j - 1);
  // v-points ja-1, ja and the harmonic mean at rho row ja-1
  const double fcyA = efc(Zm1, Zm2, vmm1), rxyA = erx(Rm1, Rm2, Qm1, Qm2, Zm1, Zm2, vmm1);
  double fcy = efc(Z0, Zm1, vm0), rxy = erx(R0, Rm1, Q0, Qm1, Z0, Zm1, vm0);
  double dZyP = harm2(fcyA, fcy);
  double dRyP = hdr(rxyA, rxy, dZyP, Qm1, Zm1);
  double rvP = rhov(Rm1, Qm1, Zm1);
  // UFe(i, ja), VFe(i, ja-1), the j-second differences at row ja, Huee(ja-1)
  double uee = sec(Um1, U0, U1);
  double UFeP;
  {
    const double ueeA = sec(Um2, Um1, U0);
    const double Hv = sec(dpp_shr(FV0), FV0, dpp_shl(FV0));
    UFeP = fUFe(U0, Um1, ueeA, uee, FV0, dpp_shr(FV0), Hv, dpp_shr(Hv));
  }
  double vee = sec(Vm1, V0, V1), Hvee = sec(FVm1, FV0, FV1);
  double VFeP;
  {
    const double veeA = sec(Vm2, Vm1, V0), HveeA = sec(FVm2, FVm1, FV0);
    VFeP = fVFe(Vm1, V0, veeA, vee, FVm1, FV0, HveeA, Hvee);
  }
  double HueeP = sec(FUm2, FUm1, FU0);
  double urP = dpp_shl(Um1);   // u(i+1, j-1)

  // ---- the march: row j's new inputs are loaded one row ahead (PF) ----
  double nU = 0, nV = 0, nFV = 0, nFU = 0, nZ = 0, nR = 0, nQ = 0, nvm = 0, nHZ = 0, nPP = 0, num = 0, ndn = 0,
         ndm = 0, nfo = 0;
  auto load_row = [&](int jr) {   // inputs new at row jr
    nU = L3(bU, jr + 2); nV = L3(bV, jr + 2); nFV = L3(bFV, jr + 2); nFU = L3(bFU, jr + 1);
    nZ = L3(bZ, jr + 1); nR = L3(bR, jr + 1); if (SPLIT) nQ = L3(bQ, jr + 1); nvm = L2(bvm, jr + 1);
    nHZ = L3(bHz, jr); nPP = L3(bP, jr); num = L2(bum, jr); ndn = L2(bdn, jr); ndm = L2(bdm, jr); nfo = L2(bfo, jr);
  };
  if (ROMS_PRS_STRIP_PF) load_row(j);
#pragma unroll
  for (int r = 0; r < J; r++) {
    if (r >= nrow) break;
    const int jr = ja + r;
    if (!ROMS_PRS_STRIP_PF) load_row(jr);
    const double U2 = nU, V2 = nV, FV2 = nFV, FU1 = nFU, Z1 = nZ, R1 = nR, Q1 = nQ, vm1 = nvm;
    const double HZ0 = nHZ, PP0 = nPP, um0 = num, dn0 = ndn, dm0 = ndm, fo0 = nfo;
    if (ROMS_PRS_STRIP_PF && r + 1 < nrow) load_row(jr + 1);   // the next row's inputs, before this row's stores
    // -- pressure gradient, XI: u-point at this lane (between i-1 and i),
    // harmonic means at rho points i (this lane) and i-1 (from the left) --
    const double Zl = dpp_shr(Z0), Rl = dpp_shr(R0), Ql = SPLIT ? dpp_shr(Q0) : 0.0;
    double fcx = efc(Z0, Zl, um0), rxx = erx(R0, Rl, Q0, Ql, Z0, Zl, um0);
    if (xedge) { fcx = __shfl(fcx, lpg); rxx = __shfl(rxx, lpg); }
    const double dZx = harm2(fcx, dpp_shl(fcx));
    const double dRx = hdr(rxx, dpp_shl(rxx), dZx, Q0, Z0);
    const double dZxm = dpp_shr(dZx), dRxm = dpp_shr(dRx);
    const double v0 = rhov(R0, Q0, Z0), vl = dpp_shr(v0);
    const double hzl = dpp_shr(HZ0), Pl = dpp_shr(PP0);
    const double pru = 0.5 * (HZ0 + hzl) * dn0 *
                       (Pl - PP0 -
                        HalfGRho * ((v0 + vl) * (Z0 - Zl) -
                                    OneFifth * ((dRx - dRxm) * (Z0 - Zl - OneTwelfth * (dZx + dZxm)) -
                                                (dZx - dZxm) * (v0 - vl - OneTwelfth * (dRx + dRxm)))));
    // -- ETA: v-point j+1, harmonic mean at rho row j (row j-1 carried) --
    const double fcy1 = efc(Z1, Z0, vm1), rxy1 = erx(R1, R0, Q1, Q0, Z1, Z0, vm1);
    const double dZy = harm2(fcy, fcy1);
    const double dRy = hdr(rxy, rxy1, dZy, Q0, Z0);
    const double prv = 0.5 * (HZ0 + HZm1) * dm0 *
                       (PPm1 - PP0 -
                        HalfGRho * ((v0 + rvP) * (Z0 - Zm1) -
                                    OneFifth * ((dRy - dRyP) * (Z0 - Zm1 - OneTwelfth * (dZy + dZyP)) -
                                                (dZy - dZyP) * (v0 - rvP - OneTwelfth * (dRy + dRyP)))));
    // -- advective fluxes: UFx at rho (i,j), VFx at psi (i,j), UFe at psi
    // (i,j+1), VFe at rho (i,j); their i-1 / i+1 / j / j-1 partners come
    // from the neighbouring lanes and the row before --
    const double ul = dpp_shr(U0), ur = dpp_shl(U0);
    double uxx = sec(ul, U0, ur);
    const double fl = dpp_shr(FU0), fr = dpp_shl(FU0);
    double Huxx = sec(fl, FU0, fr);
    if (xedge) { uxx = __shfl(uxx, lu); Huxx = __shfl(Huxx, lu); }
    const double UFx = fUFx(U0, ur, uxx, dpp_shl(uxx), FU0, fr, Huxx, dpp_shl(Huxx));
    const double vlf = dpp_shr(V0), vrt = dpp_shl(V0);
    double vxx = sec(vlf, V0, vrt);
    if (xedge) vxx = __shfl(vxx, lx);
    const double Huee = sec(FUm1, FU0, FU1);
    const double VFx = fVFx(V0, vlf, dpp_shr(vxx), vxx, FU0, FUm1, Huee, HueeP);
    const double uee1 = sec(U0, U1, U2);
    const double fvl = dpp_shr(FV1);
    const double Hv = sec(fvl, FV1, dpp_shl(FV1));
    const double UFe = fUFe(U1, U0, uee, uee1, FV1, fvl, Hv, dpp_shr(Hv));
    const double vee1 = sec(V0, V1, V2), Hvee1 = sec(FV0, FV1, FV2);
    const double VFe = fVFe(V0, V1, vee, vee1, FV0, FV1, Hvee, Hvee1);
    // -- Coriolis, then advection, into ru / rv (uv_horiz_rhs_pre order) --
    const double c0c = 0.5 * HZ0 * (fo0);
    double ru = pru;
    {
      const double c1 = 0.5 * hzl * (dpp_shr(fo0));
      const double Uc0 = c0c * (V0 + V1), Uc1 = c1 * (vlf + dpp_shr(V1));
      ru = ru + 0.5 * (Uc0 + Uc1);
    }
    ru = ru - UFx + dpp_shr(UFx) - UFe + UFeP;
    double rv = prv;
    {
      const double c1 = 0.5 * HZm1 * (fom1);
      const double Vc0 = c0c * (U0 + ur), Vc1 = c1 * (Um1 + urP);
      rv = rv - 0.5 * (Vc0 + Vc1);
    }
    rv = rv - dpp_shl(VFx) + VFx - VFe + VFeP;
    const unsigned vr = vo + (unsigned)r * rb;
    bru.st(ru, du ? vr : kBufOff, sk);
    brv.st(rv, dv ? vr : kBufOff, sk);
    // -- carry to row j+1 --
    Um1 = U0; U0 = U1; U1 = U2; urP = ur;
    V0 = V1; V1 = V2;
    FV0 = FV1; FV1 = FV2;
    FUm1 = FU0; FU0 = FU1;
    Zm1 = Z0; Z0 = Z1; R0 = R1; Q0 = Q1;
    fcy = fcy1; rxy = rxy1; dZyP = dZy; dRyP = dRy; rvP = v0;
    HZm1 = HZ0; PPm1 = PP0; fom1 = fo0;
    uee = uee1; UFeP = UFe; vee = vee1; Hvee = Hvee1; VFeP = VFe; HueeP = Huee;
  }
}

// ru, rv of rows jA..jB (every column istr..iend) in strips; false if the
// configuration is not one this kernel covers (the caller runs k_prsgrd_uv)
bool launch_prsgrd_strip(const Dev& d, hipStream_t s, int nrhs, int up, int imin, int imax, int jmin, int jmax,
                         const UVBounds& ub, int& jA, int& jB) {
  const Bounds& b = d.b;
  // rows whose stencils no j-extrapolation reaches (FC: jmin..jmax; vee,
  // Hvee: v_jmin..v_jmax; uee: e_jmin..e_jmax) and whose ru, rv both exist
  jA = std::max(std::max(jmin, ub.v_jmin), ub.e_jmin) + 1;
  jA = std::max(jA, std::max(b.jstr, b.jstrV));
  jA = std::max(jA, 1);   // rows jA-2.. are read
  jB = std::min(std::min(jmax, ub.v_jmax), ub.e_jmax) - 1;
  jB = std::min(jB, b.jend);
  jB = std::min(jB, b.Mm);   // rows ..jB+2 are read
  if (jB < jA) return false;
  StripGeom G;
  G.c00 = b.istr - 2;
  G.ilast = b.iend;
  G.jA = jA; G.jB = jB;
  G.imin = imin; G.imax = imax;
  G.uimin = ub.u_imin; G.uimax = ub.u_imax;
  G.ximin = ub.x_imin; G.ximax = ub.x_imax;
  G.xlo = std::max(std::max(imin, ub.u_imin), ub.x_imin);
  G.xhi = std::min(std::min(imax, ub.u_imax), ub.x_imax);
  if (G.c00 < -1) return false;   // lane 0 reads column c0
  constexpr int J = ROMS_PRS_STRIP_J;
  const dim3 grid((unsigned)((b.iend - b.istr + kStripOwn) / kStripOwn), (unsigned)((jB - jA + J) / J), (unsigned)b.N);
  const int split = d.p.nonlin_eos;
  if (split && up) hipLaunchKernelGGL((k_prsgrd_strip<true, true, J>), grid, dim3(64), 0, s, d, G, nrhs);
  else if (split) hipLaunchKernelGGL((k_prsgrd_strip<true, false, J>), grid, dim3(64), 0, s, d, G, nrhs);
  else if (up) hipLaunchKernelGGL((k_prsgrd_strip<false, true, J>), grid, dim3(64), 0, s, d, G, nrhs);
  else hipLaunchKernelGGL((k_prsgrd_strip<false, false, J>), grid, dim3(64), 0, s, d, G, nrhs);
  return true;
}

}  // namespace roms
