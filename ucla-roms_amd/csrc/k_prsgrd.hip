// k_prsgrd.hip -- prsgrd_tile (prsgrd.F:25-510): Shchepetkin-McWilliams (2003)
// density-Jacobian pressure gradient with harmonic-mean cubic fits.
//
// Kernel 1 (per column over 0..nx x 0..ny): elementary vertical differences,
// harmonic averages dR,dZ and the top-down hydrostatic pressure P, all in
// registers (rolling window over k) -- no (N+1)-deep scratch.  (The in-situ
// density rho1 + qp1*dpth*(1-qp2*dpth) of SPLIT_EOS is re-formed from the
// raw window wherever kernel 2 needs it; it is not stored.)
// Kernel 2 (per column): XI and ETA components ru, rv; each lane rebuilds the
// three u-point (v-point) elementary differences it needs, with the
// reference's one-sided extrapolation at closed edges expressed as a clamp.
#include "k_common.h"

namespace roms {

// k_prsgrd_strip.hip: rows jA..jB of the fused form in j-marching strips
bool launch_prsgrd_strip(const Dev& d, hipStream_t s, int nrhs, int up, int imin, int imax, int jmin, int jmax,
                         const UVBounds& ub, int& jA, int& jB);

__device__ __forceinline__ double harm(double a, double b) {
  const double c = 2.0 * a * b;
  return c > 0.0 ? c / (a + b) : 0.0;
}

__global__ void __launch_bounds__(256) k_prsgrd_P(Dev d, Range R, int split, int tides) {
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
    }
    if (doP) {
      double Pk;
      if (k == N) {
        const double zw = F.z_w[ij + (long)N * n2];
        const double rNm = rhov(rM, qM, zM);
        Pk = g * zw + grho * (v0 + 0.5 * (v0 - rNm) * (zw - zC) / (zC - zM)) * (zw - zC);
        if (tides) Pk = Pk - g * F.ptide[ij];   // TIDES: pot_tides (prsgrd.F:209-211)
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
// Raw window of the level: z_r, rho1 (rho) and qp1 over (i0-2..i0+64) x
// (j0-2..j0+4), each value loaded from HBM once per block and coalesced; the
// elementary differences, the harmonic means' split terms and the cell's own
// z_r and in-situ density are then formed from LDS, so a block issues about
// a third of the vector-memory instructions of forming every difference
// from two global loads (measured: the per-cell kernel was bound by the
// vector-memory instruction rate, not by HBM bytes).
// (The L16 form's rows are 68 wide -- one unused column at i0+65 -- so that
// every row of the window starts on a 16-B boundary in LDS.)
constexpr int kPWW = kBX + 3, kPWH = kBY + 3, kPWN = kPWW * kPWH;   // raw window (i0-2.., j0-2..)
constexpr int kPWQ = (kPWN + kBX * kBY - 1) / (kBX * kBY);
constexpr int kPQ = (kPXN + kPYN + kBX * kBY - 1) / (kBX * kBY);
// L16 (Params::ld16, the padded device pitch): the raw window and the u/v
// window are read two doubles per lane (global_load_dwordx4 / ds_write_b128):
// a window row starts at i0-2, and i0 = 1 (mod 16) puts i0-2 and every second
// column after it on a 16-B boundary, so half the vector-memory instructions
// fetch the same bytes (the per-cell kernel is bound by that instruction rate,
// DESIGN.md section 4).  Cells outside -1..Lm+2 / -1..Mm+2 read as 0, as in
// the 8-B form: bit-identical.
// BUF (8-B form only, Params::prs_buf): the windows through raw-buffer loads,
// the entry's column in a 32-bit VGPR offset and the level in an SGPR
// (a window entry outside the grid takes kBufOff and reads 0): no 64-bit
// address arithmetic per entry.  Bit-identical.
template <bool FUSE, int TY = kBY, bool L16 = false, bool BUF = false>
__global__ void __launch_bounds__(kBX * TY, L16 && TY == kBY ? 5 : 1) k_prsgrd_uv(Dev d, Range R, int split, int imin, int imax, int jmin, int jmax,
                                                   UVBounds ub, int up, int nrhs) {
  const uint3 bI = h_tile(d.p.tile_grp);
  // the file-scope window sizes for a 64 x TY tile (TY = kBY: the constants above)
  constexpr int NT = kBX * TY, XN = kPXW * TY, YH = TY + 2, YN = kBX * YH;
  constexpr int PWW = L16 ? kPWW + 1 : kPWW;   // raw window row (even for L16)
  constexpr int WN = PWW * (TY + 3), WQ = (WN + NT - 1) / NT, PQ = (XN + YN + NT - 1) / NT;
  constexpr int UWN = kUVW * (TY + 4);
  // one LDS block: the raw window, the elementary differences and the
  // harmonic means (and, FUSE, the u/v window after them)
  constexpr int kPL = 3 * WN + 4 * XN + 4 * YN;
  __shared__ __attribute__((aligned(16))) double sL[kPL];
  double* const sZ = sL;
  double* const sR = sZ + WN;
  double* const sQ = sR + WN;
  double* const sFCx = sQ + WN;
  double* const sRx = sFCx + XN;
  double* const sFCy = sRx + XN;
  double* const sRy = sFCy + YN;
  double* const sdZx = sRy + YN;
  double* const sdRx = sdZx + XN;
  double* const sdZy = sdRx + XN;
  double* const sdRy = sdZy + YN;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double HalfGRho = 0.5 * (g / rho0);
  const double* R1 = split ? F.rho1 : F.rho;
  const int k = 1 + (int)bI.z;
  const long kk = (long)(k - 1) * b.n2, sj = b.nx2;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * TY;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  auto W = [&](int i, int j) { return (i - (i0 - 2)) + (j - (j0 - 2)) * PWW; };
  // ---- loads, all issued before the first barrier ----
  // 8-B form: entry q of the window per lane and round; L16: the pair of
  // entries 2p, 2p+1 (one row holds PWW / 2 pairs)
  constexpr int WP = WN / 2, WPQ = (WP + NT - 1) / NT;
  constexpr int WL = L16 ? WPQ : WQ;
  double2 wz[WL], wr[WL], wq[WL];
#pragma unroll
  for (int m = 0; m < WL; m++) {
    const int q = tid + m * NT;
    wz[m] = wr[m] = wq[m] = double2{0.0, 0.0};
    if (L16) {
      if (q < WP) {
        const int i = i0 - 2 + 2 * (q % (PWW / 2)), j = j0 - 2 + q / (PWW / 2);
        if (i >= -1 && i <= b.Lm + 2 && j <= b.Mm + 2) {
          const long o = IJ(b, i, j) + kk;
          const bool hi = i + 1 <= b.Lm + 2;
          wz[m] = *reinterpret_cast<const double2*>(F.z_r + o);
          wr[m] = *reinterpret_cast<const double2*>(R1 + o);
          if (split) wq[m] = *reinterpret_cast<const double2*>(F.qp1 + o);
          if (!hi) { wz[m].y = 0.0; wr[m].y = 0.0; wq[m].y = 0.0; }
        }
      }
    } else if (BUF) {
      const int i = i0 - 2 + q % PWW, j = j0 - 2 + q / PWW;
      const bool ok = q < WN && i >= -1 && i <= b.Lm + 2 && j <= b.Mm + 2;
      const unsigned vq = ok ? (unsigned)IJ(b, i, j) * 8u : kBufOff, sk = (unsigned)kk * 8u;
      wz[m].x = BufF64(F.z_r).ld(vq, sk);
      wr[m].x = BufF64(R1).ld(vq, sk);
      if (split) wq[m].x = BufF64(F.qp1).ld(vq, sk);
    } else if (q < WN) {
      const int i = i0 - 2 + q % PWW, j = j0 - 2 + q / PWW;
      if (i >= -1 && i <= b.Lm + 2 && j <= b.Mm + 2) {
        const long o = IJ(b, i, j) + kk;
        wz[m].x = F.z_r[o];
        wr[m].x = R1[o];
        if (split) wq[m].x = F.qp1[o];
      }
    }
  }
  double mk[PQ];   // u-/v-mask of the entry's clamped point
  int e1[PQ], e0[PQ];
  bool eon[PQ];
#pragma unroll
  for (int m = 0; m < PQ; m++) {
    const int q = tid + m * NT;
    mk[m] = 0.0; e1[m] = e0[m] = 0; eon[m] = false;
    if (q < XN) {
      const int j = j0 + q / kPXW;
      int mm = i0 - 1 + q % kPXW;
      if (!(j > b.Mm + 1 || mm > b.Lm + 2 || mm < -1)) {
        mm = iclamp(mm, imin, imax);
        eon[m] = true; e1[m] = W(mm, j); e0[m] = W(mm - 1, j);
        mk[m] = F.umask[IJ(b, mm, j)];
      }
    } else if (q < XN + YN) {
      const int qq = q - XN;
      const int i = i0 + qq % kBX;
      int mm = j0 - 1 + qq / kBX;
      if (!(i > b.Lm + 1 || i < -1 || mm > b.Mm + 2)) {
        mm = iclamp(mm, jmin, jmax);
        eon[m] = true; e1[m] = W(i, mm); e0[m] = W(i, mm - 1);
        mk[m] = F.vmask[IJ(b, i, mm)];
      }
    }
  }
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool inr = i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, inr ? i : R.i0, inr ? j : R.j0), o = ij + kk;
  const bool du = inr && i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend;
  const bool dv = inr && i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend;
  double hz0 = 0, hzu = 0, hzv = 0, P0 = 0, Pu = 0, Pv = 0, dnu = 0, dmv = 0;
  if (du || dv) { hz0 = F.Hz[o]; P0 = F.P[o]; }
  if (du) { hzu = F.Hz[o - 1]; Pu = F.P[o - 1]; dnu = F.dn_u[ij]; }
  if (dv) { hzv = F.Hz[o - sj]; Pv = F.P[o - sj]; dmv = F.dm_v[ij]; }
  // FUSE: the horizontal momentum r.h.s. of the same cell (k_uv_horiz1's
  // window of u, v, FlxU, FlxV at nrhs and its lane inputs), loaded here
  // with everything else; ru/rv then go to HBM once, after both terms
  constexpr int UW = UWN, UR0 = (UW + NT - 1) / (NT), UP = UW / 2, URP = (UP + NT - 1) / NT;
  constexpr int UR = L16 ? URP : UR0;
  double2 wU[FUSE ? UR : 1], wV[FUSE ? UR : 1], wFU[FUSE ? UR : 1], wFV[FUSE ? UR : 1];
  double fo0 = 0.0, fox = 0.0, foy = 0.0;
  if constexpr (FUSE) {
    const long kn = kk + (long)(nrhs - 1) * b.n3;
#pragma unroll
    for (int r = 0; r < UR; r++) {
      const int q = tid + r * NT;
      if (L16) {   // pairs (ii, ii+1), ii = i0-2+2c, of the kUVW-wide rows
        const int ii = i0 - 2 + 2 * (q % (kUVW / 2)), jj = j0 - 2 + q / (kUVW / 2);
        const bool ok = q < UP && ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2;
        const bool hi = ii + 1 <= b.Lm + 2;
        const long oo = ok ? IJ(b, ii, jj) : 0;
        const double2 z2{0.0, 0.0};
        wU[r] = ok ? *reinterpret_cast<const double2*>(F.u + oo + kn) : z2;
        wV[r] = ok ? *reinterpret_cast<const double2*>(F.v + oo + kn) : z2;
        wFU[r] = ok ? *reinterpret_cast<const double2*>(F.FlxU + oo + kk) : z2;
        wFV[r] = ok ? *reinterpret_cast<const double2*>(F.FlxV + oo + kk) : z2;
        if (!hi) { wU[r].y = 0.0; wV[r].y = 0.0; wFU[r].y = 0.0; wFV[r].y = 0.0; }
      } else if (BUF) {
        const int ii = i0 - 2 + q % kUVW, jj = j0 - 2 + q / kUVW;
        const bool ok = q < UW && ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2;
        const unsigned vq = ok ? (unsigned)IJ(b, ii, jj) * 8u : kBufOff, sk = (unsigned)kk * 8u;
        wU[r].x = BufF64(F.u + (long)(nrhs - 1) * b.n3).ld(vq, sk);
        wV[r].x = BufF64(F.v + (long)(nrhs - 1) * b.n3).ld(vq, sk);
        wFU[r].x = BufF64(F.FlxU).ld(vq, sk);
        wFV[r].x = BufF64(F.FlxV).ld(vq, sk);
      } else {
        const int ii = i0 - 2 + q % kUVW, jj = j0 - 2 + q / kUVW;
        const bool ok = q < UW && ii >= -1 && ii <= b.Lm + 2 && jj >= -1 && jj <= b.Mm + 2;
        const long oo = ok ? IJ(b, ii, jj) : 0;
        wU[r].x = ok ? F.u[oo + kn] : 0.0;
        wV[r].x = ok ? F.v[oo + kn] : 0.0;
        wFU[r].x = ok ? F.FlxU[oo + kk] : 0.0;
        wFV[r].x = ok ? F.FlxV[oo + kk] : 0.0;
      }
    }
    if (d.p.uv_cor && (du || dv)) {
      fo0 = F.fomn[ij]; fox = F.fomn[ij - 1]; foy = F.fomn[ij - sj];
      if (!du) hzu = F.Hz[o - 1];
      if (!dv) hzv = F.Hz[o - sj];
    }
  }
#pragma unroll
  for (int m = 0; m < WL; m++) {
    const int q = tid + m * NT;
    if (L16) {
      if (q < WP) {
        *reinterpret_cast<double2*>(sZ + 2 * q) = wz[m];
        *reinterpret_cast<double2*>(sR + 2 * q) = wr[m];
        *reinterpret_cast<double2*>(sQ + 2 * q) = wq[m];
      }
    } else if (q < WN) {
      sZ[q] = wz[m].x; sR[q] = wr[m].x; sQ[q] = wq[m].x;
    }
  }
  __syncthreads();
  // ---- elementary differences at clamped u-points (xi) and v-points (eta) ----
#pragma unroll
  for (int m = 0; m < PQ; m++) {
    const int q = tid + m * NT;
    if (q >= XN + YN) continue;
    double fc = 0.0, rx = 0.0;
    if (eon[m]) {
      const double z1 = sZ[e1[m]], z0 = sZ[e0[m]];
      fc = (z1 - z0) * mk[m];
      if (split) {
        const double dpth = -0.5 * (z1 + z0);
        rx = (sR[e1[m]] - sR[e0[m]] + (sQ[e1[m]] - sQ[e0[m]]) * dpth * (1.0 - qp2 * dpth)) * mk[m];
      } else {
        rx = (sR[e1[m]] - sR[e0[m]]) * mk[m];
      }
    }
    if (q < XN) { sFCx[q] = fc; sRx[q] = rx; }
    else { sFCy[q - XN] = fc; sRy[q - XN] = rx; }
  }
  __syncthreads();
  // ---- harmonic averages at rho points p = i-1, i (xi) and j-1, j (eta) ----
#pragma unroll
  for (int m = 0; m < PQ; m++) {
    const int q = tid + m * NT;
    if (q >= XN + YN) continue;
    if (q < XN) {
      const int li = q % kPXW;
      if (li == kPXW - 1) continue;
      const int jj = j0 + q / kPXW, p = i0 - 1 + li;
      double dz = harm(sFCx[q], sFCx[q + 1]), dr = harm(sRx[q], sRx[q + 1]);
      if (split && jj <= b.Mm + 1 && p <= b.Lm + 1) {
        const int w = W(p, jj);
        dr = dr - sQ[w] * dz * (1.0 + 2.0 * qp2 * sZ[w]);
      }
      sdZx[q] = dz;
      sdRx[q] = dr;
    } else {
      const int qq = q - XN;
      const int lj = qq / kBX;
      if (lj == YH - 1) continue;
      const int ii = i0 + qq % kBX, p = j0 - 1 + lj;
      double dz = harm(sFCy[qq], sFCy[qq + kBX]), dr = harm(sRy[qq], sRy[qq + kBX]);
      if (split && ii <= b.Lm + 1 && p <= b.Mm + 1) {
        const int w = W(ii, p);
        dr = dr - sQ[w] * dz * (1.0 + 2.0 * qp2 * sZ[w]);
      }
      sdZy[qq] = dz;
      sdRy[qq] = dr;
    }
  }
  __syncthreads();
  // in-situ density (k_prsgrd_P's rhos: rho1 + qp1*dpth*(1 - qp2*dpth), dpth = -z_r)
  auto rhov = [&](int w) {
    if (split) {
      const double dpth = -sZ[w];
      return sR[w] + sQ[w] * dpth * (1.0 - qp2 * dpth);
    }
    return sR[w];
  };
  const int wc = W(inr ? i : i0, inr ? j : j0);
  double pru = 0.0, prv = 0.0;   // the pressure-gradient terms
  if (du) {
    const int q = threadIdx.x + threadIdx.y * kPXW;   // p = i-1 ; q+1: p = i
    const double dZ0 = sdZx[q], dZ1 = sdZx[q + 1], dR0 = sdRx[q], dR1 = sdRx[q + 1];
    const double z0 = sZ[wc], zu = sZ[wc - 1], r0 = rhov(wc), ru_ = rhov(wc - 1);
    pru = 0.5 * (hz0 + hzu) * dnu *
              (Pu - P0 -
               HalfGRho * ((r0 + ru_) * (z0 - zu) -
                           OneFifth * ((dR1 - dR0) * (z0 - zu - OneTwelfth * (dZ1 + dZ0)) -
                                       (dZ1 - dZ0) * (r0 - ru_ - OneTwelfth * (dR1 + dR0)))));
  }
  if (dv) {
    const int q = threadIdx.x + threadIdx.y * kBX;    // p = j-1 ; q+kBX: p = j
    const double dZ0 = sdZy[q], dZ1 = sdZy[q + kBX], dR0 = sdRy[q], dR1 = sdRy[q + kBX];
    const double z0 = sZ[wc], zv = sZ[wc - PWW], r0 = rhov(wc), rv_ = rhov(wc - PWW);
    prv = 0.5 * (hz0 + hzv) * dmv *
              (Pv - P0 -
               HalfGRho * ((r0 + rv_) * (z0 - zv) -
                           OneFifth * ((dR1 - dR0) * (z0 - zv - OneTwelfth * (dZ1 + dZ0)) -
                                       (dZ1 - dZ0) * (r0 - rv_ - OneTwelfth * (dR1 + dR0)))));
  }
  if constexpr (!FUSE) {
    if (du) F.ru[o] = pru;
    if (dv) F.rv[o] = prv;
  } else {
    // the window of u, v, FlxU, FlxV into the LDS of the finished stages
    __syncthreads();
    double* sU = sL;            // the finished stages' LDS, reused
    double* sV = sU + UWN;
    double* sFU = sV + UWN;
    double* sFV = sFU + UWN;
    static_assert(4 * UWN <= kPL, "uv window fits");
#pragma unroll
    for (int r = 0; r < UR; r++) {
      const int q = tid + r * NT;
      if (L16) {
        if (q < UP) {
          *reinterpret_cast<double2*>(sU + 2 * q) = wU[r];
          *reinterpret_cast<double2*>(sV + 2 * q) = wV[r];
          *reinterpret_cast<double2*>(sFU + 2 * q) = wFU[r];
          *reinterpret_cast<double2*>(sFV + 2 * q) = wFV[r];
        }
      } else if (q < UW) {
        sU[q] = wU[r].x; sV[q] = wV[r].x; sFU[q] = wFU[r].x; sFV[q] = wFV[r].x;
      }
    }
    __syncthreads();
    if (!(du || dv)) return;
    UVPre pp;
    pp.ru = pru; pp.rv = prv;
    pp.hz0 = hz0; pp.hzx = hzu; pp.hzy = hzv;
    pp.f0 = fo0; pp.fx = fox; pp.fy = foy;
    const AccL a{sU, sV, sFU, sFV, i0 - 2, j0 - 2};
    uv_horiz_rhs_pre(d, a, i, j, o, pp, ub, up != 0);
  }
}


// ---- fused form: one block per 64x4 tile walks the levels top-down.  Its
// 325 "P columns" (the tile plus one column to the west and one row to the
// south, where ru/rv read P and the in-situ density) run the vertical
// recurrences of k_prsgrd_P in registers.  The level-k slice of z_r, rho1
// (rho) and qp1 over the tile's stencil window (i0-2..i0+64 x j0-2..j0+4)
// sits in LDS, three levels deep (k and k-1 for the recurrences, k-2 being
// stored), fed from registers loaded two levels earlier.  Each tile lane then
// forms the three clamped elementary differences per direction it needs,
// their harmonic means and ru, rv, with the expressions of k_prsgrd_uv.  P
// and the in-situ density never leave the CU, z_r / rho1 / qp1 are read from
// HBM once per cell (window halo re-reads hit the neighbouring tiles' lines
// in L2), two barriers per level.  Bit-identical to the two-kernel form. ----
constexpr int kFW = kBX + 3, kFH = kBY + 3, kFN = kFW * kFH;   // window (i0-2..i0+64) x (j0-2..j0+4)
constexpr int kFPW = kBX + 1, kFPH = kBY + 1, kFPN = kFPW * kFPH;   // P columns (i0-1..i0+63) x (j0-1..j0+3)
constexpr int kFT = 384;                                         // threads: 6 wavefronts >= kFPN
constexpr int kFQ = (kFN + kFT - 1) / kFT;                       // window entries per thread
struct PrsWin {
  double z[3][kFN], r[3][kFN], q[3][kFN];
  double P[kFPN], V[kFPN];   // P and in-situ density of the P columns at level k
};
struct PrsPre {              // one level of this thread's window entries, in flight
  double z[kFQ], r[kFQ], q[kFQ];
};
__global__ void __launch_bounds__(kFT) k_prsgrd_fused(Dev d, Range R, int split, int imin, int imax, int jmin,
                                                       int jmax, int tides) {
  const uint3 bI = xcd_tile();
  __shared__ PrsWin W;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const int N = b.N;
  const double g = d.p.g, rho0 = d.p.rho0, qp2 = d.p.qp2;
  const double OneFifth = 0.2, OneTwelfth = 1.0 / 12.0;
  const double grho = g / rho0, HalfGRho = 0.5 * grho;
  const long n2 = b.n2, sj = b.nx2;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int tid = threadIdx.x;
  const double* R1 = split ? F.rho1 : F.rho;
  // window entries owned by this thread
  long wo[kFQ];
  bool won[kFQ];
#pragma unroll
  for (int m = 0; m < kFQ; m++) {
    const int e = tid + m * kFT;
    const int i = i0 - 2 + e % kFW, j = j0 - 2 + e / kFW;
    won[m] = e < kFN && i >= -1 && i <= b.Lm + 2 && j <= b.Mm + 2;
    wo[m] = IJ(b, i, j);
  }
  auto load = [&](int k, PrsPre& X) {
    if (k < 1) return;
    const long kk = (long)(k - 1) * n2;
#pragma unroll
    for (int m = 0; m < kFQ; m++) {
      X.z[m] = X.r[m] = X.q[m] = 0.0;
      if (won[m]) {
        X.z[m] = F.z_r[wo[m] + kk];
        X.r[m] = R1[wo[m] + kk];
        if (split) X.q[m] = F.qp1[wo[m] + kk];
      }
    }
  };
  auto store = [&](int k, const PrsPre& X) {
    if (k < 1) return;
    const int sl = k % 3;
#pragma unroll
    for (int m = 0; m < kFQ; m++) {
      const int e = tid + m * kFT;
      if (e < kFN) { W.z[sl][e] = X.z[m]; W.r[sl][e] = X.r[m]; W.q[sl][e] = X.q[m]; }
    }
  };
  // P column of this thread
  const bool pcol = tid < kFPN;
  const int pci = tid % kFPW, pcj = tid / kFPW;
  const int pi = i0 - 1 + pci, pj = j0 - 1 + pcj;
  const bool pon = pcol && pi >= -1 && pi <= b.Lm + 1 && pj <= b.Mm + 1;
  const int pw = (pci + 1) + (pcj + 1) * kFW;   // its window position
  const long pij = IJ(b, pi, pj);
  auto rhov = [&](double r1, double q1, double z) {
    if (split) {
      const double dpth = -z;
      return r1 + q1 * dpth * (1.0 - qp2 * dpth);
    }
    return r1;
  };
  auto eRof = [&](double ru, double rl, double qu, double ql, double zu, double zl) {
    if (split) {
      const double dpth = -0.5 * (zu + zl);
      return ru - rl + (qu - ql) * dpth * (1.0 - qp2 * dpth);
    }
    return ru - rl;
  };
  // tile lane: clamped u-/v-point window offsets and masks (level independent)
  const int ti = tid % kBX, tj = tid / kBX;
  const int i = i0 + ti, j = j0 + tj;
  const bool tile = tid < kBX * kBY && i >= R.i0 && i <= R.i1 && j <= R.j1;
  const long ij = IJ(b, i, j);
  const bool du = tile && i >= b.istrU && i <= b.iend && j >= b.jstr && j <= b.jend;
  const bool dv = tile && i >= b.istr && i <= b.iend && j >= b.jstrV && j <= b.jend;
  const int wc = (ti + 2) + (tj + 2) * kFW;   // window (i, j)
  const int pc = (ti + 1) + (tj + 1) * kFPW;  // P column (i, j)
  int wux[3], wvy[3];                         // window of the clamped u-points i-1..i+1 / v-points j-1..j+1
  double umx[3], vmy[3], dnu = 0.0, dmv = 0.0;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    wux[c] = wvy[c] = wc;
    umx[c] = vmy[c] = 0.0;
    if (du) {
      const int m = iclamp(i - 1 + c, imin, imax);
      wux[c] = (m - i0 + 2) + (tj + 2) * kFW;
      umx[c] = F.umask[IJ(b, m, j)];
    }
    if (dv) {
      const int m = iclamp(j - 1 + c, jmin, jmax);
      wvy[c] = (ti + 2) + (m - j0 + 2) * kFW;
      vmy[c] = F.vmask[IJ(b, i, m)];
    }
  }
  if (du) dnu = F.dn_u[ij];
  if (dv) dmv = F.dm_v[ij];
  // prologue: levels N and N-1 in LDS, N-2 and N-3 in flight
  {
    PrsPre X;
    load(N, X); store(N, X);
    load(N - 1, X); store(N - 1, X);
  }
  PrsPre A, B;
  load(N - 2, A);
  load(N - 3, B);
  __syncthreads();
  double eZk = 0.0, eRk = 0.0, dZ1 = 0.0, dR1 = 0.0, P1 = 0.0, z1 = 0.0, v1 = 0.0;
  if (pon) {
    const int sN = N % 3, sM = (N - 1) % 3;
    eZk = W.z[sN][pw] - W.z[sM][pw];
    eRk = eRof(W.r[sN][pw], W.r[sM][pw], W.q[sN][pw], W.q[sM][pw], W.z[sN][pw], W.z[sM][pw]);
  }
  auto level = [&](int k, PrsPre& X) {   // X holds level k-2 on entry, k-4 on exit
    const int sk = k % 3, sm = (k + 2) % 3;
    const long o = ij + (long)(k - 1) * n2;
    double hz0 = 0.0, hzu = 0.0, hzv = 0.0;
    if (du) { hz0 = F.Hz[o]; hzu = F.Hz[o - 1]; }
    if (dv) { hz0 = F.Hz[o]; hzv = F.Hz[o - sj]; }
    // (1) P columns: vertical harmonic means and the hydrostatic integral
    if (pon) {
      const double zC = W.z[sk][pw], rC = W.r[sk][pw], qC = W.q[sk][pw];
      double eZm, eRm;
      if (k >= 2) {
        const double zM = W.z[sm][pw], rM = W.r[sm][pw], qM = W.q[sm][pw];
        eZm = zC - zM;
        eRm = eRof(rC, rM, qC, qM, zC, zM);
      } else {
        eZm = eZk; eRm = eRk;
      }
      const double dZk = [&] { const double c = 2.0 * eZk * eZm; return c / (eZk + eZm); }();
      double dRk = harm(eRk, eRm);
      const double v0 = rhov(rC, qC, zC);
      if (split) {
        const double dpth = -zC;
        dRk = dRk - qC * dZk * (1.0 - 2.0 * qp2 * dpth);
      }
      double Pk;
      if (k == N) {
        const double zw = F.z_w[pij + (long)N * n2];
        const double zM = W.z[sm][pw];
        const double rNm = rhov(W.r[sm][pw], W.q[sm][pw], zM);
        Pk = g * zw + grho * (v0 + 0.5 * (v0 - rNm) * (zw - zC) / (zC - zM)) * (zw - zC);
        if (tides) Pk = Pk - g * F.ptide[pij];   // TIDES: pot_tides (prsgrd.F:209-211)
      } else {
        Pk = P1 + HalfGRho * ((v1 + v0) * (z1 - zC) -
                              OneFifth * ((dR1 - dRk) * (z1 - zC - OneTwelfth * (dZ1 + dZk)) -
                                          (dZ1 - dZk) * (v1 - v0 - OneTwelfth * (dR1 + dRk))));
      }
      W.P[tid] = Pk;
      W.V[tid] = v0;
      P1 = Pk;
      dZ1 = dZk; dR1 = dRk;
      eZk = eZm; eRk = eRm;
      z1 = zC; v1 = v0;
    }
    __syncthreads();
    // (2) ru, rv of the tile: clamped elementary differences at the three
    // u-points (v-points), harmonic means at p = i-1, i (j-1, j), then the
    // density-Jacobian pressure gradient (k_prsgrd_uv expressions)
    const double* Z = W.z[sk];
    const double* Rr = W.r[sk];
    const double* Qq = W.q[sk];
    auto diffs = [&](const int (&w)[3], const double (&mk)[3], int st, double (&fc)[3], double (&rx)[3]) {
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int w1 = w[c], w0 = w1 - st;
        fc[c] = (Z[w1] - Z[w0]) * mk[c];
        if (split) {
          const double dpth = -0.5 * (Z[w1] + Z[w0]);
          rx[c] = (Rr[w1] - Rr[w0] + (Qq[w1] - Qq[w0]) * dpth * (1.0 - qp2 * dpth)) * mk[c];
        } else {
          rx[c] = (Rr[w1] - Rr[w0]) * mk[c];
        }
      }
    };
    auto means = [&](const double (&fc)[3], const double (&rx)[3], int wp0, int wp1, double& dZ0, double& dZ1o,
                     double& dR0, double& dR1o) {
      dZ0 = harm(fc[0], fc[1]); dR0 = harm(rx[0], rx[1]);
      dZ1o = harm(fc[1], fc[2]); dR1o = harm(rx[1], rx[2]);
      if (split) {
        dR0 = dR0 - Qq[wp0] * dZ0 * (1.0 + 2.0 * qp2 * Z[wp0]);
        dR1o = dR1o - Qq[wp1] * dZ1o * (1.0 + 2.0 * qp2 * Z[wp1]);
      }
    };
    if (du) {
      double fc[3], rx[3], dZ0, dZ1x, dR0, dR1x;
      diffs(wux, umx, 1, fc, rx);
      means(fc, rx, wc - 1, wc, dZ0, dZ1x, dR0, dR1x);
      const double zr0 = Z[wc], zrm = Z[wc - 1], r0 = W.V[pc], rm = W.V[pc - 1];
      F.ru[o] = 0.5 * (hz0 + hzu) * dnu *
                (W.P[pc - 1] - W.P[pc] -
                 HalfGRho * ((r0 + rm) * (zr0 - zrm) -
                             OneFifth * ((dR1x - dR0) * (zr0 - zrm - OneTwelfth * (dZ1x + dZ0)) -
                                         (dZ1x - dZ0) * (r0 - rm - OneTwelfth * (dR1x + dR0)))));
    }
    if (dv) {
      double fc[3], rx[3], dZ0, dZ1y, dR0, dR1y;
      diffs(wvy, vmy, kFW, fc, rx);
      means(fc, rx, wc - kFW, wc, dZ0, dZ1y, dR0, dR1y);
      const double zr0 = Z[wc], zrm = Z[wc - kFW], r0 = W.V[pc], rm = W.V[pc - kFPW];
      F.rv[o] = 0.5 * (hz0 + hzv) * dmv *
                (W.P[pc - kFPW] - W.P[pc] -
                 HalfGRho * ((r0 + rm) * (zr0 - zrm) -
                             OneFifth * ((dR1y - dR0) * (zr0 - zrm - OneTwelfth * (dZ1y + dZ0)) -
                                         (dZ1y - dZ0) * (r0 - rm - OneTwelfth * (dR1y + dR0)))));
    }
    // (3) level k-2 into the slot of k+1 (free), then the loads of k-4
    store(k - 2, X);
    load(k - 4, X);
    __syncthreads();
  };
  for (int k = N; k >= 1; k -= 2) {
    level(k, A);
    if (k - 1 >= 1) level(k - 1, B);
  }
}

// prsgrd's hydrostatic pressure P alone (the two-kernel form's first kernel)
void launch_prsgrd_P(const Dev& d, hipStream_t s) {
  const Bounds& b = d.b;
  Range R1{0, b.Lm, 0, b.Mm};
  hipLaunchKernelGGL(k_prsgrd_P, grid_of(R1), dim3(kBX, kBY), 0, s, d, R1, d.p.nonlin_eos, d.p.tides);
}
void launch_prsgrd(const Dev& d, hipStream_t s, const Tlev& t, int uv_up, bool p_ready) {
  const Bounds& b = d.b;
  if (d.p.iso && t.nrhs == 3) launch_iso_slopes(d, s);   // ADV_ISONEUTRAL, CORR_STAGE (prsgrd.F:307-338)
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
  Range R2{b.istr, b.iend, b.jstr, b.jend};
  if (!d.p.prs_split) {
    hipLaunchKernelGGL(k_prsgrd_fused, grid_of(R2), dim3(kFT), 0, s, d, R2, split, imin, imax, jmin, jmax, d.p.tides);
    return;
  }
  // two-kernel form (default; k_prsgrd_fused with ROMS_GPU_PRSGRD_FUSED=1)
  Range R1{0, b.Lm, 0, b.Mm};
  if (!p_ready) hipLaunchKernelGGL(k_prsgrd_P, grid_of(R1), dim3(kBX, kBY), 0, s, d, R1, split, d.p.tides);
  ktimer_mark(s, kTimedPrsgrdUv, 0);
  auto tiles = [&](const Range& R) {   // k_prsgrd_uv over R (the variant Params selects)
    if (uv_up >= 0 && d.p.ld16 && d.p.prs_ty != 8)
      hipLaunchKernelGGL((k_prsgrd_uv<true, kBY, true>), grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, split, imin, imax,
                         jmin, jmax, uv_bounds(b), uv_up, t.nrhs);
    else if (!(uv_up >= 0) && d.p.ld16 && d.p.prs_ty != 8)
      hipLaunchKernelGGL((k_prsgrd_uv<false, kBY, true>), grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, split, imin,
                         imax, jmin, jmax, uv_bounds(b), 0, t.nrhs);
    else if (uv_up >= 0 && d.p.prs_ty == 8)
      hipLaunchKernelGGL((k_prsgrd_uv<true, 8>), grid3_ty(R, b.N, 8), dim3(kBX, 8), 0, s, d, R, split, imin, imax, jmin,
                         jmax, uv_bounds(b), uv_up, t.nrhs);
    else if (uv_up >= 0 && d.p.prs_buf)
      hipLaunchKernelGGL((k_prsgrd_uv<true, kBY, false, true>), grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, split, imin,
                         imax, jmin, jmax, uv_bounds(b), uv_up, t.nrhs);
    else if (uv_up >= 0)
      hipLaunchKernelGGL(k_prsgrd_uv<true>, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, split, imin, imax, jmin, jmax,
                         uv_bounds(b), uv_up, t.nrhs);
    else if (d.p.prs_ty == 8)
      hipLaunchKernelGGL((k_prsgrd_uv<false, 8>), grid3_ty(R, b.N, 8), dim3(kBX, 8), 0, s, d, R, split, imin, imax, jmin,
                         jmax, uv_bounds(b), 0, t.nrhs);
    else
      hipLaunchKernelGGL(k_prsgrd_uv<false>, grid3_of(R, b.N), dim3(kBX, kBY), 0, s, d, R, split, imin, imax, jmin, jmax,
                         uv_bounds(b), 0, t.nrhs);
  };
  // with the momentum r.h.s. (whole steps): rows jA..jB in j-marching strips
  // (k_prsgrd_strip.hip), the bands of rows a closed-edge j-extrapolation
  // reaches in k_prsgrd_uv tiles; ROMS_GPU_PRS_STRIP=0: tiles everywhere
  int jA = 0, jB = -1;
  if (uv_up >= 0 && d.p.prs_strip && d.p.uv_cor && d.p.uv_adv && !d.p.curvgrid &&
      launch_prsgrd_strip(d, s, t.nrhs, uv_up, imin, imax, jmin, jmax, uv_bounds(b), jA, jB)) {
    if (jA > R2.j0) tiles(Range{R2.i0, R2.i1, R2.j0, jA - 1});
    if (jB < R2.j1) tiles(Range{R2.i0, R2.i1, jB + 1, R2.j1});
  } else {
    tiles(R2);
  }
  ktimer_mark(s, kTimedPrsgrdUv, 1, 1);
}
// k_prsgrd_uv<true> adds the horizontal momentum r.h.s. of k_uv_horiz1 on
// the same inputs: usable when the caller runs uv_horiz next with nothing
// between them that changes u, v(nrhs), FlxU, FlxV, Hz or ru, rv
bool prsgrd_can_fuse_uv(const Dev& d) {
  return d.p.prs_split && d.p.hoist && d.p.prs_fuse_uv && !d.p.curvgrid && (d.p.uv_cor || d.p.uv_adv);
}

}  // namespace roms
