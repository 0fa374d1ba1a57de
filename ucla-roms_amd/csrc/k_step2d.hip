// k_step2d.hip -- step2d_FB_tile (step2d_FB.F:24-576): one generalized
// forward-backward AB3-AM4 barotropic step with fast-time averaging and the
// 3-D -> 2-D coupling at the first fast step.
//
// Kernel A (zeta range istrU-1..iend x jstrV-1..jend): free surface zeta_new,
// Dnew and the backward-averaged zwrk/rzeta/rzeta2/rzetaSA into 2-D scratch;
// the extrapolated fluxes DUon/DVom are rebuilt per lane from Drhs.
// Kernel B (istrR..iendR x jstrR..jendR): zeta(knew), fast averages,
// pressure-gradient rubar/rvbar (+ PGF_FB correction at iif=1) and the
// momentum update ubar/vbar(knew), DU_avg1/DV_avg1.
// Kernel C (closed edges only): u2dbc/v2dbc and the boundary flux averages.
#include "roms_dev.h"
#include "halo.h"

namespace roms {

struct FBCoef {
  int kstp, kbak, kold, knew, iif, nfast;
  double fwd, fwd1, fwd2, bkw_new, bkw, bkw1, bkw2;
  double w1, w2;  // weight(1,iif), weight(2,iif)
};

__device__ __forceinline__ double s2d_Drhs(const Dev& d, const FBCoef& c, long ij) {
  const Fields& F = d.f;
  const long n2 = d.b.n2;
  return F.h[ij] + c.fwd * F.zeta[ij + (long)(c.kstp - 1) * n2] + c.fwd1 * F.zeta[ij + (long)(c.kbak - 1) * n2] +
         c.fwd2 * F.zeta[ij + (long)(c.kold - 1) * n2];
}
__device__ __forceinline__ double s2d_DUon(const Dev& d, const FBCoef& c, long ij) {
  const Fields& F = d.f;
  const long n2 = d.b.n2;
  const double urhs = c.fwd * F.ubar[ij + (long)(c.kstp - 1) * n2] + c.fwd1 * F.ubar[ij + (long)(c.kbak - 1) * n2] +
                      c.fwd2 * F.ubar[ij + (long)(c.kold - 1) * n2];
  return 0.5 * (s2d_Drhs(d, c, ij) + s2d_Drhs(d, c, ij - 1)) * F.dn_u[ij] * (urhs);
}
__device__ __forceinline__ double s2d_DVom(const Dev& d, const FBCoef& c, long ij) {
  const Fields& F = d.f;
  const long n2 = d.b.n2, sj = d.b.nx2;
  const double vrhs = c.fwd * F.vbar[ij + (long)(c.kstp - 1) * n2] + c.fwd1 * F.vbar[ij + (long)(c.kbak - 1) * n2] +
                      c.fwd2 * F.vbar[ij + (long)(c.kold - 1) * n2];
  return 0.5 * (s2d_Drhs(d, c, ij) + s2d_Drhs(d, c, ij - sj)) * F.dm_v[ij] * (vrhs);
}

__global__ void __launch_bounds__(256) k_s2d_zeta(Dev d, Range R, FBCoef c) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), sj = b.nx2, n2 = b.n2;
  const double zk = F.zeta[ij + (long)(c.kstp - 1) * n2];
  double zn = zk + d.p.dtfast * F.pm[ij] * F.pn[ij] *
                       (s2d_DUon(d, c, ij) - s2d_DUon(d, c, ij + 1) + s2d_DVom(d, c, ij) - s2d_DVom(d, c, ij + sj)) +
              d.p.dtfast * F.swflx[ij];
  if (d.p.npip > 0 && F.pipe_idx[ij] > 0) zn = zn + d.p.dtfast * F.pm[ij] * F.pn[ij] * F.pipe_flx[ij];  // step2d_FB.F:155-159
  zn = zn * F.rmask[ij];
  F.s0[ij] = zn;
  F.s1[ij] = zn + F.h[ij];
  const double zwrk = c.bkw_new * zn + c.bkw * zk + c.bkw1 * F.zeta[ij + (long)(c.kbak - 1) * n2] +
                      c.bkw2 * F.zeta[ij + (long)(c.kold - 1) * n2];
  const double rzeta = (1.0 + F.rhoS[ij]) * zwrk;
  F.s2[ij] = zwrk;
  F.s3[ij] = rzeta;
  F.s5[ij] = zwrk * (F.rhoS[ij] - F.rhoA[ij]);
  F.s4[ij] = rzeta * zwrk;
}

// zetabc_tile (zetabc.F:3-224): zero-gradient on closed edges, OBC_M2FLATHER
// on open ones (from zeta(kstp)), corners averaged
__global__ void k_s2d_zetabc(Dev d, int phase, int kstp) {
  const Bounds& b = d.b;
  double* zn = d.f.s0;
  const double* rm = d.f.rmask;
  const double* zk = d.f.zeta + (long)(kstp - 1) * b.n2;
  const double dtf = d.p.dtfast, g = d.p.g;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (phase == 0) {
    const int nj = b.jend - (b.jstrV - 1) + 1, ni = b.iend - (b.istrU - 1) + 1;
    if (p < nj) {
      const int j = b.jstrV - 1 + p;
      if (b.west_edge) {
        const int i = b.istr;
        if (d.p.obc & 1) {
          const double cx = dtf * d.f.pm[IJ(b, i, j)] * sqrt(g * d.f.h[IJ(b, i, j)]);
          zn[IJ(b, i - 1, j)] = ((1. - cx) * zk[IJ(b, i - 1, j)] + cx * zk[IJ(b, i, j)]) * rm[IJ(b, i - 1, j)];
        } else {
          zn[IJ(b, i - 1, j)] = zn[IJ(b, i, j)] * rm[IJ(b, i - 1, j)];
        }
      }
      if (b.east_edge) {
        const int i = b.iend;
        if (d.p.obc & 2) {
          const double cx = dtf * d.f.pm[IJ(b, i, j)] * sqrt(g * d.f.h[IJ(b, i, j)]);
          zn[IJ(b, i + 1, j)] = ((1. - cx) * zk[IJ(b, i + 1, j)] + cx * zk[IJ(b, i, j)]) * rm[IJ(b, i + 1, j)];
        } else {
          zn[IJ(b, i + 1, j)] = zn[IJ(b, i, j)] * rm[IJ(b, i + 1, j)];
        }
      }
    } else if (p < nj + ni) {
      const int i = b.istrU - 1 + p - nj;
      if (b.south_edge) {
        const int j = b.jstr;
        if (d.p.obc & 4) {
          const double cx = dtf * d.f.pn[IJ(b, i, j)] * sqrt(g * d.f.h[IJ(b, i, j)]);
          zn[IJ(b, i, j - 1)] = ((1. - cx) * zk[IJ(b, i, j - 1)] + cx * zk[IJ(b, i, j)]) * rm[IJ(b, i, j - 1)];
        } else {
          zn[IJ(b, i, j - 1)] = zn[IJ(b, i, j)] * rm[IJ(b, i, j - 1)];
        }
      }
      if (b.north_edge) {
        const int j = b.jend;
        if (d.p.obc & 8) {
          const double cx = dtf * d.f.pn[IJ(b, i, j)] * sqrt(g * d.f.h[IJ(b, i, j)]);
          zn[IJ(b, i, j + 1)] = ((1. - cx) * zk[IJ(b, i, j + 1)] + cx * zk[IJ(b, i, j)]) * rm[IJ(b, i, j + 1)];
        } else {
          zn[IJ(b, i, j + 1)] = zn[IJ(b, i, j)] * rm[IJ(b, i, j + 1)];
        }
      }
    }
  } else if (p == 0) {
    const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
    if (b.south_edge && b.west_edge) zn[IJ(b, is - 1, js - 1)] = 0.5 * (zn[IJ(b, is, js - 1)] + zn[IJ(b, is - 1, js)]);
    if (b.south_edge && b.east_edge) zn[IJ(b, ie + 1, js - 1)] = 0.5 * (zn[IJ(b, ie, js - 1)] + zn[IJ(b, ie + 1, js)]);
    if (b.north_edge && b.west_edge) zn[IJ(b, is - 1, je + 1)] = 0.5 * (zn[IJ(b, is, je + 1)] + zn[IJ(b, is - 1, je)]);
    if (b.north_edge && b.east_edge) zn[IJ(b, ie + 1, je + 1)] = 0.5 * (zn[IJ(b, ie, je + 1)] + zn[IJ(b, ie + 1, je)]);
  }
}

__device__ __forceinline__ double pgf_x(const Dev& d, long ij, long s, const double* rz, const double* rz2,
                                        const double* rzSA, const double* zw, double dn) {
  const Fields& F = d.f;
  const double cff = 0.5 * d.p.g;
  return cff * dn *
         ((F.h[ij - s] + F.h[ij]) * (rz[ij - s] - rz[ij]) + rz2[ij - s] - rz2[ij] +
          (F.h[ij - s] - F.h[ij]) * (rzSA[ij - s] + rzSA[ij] + 0.333333333333 * (F.rhoA[ij - s] - F.rhoA[ij]) * (zw[ij - s] - zw[ij])));
}
// PGF_FB correction terms at one point (iif==1)
__device__ __forceinline__ void fb_corr(const Dev& d, const FBCoef& c, long ij, double& zwrk, double& rzeta,
                                        double& rzeta2, double& rzetaSA) {
  const Fields& F = d.f;
  const double zn = F.s0[ij], zk = F.zeta[ij + (long)(c.kstp - 1) * d.b.n2];
  zwrk = zn - zk;
  rzeta = (1.0 + F.rhoS[ij]) * zwrk;
  rzeta2 = rzeta * (zn + zk);
  rzetaSA = zwrk * (F.rhoS[ij] - F.rhoA[ij]);
}

__global__ void __launch_bounds__(256) k_s2d_mom(Dev d, Range R, FBCoef c) {
  ROMS_IJ_OR_RETURN(R)
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long ij = IJ(b, i, j), sj = b.nx2, n2 = b.n2;
  const double* zn = F.s0;
  const double* Dnew = F.s1;
  const bool avg = i >= b.istrR && i <= b.iendR && j >= b.jstrR && j <= b.jendR;
  if (avg) {
    const double z = zn[ij];
    F.zeta[ij + (long)(c.knew - 1) * n2] = z;
    if (c.iif == 1) {
      F.DU_avg_bak[ij] = F.DU_avg1[ij] - 0.1024390243902439 * F.DU_avg2[ij];
      F.DV_avg_bak[ij] = F.DV_avg1[ij] - 0.1024390243902439 * F.DV_avg2[ij];
      F.Zt_avg1[ij] = c.w1 * z;
      F.DU_avg1[ij] = 0.0;
      F.DV_avg1[ij] = 0.0;
      F.DU_avg2[ij] = c.w2 * s2d_DUon(d, c, ij);
      F.DV_avg2[ij] = c.w2 * s2d_DVom(d, c, ij);
    } else {
      F.Zt_avg1[ij] = F.Zt_avg1[ij] + c.w1 * z;
      F.DU_avg2[ij] = F.DU_avg2[ij] + c.w2 * s2d_DUon(d, c, ij);
      F.DV_avg2[ij] = F.DV_avg2[ij] + c.w2 * s2d_DVom(d, c, ij);
    }
  }
  if (i < b.istr || i > b.iend || j < b.jstr || j > b.jend) return;
  double rubar = pgf_x(d, ij, 1, F.s3, F.s4, F.s5, F.s2, F.dn_u[ij]);
  double rvbar = pgf_x(d, ij, sj, F.s3, F.s4, F.s5, F.s2, F.dm_v[ij]);
  double rufrc = F.rufrc[ij], rvfrc = F.rvfrc[ij];
  if (c.iif == 1) {
    rufrc = rufrc - rubar;
    rvfrc = rvfrc - rvbar;
    F.rufrc[ij] = rufrc;
    F.rvfrc[ij] = rvfrc;
    double zw0, rz0, rz20, sa0, zw1, rz1, rz21, sa1, zw2, rz2_, rz22, sa2;
    fb_corr(d, c, ij, zw0, rz0, rz20, sa0);
    fb_corr(d, c, ij - 1, zw1, rz1, rz21, sa1);
    fb_corr(d, c, ij - sj, zw2, rz2_, rz22, sa2);
    const double cff = 0.5 * d.p.g;
    rubar = rubar + cff * F.dn_u[ij] *
                        ((F.h[ij - 1] + F.h[ij]) * (rz1 - rz0) + rz21 - rz20 +
                         (F.h[ij - 1] - F.h[ij]) * (sa1 + sa0 + 0.333333333333 * (F.rhoA[ij - 1] - F.rhoA[ij]) * (zw1 - zw0)));
    rvbar = rvbar + cff * F.dm_v[ij] *
                        ((F.h[ij - sj] + F.h[ij]) * (rz2_ - rz0) + rz22 - rz20 +
                         (F.h[ij - sj] - F.h[ij]) * (sa2 + sa0 + 0.333333333333 * (F.rhoA[ij - sj] - F.rhoA[ij]) * (zw2 - zw0)));
  }
  const double cff = 0.5 * d.p.dtfast, cff1 = 0.5 * c.w1;
  const long lk = (long)(c.kstp - 1) * n2;
  const double Dstp0 = F.zeta[ij + lk] + F.h[ij];
  if (i >= b.istrU) {
    const double Dstpm = F.zeta[ij - 1 + lk] + F.h[ij - 1];
    const double DUnew = ((Dstp0 + Dstpm) * F.ubar[ij + lk] +
                          cff * (F.pm[ij] + F.pm[ij - 1]) * (F.pn[ij] + F.pn[ij - 1]) * (rubar + rufrc)) *
                         F.umask[ij];
    F.ubar[ij + (long)(c.knew - 1) * n2] = DUnew / (Dnew[ij] + Dnew[ij - 1]);
    F.DU_avg1[ij] = F.DU_avg1[ij] + cff1 * F.dn_u[ij] * (DUnew);
  }
  if (j >= b.jstrV) {
    const double Dstpm = F.zeta[ij - sj + lk] + F.h[ij - sj];
    const double DVnew = ((Dstp0 + Dstpm) * F.vbar[ij + lk] +
                          cff * (F.pm[ij] + F.pm[ij - sj]) * (F.pn[ij] + F.pn[ij - sj]) * (rvbar + rvfrc)) *
                         F.vmask[ij];
    F.vbar[ij + (long)(c.knew - 1) * n2] = DVnew / (Dnew[ij] + Dnew[ij - sj]);
    F.DV_avg1[ij] = F.DV_avg1[ij] + cff1 * F.dm_v[ij] * (DVnew);
  }
}

// ---------------------------------------------------------------------------
// Fused fast step: one block owns a 64x4 tile of the averaging range RB and
// first evaluates the free-surface part (k_s2d_zeta's formulas) on the tile
// plus one row/column on its low side into LDS, applies the closed-wall
// zetabc to ghost cells inside that window, then runs the averaging and
// momentum part (k_s2d_mom's formulas) reading its i-1 / j-1 neighbours from
// LDS.  zeta_new/Dnew also go to global scratch when closed-edge kernels
// need them afterwards.
// ---------------------------------------------------------------------------
constexpr int kFX = kBX + 1, kFY = kBY + 1, kFN = kFX * kFY;  // zeta-part window (i0-1.., j0-1..)
constexpr int kGX = kBX + 3, kGY = kBY + 3, kGN = kGX * kGY;  // input window (i0-2.., j0-2..)
constexpr int kUX = kBX + 2, kUN = kUX * kFY;                 // DUon faces i0-1..i0+64, rows j0-1..j0+3
constexpr int kVN = kFX * (kBY + 2);                          // DVom faces i0-1..i0+63, rows j0-1..j0+4
struct FBTile {
  double z0[kGN], z1[kGN], z2[kGN], h[kGN], Dr[kGN];   // zeta(kstp,kbak,kold), h, Drhs
  double DU[kUN], DV[kVN];                              // DUon, DVom
  double zn[kFN], Dn[kFN], zw[kFN], rz[kFN], rz2[kFN], rzSA[kFN];
  unsigned char st[kFN];  // 0: outside, 1: computed, 2: set by zetabc
};

// kClosed: 0 no closed edge, 1 closed edges finished by k_s2d_edges, 2 closed
// walls folded in; kWrap: single-rank periodic images (vwrap bits).  Compile-
// time switches, so each instance carries only its own branches.
// How the fast step's results are stored.  1 (default): write-through
// (sc1, an agent-scope relaxed atomic store): the lines go on to memory while
// the kernel runs instead of sitting dirty in the XCDs' L2s until the end of
// the dispatch, whose write-back the next fast step would wait for -- 16.8 MB
// per C2 launch; -10% per fast step at C2 and C3 (profiles/r4_y_s2d_store_ab.txt).
// 0 plain stores, 2 nontemporal (no gain); ROMS_GPU_S2D_WT selects for A/B.
// (Write-through in the long 3-D kernels measured neutral at C2 and 1 ms/step
// slower at C3, so they keep plain stores.)
template <int WT>
__device__ __forceinline__ void gst(double* p, double v) {
  if constexpr (WT == 1)
    __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (WT == 2)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
#ifdef ROMS_S2D_PROBE
// Timing probe (A/B builds only, tools/s2d_phase_probe.py): thread 0 of each
// block stores the shader clock at the phase boundaries into
// ptide[block*8 + phase] (ptide is unused without TIDES)
#define S2D_T(ph) do { if (threadIdx.x == 0 && threadIdx.y == 0) { \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    d.f.ptide[(long)(blockIdx.x + gridDim.x * blockIdx.y) * 8 + (ph)] = (double)t_; } } while (0)
#else
#define S2D_T(ph) do { } while (0)
#endif
// kWin: the 2-D fields through the buffer window d.w2 (S2dWin, roms_dev.h),
// else through the pointers of Fields; the same loads and stores either way.
template <bool kPipe, int kClosed, bool kWrap, int kWT = 1, bool kWin = false>
__global__ void __launch_bounds__(256) k_s2d_fb(Dev d, Range R, FBCoef c, int vwrap, int part) {
  constexpr int closed = kClosed;
  const uint3 bI = xcd_tile();
  S2D_T(0);
  const Fields& Fp = d.f;
  auto fp = [&](int f) -> double* {
    switch (f) {
      case kW_zeta: return Fp.zeta; case kW_ubar: return Fp.ubar; case kW_vbar: return Fp.vbar; case kW_h: return Fp.h;
      case kW_dn_u: return Fp.dn_u; case kW_dm_v: return Fp.dm_v; case kW_pm: return Fp.pm; case kW_pn: return Fp.pn;
      case kW_swflx: return Fp.swflx; case kW_rmask: return Fp.rmask; case kW_rhoS: return Fp.rhoS;
      case kW_rhoA: return Fp.rhoA; case kW_umask: return Fp.umask; case kW_vmask: return Fp.vmask;
      case kW_rufrc: return Fp.rufrc; case kW_rvfrc: return Fp.rvfrc; case kW_DU_avg1: return Fp.DU_avg1;
      case kW_DV_avg1: return Fp.DV_avg1; case kW_DU_avg2: return Fp.DU_avg2; case kW_DV_avg2: return Fp.DV_avg2;
      case kW_Zt_avg1: return Fp.Zt_avg1; case kW_DU_avg_bak: return Fp.DU_avg_bak;
      case kW_DV_avg_bak: return Fp.DV_avg_bak; case kW_s0: return Fp.s0; default: return Fp.s1;
    }
  };
  // element idx (+ a uniform slot offset sl) of field f; in the window the
  // lane's part is the VGPR offset, the field's origin and the slot the SGPR one
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(d.w2.base), (short)0, 0x7fffffff, 0x00020000);
  auto LD = [&](int f, long idx, long sl = 0) -> double {
    if constexpr (kWin)
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                            wrs, (int)((unsigned)(idx + sl + d.w2.lead) * 8u),
                                            (int)d.w2.off[f], 0));
    else
      return fp(f)[idx + sl];
  };
  auto ST = [&](int f, long idx, double v, long sl = 0) {
    if constexpr (kWin)   // cache policy of gst<kWT>: 16 = sc1 (write-through), 2 = nt
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) int, v), wrs,
                                            (int)((unsigned)(idx + sl + d.w2.lead) * 8u),
                                            (int)d.w2.off[f],
                                            kWT == 1 ? 16 : (kWT == 2 ? 2 : 0));
    else
      gst<kWT>(&fp(f)[idx + sl], v);
  };
  // part 1: interior tiles only (their windows hold no halo cell), 2: the rim
  // tiles, 0: all (see the fast-loop overlap in launch_step2d)
  if (part) {
    const bool rim = bI.x == 0 || bI.x + 1 == gridDim.x || bI.y == 0 || bI.y + 1 == gridDim.y;
    if (rim != (part == 2)) return;
  }
  __shared__ FBTile T;
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long sj = b.nx2, n2 = b.n2;
  const int i0 = tile_i0(R.i0) + (int)bI.x * kBX, j0 = R.j0 + (int)bI.y * kBY;
  const int tid = threadIdx.x + kBX * threadIdx.y;
  constexpr int NT = kBX * kBY;
  auto G = [&](int i, int j) { return (i - (i0 - 2)) + (j - (j0 - 2)) * kGX; };
  // inside the allocated planes (wide fast halos: gx more ghost cells, roms_dev.h)
  auto inarr = [&](int i, int j) {
    return i >= -1 - b.gx && i <= b.Lm + 2 + b.gx && j >= -1 - b.gx && j <= b.Mm + 2 + b.gx;
  };
  // vwrap: single-rank periodic directions read the fast-time fields' halo
  // cells from their periodic images (the per-step wrap is deferred to the
  // end of the fast loop, see launch_step2d)
  auto FT = [&](int i, int j) -> long {
    if (kWrap && (vwrap & 1)) i = i < 1 ? i + b.Lm : (i > b.Lm ? i - b.Lm : i);
    if (kWrap && (vwrap & 2)) j = j < 1 ? j + b.Mm : (j > b.Mm ? j - b.Mm : j);
    return IJ(b, i, j);
  };
  // All global loads are issued at entry -- the staging window first, then
  // the face fluxes, then the later phases -- so each block waits for memory
  // once (the grid is one wave of blocks: a block's critical path is the
  // kernel time) and the window stores start as soon as their data lands.
  double g_z0[2], g_z1[2], g_z2[2], g_h[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int q = tid + r * NT;
    const int i = i0 - 2 + q % kGX, j = j0 - 2 + q / kGX;
    g_z0[r] = g_z1[r] = g_z2[r] = g_h[r] = 0.0;
    if (q < kGN && inarr(i, j)) {
      const long ij = IJ(b, i, j), ft = FT(i, j);
      g_z0[r] = LD(kW_zeta, ft, (long)(c.kstp - 1) * n2);
      g_z1[r] = LD(kW_zeta, ft, (long)(c.kbak - 1) * n2);
      g_z2[r] = LD(kW_zeta, ft, (long)(c.kold - 1) * n2);
      g_h[r] = LD(kW_h, ij);
    }
  }
  double f_a[3], f_b[3], f_c[3], f_d[3];  // 3 time levels of ubar/vbar and dn_u/dm_v at the thread's faces
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int q = tid + r * NT;
    f_a[r] = f_b[r] = f_c[r] = f_d[r] = 0.0;
    if (q < kUN) {
      const int i = i0 - 1 + q % kUX, j = j0 - 1 + q / kUX;
      if (i >= -b.gx && inarr(i, j)) {   // DUon needs Drhs(i-1)
        const long ij = IJ(b, i, j), ft = FT(i, j);
        f_a[r] = LD(kW_ubar, ft, (long)(c.kstp - 1) * n2); f_b[r] = LD(kW_ubar, ft, (long)(c.kbak - 1) * n2);
        f_c[r] = LD(kW_ubar, ft, (long)(c.kold - 1) * n2); f_d[r] = LD(kW_dn_u, ij);
      }
    } else if (q < kUN + kVN) {
      const int qq = q - kUN;
      const int i = i0 - 1 + qq % kFX, j = j0 - 1 + qq / kFX;
      if (j >= -b.gx && inarr(i, j)) {   // DVom needs Drhs(j-1)
        const long ij = IJ(b, i, j), ft = FT(i, j);
        f_a[r] = LD(kW_vbar, ft, (long)(c.kstp - 1) * n2); f_b[r] = LD(kW_vbar, ft, (long)(c.kbak - 1) * n2);
        f_c[r] = LD(kW_vbar, ft, (long)(c.kold - 1) * n2); f_d[r] = LD(kW_dm_v, ij);
      }
    }
  }
  const int za = b.istrU - 1, zb = b.iend, zc = b.jstrV - 1, zd = b.jend;
  double e_pm[2], e_pn[2], e_sw[2], e_rm[2], e_rS[2], e_rA[2], e_pf[2];
  bool e_pp[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int q = tid + r * NT;
    const int i = i0 - 1 + q % kFX, j = j0 - 1 + q / kFX;
    e_pm[r] = e_pn[r] = e_sw[r] = e_rm[r] = e_rS[r] = e_rA[r] = e_pf[r] = 0.0;
    e_pp[r] = false;
    if (q < kFN && i >= za && i <= zb && j >= zc && j <= zd) {
      const long ij = IJ(b, i, j);
      e_pm[r] = LD(kW_pm, ij);
      e_pn[r] = LD(kW_pn, ij);
      e_sw[r] = LD(kW_swflx, ij); e_rS[r] = LD(kW_rhoS, ij); e_rA[r] = LD(kW_rhoA, ij);
      if (kPipe) { e_pp[r] = F.pipe_idx[ij] > 0; e_pf[r] = F.pipe_flx[ij]; }
    }
    // rmask of every window cell: the zeta range's, and the closed-wall
    // ghost cells' that zetabc multiplies by below (loaded with the rest, so
    // zetabc issues no load and waits for no memory round trip of its own)
    if (closed != 0 ? (q < kFN && inarr(i, j)) : (q < kFN && i >= za && i <= zb && j >= zc && j <= zd))
      e_rm[r] = LD(kW_rmask, IJ(b, i, j));
  }
  const int pi = i0 + (int)threadIdx.x, pj = j0 + (int)threadIdx.y;
  const bool pact = pi >= R.i0 && pi <= R.i1 && pj <= R.j1;
  const bool pint = pact && pi >= b.istr && pi <= b.iend && pj >= b.jstr && pj <= b.jend;
  const long pij = pact ? IJ(b, pi, pj) : 0;
  double x_rA0 = 0, x_rAx = 0, x_rAy = 0, x_dnu = 0, x_dmv = 0, x_rufrc = 0, x_rvfrc = 0, x_ub = 0, x_vb = 0;
  double x_pmx = 0, x_pnx = 0, x_pmy = 0, x_pny = 0, x_pm0 = 0, x_pn0 = 0, x_um = 0, x_vm = 0, x_DU1 = 0, x_DV1 = 0;
  double x_rS0 = 0, x_rSx = 0, x_rSy = 0, x_DU2 = 0, x_DV2 = 0, x_Zt = 0;
  if (pint) {
    const long lk = (long)(c.kstp - 1) * n2;
    x_rA0 = LD(kW_rhoA, pij); x_rAx = LD(kW_rhoA, pij - 1); x_rAy = LD(kW_rhoA, pij - sj);
    x_dnu = LD(kW_dn_u, pij); x_dmv = LD(kW_dm_v, pij);
    x_rufrc = LD(kW_rufrc, pij); x_rvfrc = LD(kW_rvfrc, pij);
    x_ub = LD(kW_ubar, pij, lk); x_vb = LD(kW_vbar, pij, lk);
    x_pm0 = LD(kW_pm, pij); x_pn0 = LD(kW_pn, pij); x_pmx = LD(kW_pm, pij - 1); x_pnx = LD(kW_pn, pij - 1);
    x_pmy = LD(kW_pm, pij - sj); x_pny = LD(kW_pn, pij - sj);
    x_um = LD(kW_umask, pij); x_vm = LD(kW_vmask, pij);
    x_DU1 = LD(kW_DU_avg1, pij); x_DV1 = LD(kW_DV_avg1, pij);
    x_DU2 = LD(kW_DU_avg2, pij); x_DV2 = LD(kW_DV_avg2, pij); x_Zt = LD(kW_Zt_avg1, pij);
    if (c.iif == 1) { x_rS0 = LD(kW_rhoS, pij); x_rSx = LD(kW_rhoS, pij - 1); x_rSy = LD(kW_rhoS, pij - sj); }
  }
  S2D_T(1);   // entry loads issued
  // P0: time levels of zeta, h and Drhs = h + fwd*z(kstp) + fwd1*z(kbak) + fwd2*z(kold)
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int q = tid + r * NT;
    if (q >= kGN) break;
    T.z0[q] = g_z0[r]; T.z1[q] = g_z1[r]; T.z2[q] = g_z2[r]; T.h[q] = g_h[r];
    T.Dr[q] = g_h[r] + c.fwd * g_z0[r] + c.fwd1 * g_z1[r] + c.fwd2 * g_z2[r];
  }
  __syncthreads();
  S2D_T(2);   // window in LDS
  // P1: barotropic fluxes DUon (u faces) and DVom (v faces), once each
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int q = tid + r * NT;
    if (q < kUN) {
      const int i = i0 - 1 + q % kUX, j = j0 - 1 + q / kUX;
      double v = 0.0;
      if (i >= -b.gx && inarr(i, j)) {   // DUon needs Drhs(i-1)
        const double urhs = c.fwd * f_a[r] + c.fwd1 * f_b[r] + c.fwd2 * f_c[r];
        v = 0.5 * (T.Dr[G(i, j)] + T.Dr[G(i - 1, j)]) * f_d[r] * (urhs);
      }
      T.DU[q] = v;
    } else if (q < kUN + kVN) {
      const int qq = q - kUN;
      const int i = i0 - 1 + qq % kFX, j = j0 - 1 + qq / kFX;
      double v = 0.0;
      if (j >= -b.gx && inarr(i, j)) {   // DVom needs Drhs(j-1)
        const double vrhs = c.fwd * f_a[r] + c.fwd1 * f_b[r] + c.fwd2 * f_c[r];
        v = 0.5 * (T.Dr[G(i, j)] + T.Dr[G(i, j - 1)]) * f_d[r] * (vrhs);
      }
      T.DV[qq] = v;
    }
  }
  __syncthreads();
  auto DU = [&](int i, int j) { return T.DU[(i - (i0 - 1)) + (j - (j0 - 1)) * kUX]; };
  auto DV = [&](int i, int j) { return T.DV[(i - (i0 - 1)) + (j - (j0 - 1)) * kFX]; };
  S2D_T(3);   // DU/DV
  // P2: free surface and the backward-averaged terms of the reference's
  // zeta range (istrU-1..iend, jstrV-1..jend) inside the window
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int q = tid + r * NT;
    if (q >= kFN) break;
    const int i = i0 - 1 + q % kFX, j = j0 - 1 + q / kFX;
    if (i < za || i > zb || j < zc || j > zd) {  // never consumed
      T.zn[q] = T.Dn[q] = T.zw[q] = T.rz[q] = T.rz2[q] = T.rzSA[q] = 0.0;
      T.st[q] = 0;
      continue;
    }
    T.st[q] = 1;
    const int g = G(i, j);
    const double zk = T.z0[g];
    double zn = zk + d.p.dtfast * e_pm[r] * e_pn[r] * (DU(i, j) - DU(i + 1, j) + DV(i, j) - DV(i, j + 1)) +
                d.p.dtfast * e_sw[r];
    if (kPipe && e_pp[r]) zn = zn + d.p.dtfast * e_pm[r] * e_pn[r] * e_pf[r];  // step2d_FB.F:155-159
    zn = zn * e_rm[r];
    const double zwrk = c.bkw_new * zn + c.bkw * zk + c.bkw1 * T.z1[g] + c.bkw2 * T.z2[g];
    const double rhoS = e_rS[r];
    const double rzeta = (1.0 + rhoS) * zwrk;
    T.zn[q] = zn;
    T.Dn[q] = zn + T.h[g];
    T.zw[q] = zwrk;
    T.rz[q] = rzeta;
    T.rzSA[q] = zwrk * (rhoS - e_rA[r]);
    T.rz2[q] = rzeta * zwrk;
  }
  __syncthreads();
  S2D_T(4);   // zeta part
  // blocks whose window (i0-1..i0+63, j0-1..j0+3) reaches a closed wall's
  // ghost line: only they have zetabc cells (block-uniform, so the others
  // skip its two barriers)
  const bool wall_win = (b.west_edge && b.istr - 1 >= i0 - 1 && b.istr - 1 <= i0 + kBX - 1) ||
                        (b.east_edge && b.iend + 1 >= i0 - 1 && b.iend + 1 <= i0 + kBX - 1) ||
                        (b.south_edge && b.jstr - 1 >= j0 - 1 && b.jstr - 1 <= j0 + kBY - 1) ||
                        (b.north_edge && b.jend + 1 >= j0 - 1 && b.jend + 1 <= j0 + kBY - 1);
  if (closed != 0 && wall_win) {
    // zetabc_tile (zetabc.F), closed walls: edges, then corners
    auto L = [&](int i, int j) { return (i - (i0 - 1)) + (j - (j0 - 1)) * kFX; };
    auto in = [&](int i, int j) { return i >= i0 - 1 && i <= i0 + kBX - 1 && j >= j0 - 1 && j <= j0 + kBY - 1; };
#pragma unroll
    for (int r = 0; r < 2; r++) {   // window cell q = tid + r*NT: its rmask is e_rm[r]
      const int q = tid + r * NT;
      if (q >= kFN) break;
      const int i = i0 - 1 + q % kFX, j = j0 - 1 + q / kFX;
      if (j >= b.jstrV - 1 && j <= b.jend) {
        if (b.west_edge && i == b.istr - 1 && in(b.istr, j)) { T.zn[q] = T.zn[L(b.istr, j)] * e_rm[r]; T.st[q] = 2; }
        if (b.east_edge && i == b.iend + 1 && in(b.iend, j)) { T.zn[q] = T.zn[L(b.iend, j)] * e_rm[r]; T.st[q] = 2; }
      }
      if (i >= b.istrU - 1 && i <= b.iend) {
        if (b.south_edge && j == b.jstr - 1 && in(i, b.jstr)) { T.zn[q] = T.zn[L(i, b.jstr)] * e_rm[r]; T.st[q] = 2; }
        if (b.north_edge && j == b.jend + 1 && in(i, b.jend)) { T.zn[q] = T.zn[L(i, b.jend)] * e_rm[r]; T.st[q] = 2; }
      }
    }
    __syncthreads();
    if (tid == 0) {
      const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
      if (b.south_edge && b.west_edge && in(is - 1, js - 1) && in(is, js - 1) && in(is - 1, js)) { T.zn[L(is - 1, js - 1)] = 0.5 * (T.zn[L(is, js - 1)] + T.zn[L(is - 1, js)]); T.st[L(is - 1, js - 1)] = 2; }
      if (b.south_edge && b.east_edge && in(ie + 1, js - 1) && in(ie, js - 1) && in(ie + 1, js)) { T.zn[L(ie + 1, js - 1)] = 0.5 * (T.zn[L(ie, js - 1)] + T.zn[L(ie + 1, js)]); T.st[L(ie + 1, js - 1)] = 2; }
      if (b.north_edge && b.west_edge && in(is - 1, je + 1) && in(is, je + 1) && in(is - 1, je)) { T.zn[L(is - 1, je + 1)] = 0.5 * (T.zn[L(is, je + 1)] + T.zn[L(is - 1, je)]); T.st[L(is - 1, je + 1)] = 2; }
      if (b.north_edge && b.east_edge && in(ie + 1, je + 1) && in(ie, je + 1) && in(ie + 1, je)) { T.zn[L(ie + 1, je + 1)] = 0.5 * (T.zn[L(ie, je + 1)] + T.zn[L(ie + 1, je)]); T.st[L(ie + 1, je + 1)] = 2; }
    }
    __syncthreads();
  }
  if (closed == 1) {
    // the edge kernels read zeta_new / Dnew from global scratch: every block
    // stores the window cells it computed or set (identical values where
    // windows overlap); with the edges folded in (closed == 2) the block
    // reads them from its window instead
    for (int q = tid; q < kFN; q += NT) {
      if (!T.st[q]) continue;
      const long o = IJ(b, i0 - 1 + q % kFX, j0 - 1 + q / kFX);
      ST(kW_s0, o, T.zn[q]);
      if (T.st[q] == 1) ST(kW_s1, o, T.Dn[q]);
    }
  }
  S2D_T(5);   // zetabc
  // P3: zeta(knew), fast averages, pressure gradient, momentum
  const int i = i0 + (int)threadIdx.x, j = j0 + (int)threadIdx.y;
  const bool pin = i >= R.i0 && i <= R.i1 && j <= R.j1;
  if (closed != 2 && !pin) return;
  const int q = (threadIdx.x + 1) + (threadIdx.y + 1) * kFX;  // (i,j); q-1 = (i-1,j); q-kFX = (i,j-1)
  const int g = G(i, j);                                        // g-1: (i-1,j); g-kGX: (i,j-1)
  const long ij = IJ(b, i, j);
  double ubn = 0.0, vbn = 0.0;   // ubar/vbar(knew) this lane formed (closed == 2)
  if (pin) {
    const double z = T.zn[q];
    ST(kW_zeta, ij, z, (long)(c.knew - 1) * n2);
    const double du = DU(i, j), dv = DV(i, j);
    if (c.iif == 1) {
      ST(kW_DU_avg_bak, ij, (pint ? x_DU1 : LD(kW_DU_avg1, ij)) - 0.1024390243902439 * (pint ? x_DU2 : LD(kW_DU_avg2, ij)));
      ST(kW_DV_avg_bak, ij, (pint ? x_DV1 : LD(kW_DV_avg1, ij)) - 0.1024390243902439 * (pint ? x_DV2 : LD(kW_DV_avg2, ij)));
      ST(kW_Zt_avg1, ij, c.w1 * z);
      ST(kW_DU_avg1, ij, 0.0);
      ST(kW_DV_avg1, ij, 0.0);
      ST(kW_DU_avg2, ij, c.w2 * du);
      ST(kW_DV_avg2, ij, c.w2 * dv);
    } else {
      ST(kW_Zt_avg1, ij, (pint ? x_Zt : LD(kW_Zt_avg1, ij)) + c.w1 * z);
      ST(kW_DU_avg2, ij, (pint ? x_DU2 : LD(kW_DU_avg2, ij)) + c.w2 * du);
      ST(kW_DV_avg2, ij, (pint ? x_DV2 : LD(kW_DV_avg2, ij)) + c.w2 * dv);
    }
  }
  if (pint) {
    const double gh = 0.5 * d.p.g;
    const double h0 = T.h[g], hxm = T.h[g - 1], hym = T.h[g - kGX];
    const double rA0 = x_rA0, rAx = x_rAx, rAy = x_rAy;
    // pressure gradient at u (neighbour q-1) and v (neighbour q-kFX) points
    auto pgf = [&](int qm, double hm, double rAm, double dn) {
      return gh * dn *
             ((hm + h0) * (T.rz[qm] - T.rz[q]) + T.rz2[qm] - T.rz2[q] +
              (hm - h0) * (T.rzSA[qm] + T.rzSA[q] + 0.333333333333 * (rAm - rA0) * (T.zw[qm] - T.zw[q])));
    };
    const double dn_u = x_dnu, dm_v = x_dmv;
    double rubar = pgf(q - 1, hxm, rAx, dn_u);
    double rvbar = pgf(q - kFX, hym, rAy, dm_v);
    double rufrc = x_rufrc, rvfrc = x_rvfrc;
    if (c.iif == 1) {
      rufrc = rufrc - rubar;
      rvfrc = rvfrc - rvbar;
      ST(kW_rufrc, ij, rufrc);
      ST(kW_rvfrc, ij, rvfrc);
      auto corr = [&](int qq, int gg, double rS, double rA, double& zwrk, double& rzeta, double& rzeta2,
                      double& rzetaSA) {
        const double zn = T.zn[qq], zk = T.z0[gg];
        zwrk = zn - zk;
        rzeta = (1.0 + rS) * zwrk;
        rzeta2 = rzeta * (zn + zk);
        rzetaSA = zwrk * (rS - rA);
      };
      double zw0, rz0, rz20, sa0, zw1, rz1, rz21, sa1, zw2, rz2_, rz22, sa2;
      corr(q, g, x_rS0, rA0, zw0, rz0, rz20, sa0);
      corr(q - 1, g - 1, x_rSx, rAx, zw1, rz1, rz21, sa1);
      corr(q - kFX, g - kGX, x_rSy, rAy, zw2, rz2_, rz22, sa2);
      rubar = rubar + gh * dn_u *
                          ((hxm + h0) * (rz1 - rz0) + rz21 - rz20 +
                           (hxm - h0) * (sa1 + sa0 + 0.333333333333 * (rAx - rA0) * (zw1 - zw0)));
      rvbar = rvbar + gh * dm_v *
                          ((hym + h0) * (rz2_ - rz0) + rz22 - rz20 +
                           (hym - h0) * (sa2 + sa0 + 0.333333333333 * (rAy - rA0) * (zw2 - zw0)));
    }
    const double cff = 0.5 * d.p.dtfast, cff1 = 0.5 * c.w1;
    const double Dstp0 = T.z0[g] + h0;
    if (i >= b.istrU) {
      const double Dstpm = T.z0[g - 1] + hxm;
      const double DUnew = ((Dstp0 + Dstpm) * x_ub + cff * (x_pm0 + x_pmx) * (x_pn0 + x_pnx) * (rubar + rufrc)) * x_um;
      ubn = DUnew / (T.Dn[q] + T.Dn[q - 1]);
      ST(kW_ubar, ij, ubn, (long)(c.knew - 1) * n2);
      ST(kW_DU_avg1, ij, (c.iif == 1 ? 0.0 : x_DU1) + cff1 * dn_u * (DUnew));
    }
    if (j >= b.jstrV) {
      const double Dstpm = T.z0[g - kGX] + hym;
      const double DVnew = ((Dstp0 + Dstpm) * x_vb + cff * (x_pm0 + x_pmy) * (x_pn0 + x_pny) * (rvbar + rvfrc)) * x_vm;
      vbn = DVnew / (T.Dn[q] + T.Dn[q - kFX]);
      ST(kW_vbar, ij, vbn, (long)(c.knew - 1) * n2);
      ST(kW_DV_avg1, ij, (c.iif == 1 ? 0.0 : x_DV1) + cff1 * dm_v * (DVnew));
    }
  }
  S2D_T(6);   // P3 stores issued
  // the folded wall phases act on lanes of a wall's first or ghost row /
  // column only (i = istr-1..istr, iend+1; j = jstr-1..jstr, jend+1):
  // blocks whose tile holds none skip them and their barrier (block-uniform)
  const bool wall_tile = (b.west_edge && b.istr >= i0 && b.istr - 1 <= i0 + kBX - 1) ||
                         (b.east_edge && b.iend + 1 >= i0 && b.iend + 1 <= i0 + kBX - 1) ||
                         (b.south_edge && b.jstr >= j0 && b.jstr - 1 <= j0 + kBY - 1) ||
                         (b.north_edge && b.jend + 1 >= j0 && b.jend + 1 <= j0 + kBY - 1);
  if (closed != 2 || !wall_tile) return;
  // ---- closed walls folded in (k_s2d_edges phases 0, 1, 3 with no open
  // edge; the host folds only when every edge cell and its interior
  // neighbour fall in one tile).  Same expressions as k_s2d_edges. ----
  {
    const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
    const long kn = (long)(c.knew - 1) * n2;
    double* sU = T.z1;   // ubar / vbar(knew) of the tile cells (z1, z2: last read in P2)
    double* sV = T.z2;
    const int t = threadIdx.x + kBX * threadIdx.y;
    // phase 0: wall-normal components (u2dbc_im.F / v2dbc_im.F closed walls)
    if (pin && j >= js && j <= je && ((b.west_edge && i == is) || (b.east_edge && i == ie + 1))) {
      ubn = 0.0;
      ST(kW_ubar, ij, ubn, kn);
    }
    if (pin && i >= is && i <= ie && ((b.south_edge && j == js) || (b.north_edge && j == je + 1))) {
      vbn = 0.0;
      ST(kW_vbar, ij, vbn, kn);
    }
    sU[t] = ubn;
    sV[t] = vbn;
    __syncthreads();
    if (!pin) return;
    const double g2 = d.p.gamma2;
    // phase 1: tangential components from the first interior row / column
    {
      const int i0t = b.ew_periodic ? b.istrU : is, i1t = b.ew_periodic ? ie : b.iendR;
      if (b.south_edge && j == js - 1 && i >= i0t && i <= i1t) {
        ubn = g2 * sU[t + kBX] * LD(kW_umask, ij);
        ST(kW_ubar, ij, ubn, kn);
      }
      if (b.north_edge && j == je + 1 && i >= i0t && i <= i1t) {
        ubn = g2 * sU[t - kBX] * LD(kW_umask, ij);
        ST(kW_ubar, ij, ubn, kn);
      }
      const int j0t = b.ns_periodic ? b.jstrV : js, j1t = b.ns_periodic ? je : b.jendR;
      if (b.west_edge && i == is - 1 && j >= j0t && j <= j1t) {
        vbn = g2 * sV[t + 1] * LD(kW_vmask, ij);
        ST(kW_vbar, ij, vbn, kn);
      }
      if (b.east_edge && i == ie + 1 && j >= j0t && j <= j1t) {
        vbn = g2 * sV[t - 1] * LD(kW_vmask, ij);
        ST(kW_vbar, ij, vbn, kn);
      }
    }
    // phase 3: fast-time-averaged fluxes through the boundary faces; Dnew of
    // a window cell is Dn (computed) or h + zeta_new (set by zetabc)
    auto Dn = [&](int qq, int gg) { return T.st[qq] == 1 ? T.Dn[qq] : T.h[gg] + T.zn[qq]; };
    const double cff1 = 0.5 * c.w1;
    const long sj = b.nx2;
    bool du = false, dv = false;
    if (b.west_edge && i == b.istrU - 1 && j >= b.jstrR && j <= b.jendR) du = true;
    if (b.east_edge && i == ie + 1 && j >= b.jstrR && j <= b.jendR) du = true;
    if (b.south_edge && j == js - 1 && i >= b.istrU && i <= ie) du = true;
    if (b.north_edge && j == je + 1 && i >= b.istrU && i <= ie) du = true;
    if (b.west_edge && i == is - 1 && j >= b.jstrV && j <= je) dv = true;
    if (b.east_edge && i == ie + 1 && j >= b.jstrV && j <= je) dv = true;
    if (b.south_edge && j == b.jstrV - 1 && i >= b.istrR && i <= b.iendR) dv = true;
    if (b.north_edge && j == je + 1 && i >= b.istrR && i <= b.iendR) dv = true;
    if (du) ST(kW_DU_avg1, ij, LD(kW_DU_avg1, ij) + cff1 * (Dn(q, g) + Dn(q - 1, g - 1)) * (ubn) * LD(kW_dn_u, ij));
    if (dv) ST(kW_DV_avg1, ij, LD(kW_DV_avg1, ij) + cff1 * (Dn(q, g) + Dn(q - kFX, g - kGX)) * (vbn) * LD(kW_dm_v, ij));
    (void)sj;
    S2D_T(7);   // walls folded in
  }
}

// u2dbc/v2dbc (u2dbc_im.F:3-481, v2dbc_im.F:3-472), boundary Dnew and the
// boundary flux averages (step2d_FB.F:444-529).  Phase 0: wall-normal
// components (closed: 0; open: OBC_M2FLATHER with zeta/ubar_west...),
// 1: tangential components (closed: gamma2; open: the OBC_M2ORLANSKI branch
// the reference switches to under OBC_M2FLATHER, u2dbc_im.F:270-273) and the
// boundary Dnew, 2: corners between adjacent open edges, 3: flux averages.
__device__ __forceinline__ double flather_zx(double cx, double zi, double zb, double zin) {
  double zx = (0.5 + cx) * zi + (0.5 - cx) * zb;
  if (cx > 0.292893218813452) {
    const double q = 1. - 0.292893218813452 / cx;
    zx = zx + (zin + cx * zb - (1. + cx) * zi) * (q * q);
  }
  return zx;
}
__device__ __forceinline__ double orl_tan2(double cx, double cy, double bs, double is, double gb0, double gb1,
                                           double gi0, double gi1, double bry) {
  double cext;
  if (cx > 0.) cext = 0.;
  else { cext = -cx; cx = 0.; }
  double r = (1. - cx) * (bs - fmax0(cy) * gb0 - fmin0(cy) * gb1) + cx * (is - fmax0(cy) * gi0 - fmin0(cy) * gi1);
  return (1. - cext) * r + cext * bry;
}
__global__ void k_s2d_edges(Dev d, FBCoef c, int phase) {
  const Bounds& b = d.b;
  const Fields& F = d.f;
  const long n2 = b.n2, kn = (long)(c.knew - 1) * n2, ksl = (long)(c.kstp - 1) * n2;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int L = (b.Lm > b.Mm ? b.Lm : b.Mm) + 4 + 2 * b.gx;  // edge lanes per side
  const int side = p / L, q = p - side * L;
  if (side > 3) return;
  double* ub = F.ubar + kn;
  double* vb = F.vbar + kn;
  const double* ubs = F.ubar + ksl;
  const double* vbs = F.vbar + ksl;
  const double* zs = F.zeta + ksl;
  const double* zn = F.zeta + kn;
  double* Dn = F.s1;
  const double g2 = d.p.gamma2, dtf = d.p.dtfast, g = d.p.g;
  const int is = b.istr, ie = b.iend, js = b.jstr, je = b.jend;
  const bool oW = d.p.obc & 1, oE = d.p.obc & 2, oS = d.p.obc & 4, oN = d.p.obc & 8;
  auto pm = [&](int i, int j) { return F.pm[IJ(b, i, j)]; };
  auto pn = [&](int i, int j) { return F.pn[IJ(b, i, j)]; };
  auto hh = [&](int i, int j) { return F.h[IJ(b, i, j)]; };
  auto U = [&](const double* a, int i, int j) { return a[IJ(b, i, j)]; };
  if (phase == 0) {  // wall-normal components
    if (side == 0 && b.west_edge && q <= je - js) {
      const int j = js + q;
      double val = 0.0;
      if (oW) {
        const double cff = 0.5 * (hh(is - 1, j) + hh(is, j));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (pm(is - 1, j) + pm(is, j));
        const double zx = flather_zx(cx, U(zs, is, j), U(zs, is - 1, j), U(zn, is, j));
        val = 0.5 * ((1. - cx) * U(ubs, is, j) + cx * U(ubs, is + 1, j) + F.bubar[0][j] - hx * (zx - F.bzeta[0][j])) *
              F.umask[IJ(b, is, j)];
      }
      ub[IJ(b, is, j)] = val;
    }
    if (side == 1 && b.east_edge && q <= je - js) {
      const int j = js + q;
      double val = 0.0;
      if (oE) {
        const double cff = 0.5 * (hh(ie, j) + hh(ie + 1, j));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (pm(ie, j) + pm(ie + 1, j));
        const double zx = flather_zx(cx, U(zs, ie, j), U(zs, ie + 1, j), U(zn, ie, j));
        val = 0.5 * ((1. - cx) * U(ubs, ie + 1, j) + cx * U(ubs, ie, j) + F.bubar[1][j] + hx * (zx - F.bzeta[1][j])) *
              F.umask[IJ(b, ie + 1, j)];
      }
      ub[IJ(b, ie + 1, j)] = val;
    }
    if (side == 2 && b.south_edge && q <= ie - is) {
      const int i = is + q;
      double val = 0.0;
      if (oS) {
        const double cff = 0.5 * (hh(i, js - 1) + hh(i, js));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (pn(i, js - 1) + pn(i, js));
        const double zx = flather_zx(cx, U(zs, i, js), U(zs, i, js - 1), U(zn, i, js));
        val = 0.5 * ((1. - cx) * U(vbs, i, js) + cx * U(vbs, i, js + 1) + F.bvbar[2][i] - hx * (zx - F.bzeta[2][i])) *
              F.vmask[IJ(b, i, js)];
      }
      vb[IJ(b, i, js)] = val;
    }
    if (side == 3 && b.north_edge && q <= ie - is) {
      const int i = is + q;
      double val = 0.0;
      if (oN) {
        const double cff = 0.5 * (hh(i, je) + hh(i, je + 1));
        const double hx = sqrt(g / cff);
        const double cx = dtf * cff * hx * 0.5 * (pn(i, je) + pn(i, je + 1));
        const double zx = flather_zx(cx, U(zs, i, je), U(zs, i, je + 1), U(zn, i, je));
        val = 0.5 * ((1. - cx) * U(vbs, i, je + 1) + cx * U(vbs, i, je) + F.bvbar[3][i] + hx * (zx - F.bzeta[3][i])) *
              F.vmask[IJ(b, i, je + 1)];
      }
      vb[IJ(b, i, je + 1)] = val;
    }
  } else if (phase == 1) {  // tangential components + boundary Dnew
    if (side == 2 && b.south_edge) {
      if (oS) {
        const int i = b.istrU + q;
        if (i <= ie) {
          auto gr = [&](int ii, int jj) { return U(ubs, ii + 1, jj) - U(ubs, ii, jj); };
          const double cx = -0.125 * dtf * (U(vbs, i, js) + U(vbs, i - 1, js)) * (pn(i, js - 1) + pn(i - 1, js - 1) + pn(i, js) + pn(i - 1, js));
          const double cy = 0.125 * dtf * (U(ubs, i, js - 1) + U(ubs, i, js)) * (pm(i, js - 1) + pm(i - 1, js - 1) + pm(i, js) + pm(i - 1, js));
          const double r = orl_tan2(cx, cy, U(ubs, i, js - 1), U(ubs, i, js), gr(i - 1, js - 1), gr(i, js - 1),
                                    gr(i - 1, js), gr(i, js), F.bubar[2][i]);
          ub[IJ(b, i, js - 1)] = r * F.umask[IJ(b, i, js - 1)];
        }
      } else if (q <= b.iendR - is) {
        const int i0 = b.ew_periodic ? b.istrU : is, i1 = b.ew_periodic ? ie : b.iendR;
        const int i = i0 + q;
        if (i <= i1) ub[IJ(b, i, js - 1)] = g2 * ub[IJ(b, i, js)] * F.umask[IJ(b, i, js - 1)];
      }
    }
    if (side == 3 && b.north_edge) {
      if (oN) {
        const int i = b.istrU + q;
        if (i <= ie) {
          auto gr = [&](int ii, int jj) { return U(ubs, ii + 1, jj) - U(ubs, ii, jj); };
          const double cx = 0.125 * dtf * (U(vbs, i, je + 1) + U(vbs, i - 1, je + 1)) * (pn(i, je) + pn(i - 1, je) + pn(i, je + 1) + pn(i - 1, je + 1));
          const double cy = 0.125 * dtf * (U(ubs, i, je) + U(ubs, i, je + 1)) * (pm(i, je) + pm(i - 1, je) + pm(i, je + 1) + pm(i - 1, je + 1));
          const double r = orl_tan2(cx, cy, U(ubs, i, je + 1), U(ubs, i, je), gr(i - 1, je + 1), gr(i, je + 1),
                                    gr(i - 1, je), gr(i, je), F.bubar[3][i]);
          ub[IJ(b, i, je + 1)] = r * F.umask[IJ(b, i, je + 1)];
        }
      } else if (q <= b.iendR - is) {
        const int i0 = b.ew_periodic ? b.istrU : is, i1 = b.ew_periodic ? ie : b.iendR;
        const int i = i0 + q;
        if (i <= i1) ub[IJ(b, i, je + 1)] = g2 * ub[IJ(b, i, je)] * F.umask[IJ(b, i, je + 1)];
      }
    }
    if (side == 0 && b.west_edge) {
      if (oW) {
        const int j = b.jstrV + q;
        if (j <= je) {
          auto gr = [&](int ii, int jj) { return U(vbs, ii, jj + 1) - U(vbs, ii, jj); };
          const double cx = -0.125 * dtf * (U(ubs, is, j) + U(ubs, is, j - 1)) * (pm(is - 1, j) + pm(is - 1, j - 1) + pm(is, j) + pm(is, j - 1));
          const double cy = 0.125 * dtf * (U(vbs, is - 1, j) + U(vbs, is, j)) * (pn(is - 1, j) + pn(is - 1, j - 1) + pn(is, j) + pn(is, j - 1));
          const double r = orl_tan2(cx, cy, U(vbs, is - 1, j), U(vbs, is, j), gr(is - 1, j - 1), gr(is - 1, j),
                                    gr(is, j - 1), gr(is, j), F.bvbar[0][j]);
          vb[IJ(b, is - 1, j)] = r * F.vmask[IJ(b, is - 1, j)];
        }
      } else {
        const int j0 = b.ns_periodic ? b.jstrV : js, j1 = b.ns_periodic ? je : b.jendR;
        const int j = j0 + q;
        if (j <= j1) vb[IJ(b, is - 1, j)] = g2 * vb[IJ(b, is, j)] * F.vmask[IJ(b, is - 1, j)];
      }
    }
    if (side == 1 && b.east_edge) {
      if (oE) {
        const int j = b.jstrV + q;
        if (j <= je) {
          auto gr = [&](int ii, int jj) { return U(vbs, ii, jj + 1) - U(vbs, ii, jj); };
          const double cx = 0.125 * dtf * (U(ubs, ie + 1, j) + U(ubs, ie + 1, j - 1)) * (pm(ie, j) + pm(ie, j - 1) + pm(ie + 1, j) + pm(ie + 1, j - 1));
          const double cy = 0.125 * dtf * (U(vbs, ie, j) + U(vbs, ie + 1, j)) * (pn(ie, j) + pn(ie, j - 1) + pn(ie + 1, j) + pn(ie + 1, j - 1));
          const double r = orl_tan2(cx, cy, U(vbs, ie + 1, j), U(vbs, ie, j), gr(ie + 1, j - 1), gr(ie + 1, j),
                                    gr(ie, j - 1), gr(ie, j), F.bvbar[1][j]);
          vb[IJ(b, ie + 1, j)] = r * F.vmask[IJ(b, ie + 1, j)];
        }
      } else {
        const int j0 = b.ns_periodic ? b.jstrV : js, j1 = b.ns_periodic ? je : b.jendR;
        const int j = j0 + q;
        if (j <= j1) vb[IJ(b, ie + 1, j)] = g2 * vb[IJ(b, ie, j)] * F.vmask[IJ(b, ie + 1, j)];
      }
    }
    if (side == 0 && b.west_edge && q <= b.jendR - (b.jstr - 1)) {
      const long o = IJ(b, b.istr - 1, b.jstr - 1 + q);
      Dn[o] = F.h[o] + F.s0[o];
    }
    if (side == 1 && b.east_edge && q <= b.jendR - (b.jstr - 1)) {
      const long o = IJ(b, b.iend + 1, b.jstr - 1 + q);
      Dn[o] = F.h[o] + F.s0[o];
    }
    if (side == 2 && b.south_edge && q <= b.iendR - (b.istr - 1)) {
      const long o = IJ(b, b.istr - 1 + q, b.jstr - 1);
      Dn[o] = F.h[o] + F.s0[o];
    }
    if (side == 3 && b.north_edge && q <= b.iendR - (b.istr - 1)) {
      const long o = IJ(b, b.istr - 1 + q, b.jend + 1);
      Dn[o] = F.h[o] + F.s0[o];
    }
  } else if (phase == 2) {  // corners between adjacent open edges (u2dbc_im.F:445-478, v2dbc_im.F:440-469)
    if (p != 0) return;
    const bool W = b.west_edge && oW, E = b.east_edge && oE, S = b.south_edge && oS, N = b.north_edge && oN;
    if (S && W) ub[IJ(b, is, js - 1)] = 0.5 * (ub[IJ(b, is + 1, js - 1)] + ub[IJ(b, is, js)]);
    if (S && E) ub[IJ(b, ie + 1, js - 1)] = 0.5 * (ub[IJ(b, ie, js - 1)] + ub[IJ(b, ie + 1, js)]);
    if (N && W) ub[IJ(b, is, je + 1)] = 0.5 * (ub[IJ(b, is + 1, je + 1)] + ub[IJ(b, is, je)]);
    if (N && E) ub[IJ(b, ie + 1, je + 1)] = 0.5 * (ub[IJ(b, ie, je + 1)] + ub[IJ(b, ie + 1, je)]);
    if (S && W) vb[IJ(b, is - 1, js)] = 0.5 * (vb[IJ(b, is - 1, js + 1)] + vb[IJ(b, is, js)]);
    if (S && E) vb[IJ(b, ie + 1, js)] = 0.5 * (vb[IJ(b, ie + 1, js + 1)] + vb[IJ(b, ie, js)]);
    if (N && W) vb[IJ(b, is - 1, je + 1)] = 0.5 * (vb[IJ(b, is - 1, je)] + vb[IJ(b, is, je + 1)]);
    if (N && E) vb[IJ(b, ie + 1, je + 1)] = 0.5 * (vb[IJ(b, ie + 1, je)] + vb[IJ(b, ie, je + 1)]);
  } else {  // boundary fast-time-averaged fluxes
    const double cff1 = 0.5 * c.w1;
    const long sj = b.nx2;
    if (side == 0 && b.west_edge) {
      const int iu = b.istrU - 1;
      if (q <= b.jendR - b.jstrR) {
        const long o = IJ(b, iu, b.jstrR + q);
        F.DU_avg1[o] = F.DU_avg1[o] + cff1 * (Dn[o] + Dn[o - 1]) * (ub[o]) * F.dn_u[o];
      }
      if (q <= b.jend - b.jstrV) {
        const long o = IJ(b, b.istr - 1, b.jstrV + q);
        F.DV_avg1[o] = F.DV_avg1[o] + cff1 * (Dn[o] + Dn[o - sj]) * (vb[o]) * F.dm_v[o];
      }
    }
    if (side == 1 && b.east_edge) {
      if (q <= b.jendR - b.jstrR) {
        const long o = IJ(b, b.iend + 1, b.jstrR + q);
        F.DU_avg1[o] = F.DU_avg1[o] + cff1 * (Dn[o] + Dn[o - 1]) * (ub[o]) * F.dn_u[o];
      }
      if (q <= b.jend - b.jstrV) {
        const long o = IJ(b, b.iend + 1, b.jstrV + q);
        F.DV_avg1[o] = F.DV_avg1[o] + cff1 * (Dn[o] + Dn[o - sj]) * (vb[o]) * F.dm_v[o];
      }
    }
    if (side == 2 && b.south_edge) {
      if (q <= b.iend - b.istrU) {
        const long o = IJ(b, b.istrU + q, b.jstr - 1);
        F.DU_avg1[o] = F.DU_avg1[o] + cff1 * (Dn[o] + Dn[o - 1]) * (ub[o]) * F.dn_u[o];
      }
      if (q <= b.iendR - b.istrR) {
        const long o = IJ(b, b.istrR + q, b.jstrV - 1);
        F.DV_avg1[o] = F.DV_avg1[o] + cff1 * (Dn[o] + Dn[o - sj]) * (vb[o]) * F.dm_v[o];
      }
    }
    if (side == 3 && b.north_edge) {
      if (q <= b.iend - b.istrU) {
        const long o = IJ(b, b.istrU + q, b.jend + 1);
        F.DU_avg1[o] = F.DU_avg1[o] + cff1 * (Dn[o] + Dn[o - 1]) * (ub[o]) * F.dn_u[o];
      }
      if (q <= b.iendR - b.istrR) {
        const long o = IJ(b, b.istrR + q, b.jend + 1);
        F.DV_avg1[o] = F.DV_avg1[o] + cff1 * (Dn[o] + Dn[o - sj]) * (vb[o]) * F.dm_v[o];
      }
    }
  }
}

void launch_fast_step(const Dev& d, hipStream_t s, const FBCoef& c, const Tlev& t);

void launch_step2d(const Dev& d, hipStream_t s, const Tlev& t, const double* w1, const double* w2) {
  const Bounds& b = d.b;
  FBCoef c;
  c.kstp = t.kstp; c.knew = t.knew; c.iif = t.iif; c.nfast = t.nfast;
  if (t.iif == 1) {
    c.kbak = t.kstp; c.kold = t.kstp;
    c.fwd = 1.0; c.fwd1 = 0.0; c.fwd2 = 0.0;
    c.bkw_new = 0.0; c.bkw = 1.0; c.bkw1 = 0.0; c.bkw2 = 0.0;
  } else if (t.iif == 2) {
    c.kbak = t.kstp - 1; if (c.kbak < 1) c.kbak = 4;
    c.kold = c.kbak;
    c.fwd = 1.0; c.fwd1 = 0.0; c.fwd2 = 0.0;
    c.bkw_new = 1.0833333333333; c.bkw = -0.1666666666666; c.bkw1 = 0.0833333333333; c.bkw2 = 0.0;
  } else {
    c.kbak = t.kstp - 1; if (c.kbak < 1) c.kbak = 4;
    c.kold = c.kbak - 1; if (c.kold < 1) c.kold = 4;
    c.fwd = 1.781105; c.fwd1 = -1.06221; c.fwd2 = 0.281105;
    c.bkw_new = 0.614; c.bkw = 0.285; c.bkw1 = 0.088; c.bkw2 = 0.013;
  }
  c.w1 = w1[t.iif - 1];
  c.w2 = w2[t.iif - 1];
  // Multi-rank fast loop with wide halos (Params::s2d_k = K > 1): the
  // zeta/ubar/vbar levels are exchanged 2K deep after every K-th fast step
  // only.  One fast step reads its inputs up to 2 cells beyond the cells it
  // updates, so the m-th step of a group updates the subdomain widened by
  // 2(K-m) cells on every exchange side -- the same cells, with the same
  // inputs and operations, as the neighbour owning them -- and the group's
  // last step updates the subdomain alone.  The exchange after it carries the
  // group's last min(K,3) levels (the AB3 steps read three).  The fields the
  // fast step reads besides those levels are exchanged 2K deep before the
  // first fast step.  Rivers and pipes (their face lists are the owner's)
  // take every step.
  const Halo* Hk = d.halo;
  const int K = (d.p.s2d_k > 1 && Hk && Hk->comm && Hk->wide.g.w == 2 * d.p.s2d_k && d.p.npip == 0 &&
                 d.p.nriv == 0 && !d.p.s2d_split) ? d.p.s2d_k : 1;
  const int gend = K > 1 ? ((t.iif - 1) / K + 1) * K < t.nfast ? ((t.iif - 1) / K + 1) * K : t.nfast : t.iif;
  Dev de = d;   // the bounds this fast step updates
  if (K > 1) {
    const long n2 = b.n2, ks = (long)(t.kstp - 1) * n2;
    const int w = 2 * K;
    if (t.iif == 1) {
      const Fields& F = d.f;
      launch_exchange_list(d, s, ExchList{{F.zeta + ks, F.ubar + ks, F.vbar + ks, F.rufrc, F.rvfrc, F.rhoS, F.rhoA, F.swflx,
                                           F.h, F.pm, F.pn, F.dn_u, F.dm_v, F.rmask, F.umask, F.vmask},
                                          {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}, 16, w});
    }
    const int ext = 2 * (gend - t.iif);
    Bounds& e = de.b;
    if (!e.west_edge) e.istr -= ext;
    if (!e.east_edge) e.iend += ext;
    if (!e.south_edge) e.jstr -= ext;
    if (!e.north_edge) e.jend += ext;
    e.istrR = e.west_edge ? e.istr - 1 : e.istr;
    e.istrU = e.west_edge ? e.istr + 1 : e.istr;
    e.iendR = e.east_edge ? e.iend + 1 : e.iend;
    e.jstrR = e.south_edge ? e.jstr - 1 : e.jstr;
    e.jstrV = e.south_edge ? e.jstr + 1 : e.jstr;
    e.jendR = e.north_edge ? e.jend + 1 : e.jend;
  }
  launch_fast_step(de, s, c, t);
  launch_river_s2d(d, s, t.knew);   // step2d_FB.F:531-554
  const int vwrap = (d.halo == nullptr && !d.p.s2d_split) ? (b.ew_periodic ? 1 : 0) | (b.ns_periodic ? 2 : 0) : 0;
  if (t.iif == t.nfast)   // zeta(knew) = Zt_avg1 (step2d_FB.F:566) inside set_depth's kernel, same range
    launch_set_depth(d, s, t, !vwrap, true);   // vwrap: its z_w, z_r, Hz wrap joins the list below
  if (vwrap) {
    // halos were read from periodic images during the loop; refresh all four
    // time slots once at its end (the same values the per-step wraps give),
    // in one launch with set_depth's z_w, z_r, Hz (set_depth reads no zeta halo)
    if (t.iif == t.nfast)
      launch_exchange_list(d, s, ExchList{{d.f.zeta, d.f.ubar, d.f.vbar, d.f.z_w, d.f.z_r, d.f.Hz},
                                          {4, 4, 4, b.N + 1, b.N, b.N}, 6});
    return;
  }
  if (K > 1) {
    if (t.iif != gend) return;
    const int gstart = ((t.iif - 1) / K) * K + 1;
    const int nl = t.iif - gstart + 1 < 3 ? t.iif - gstart + 1 : 3;
    ExchList L{};
    for (int m = 0; m < nl; m++) {
      const long kl = (long)((((t.knew - 1 - m) % 4) + 4) % 4) * b.n2;   // knew of fast step iif-m
      L.p[L.n] = d.f.zeta + kl; L.nlev[L.n++] = 1;
      L.p[L.n] = d.f.ubar + kl; L.nlev[L.n++] = 1;
      L.p[L.n] = d.f.vbar + kl; L.nlev[L.n++] = 1;
    }
    L.w = 2 * K;
    launch_exchange_list(d, s, L);
    return;
  }
  const long kn = (long)(t.knew - 1) * b.n2;
  const ExchList L{{d.f.zeta + kn, d.f.ubar + kn, d.f.vbar + kn}, {1, 1, 1}, 3};
  Halo* H = const_cast<Halo*>(d.halo);
  if (H && H->overlap && t.iif < t.nfast && !d.p.s2d_split) {
    // overlap the exchange with the next fast step's interior tiles; that
    // step joins it before its rim tiles (the last fast step never forks)
    halo_fork_exchange(*H, s, L);
    return;
  }
  launch_exchange_list(d, s, L);
}

// one fast step's kernels over the bounds of d (launch_step2d): the fused
// step (or the split form), then the open / closed edges
void launch_fast_step(const Dev& d, hipStream_t s, const FBCoef& c, const Tlev& t) {
  const Bounds& b = d.b;
  const bool closed = b.west_edge || b.east_edge || b.south_edge || b.north_edge;
  Range RB{b.istrR, b.iendR, b.jstrR, b.jendR};
  // closed walls folded into k_s2d_fb when no edge is open and every edge
  // row / column shares its tile with the interior row / column beside it
  // (tiles start at tile_i0(istrR) / jstrR; ROMS_GPU_S2D_EDGES=1 keeps k_s2d_edges)
  const bool fold = closed && !d.p.obc && !d.p.s2d_split && d.p.s2d_fold &&
                    (!b.east_edge || (b.iendR - tile_i0(b.istrR)) % kBX != 0) &&
                    (!b.west_edge || (b.istrR - tile_i0(b.istrR)) % kBX != kBX - 1) &&
                    (!b.north_edge || (b.jendR - b.jstrR) % kBY != 0);
  const int cmode = !closed ? 0 : (fold ? 2 : 1);
  Halo* H = const_cast<Halo*>(d.halo);   // multi-rank exchange state (host bookkeeping)
  // single rank (no halo exchange object) with the fused kernel: periodic
  // halos of the fast-time fields are read through their images
  const int vwrap = (d.halo == nullptr && !d.p.s2d_split) ? (b.ew_periodic ? 1 : 0) | (b.ns_periodic ? 2 : 0) : 0;
  if (d.p.s2d_split) {  // two-kernel form (kept for A/B timing)
    Range RA{b.istrU - 1, b.iend, b.jstrV - 1, b.jend};
    hipLaunchKernelGGL(k_s2d_zeta, grid_of(RA), dim3(kBX, kBY), 0, s, d, RA, c);
    if (closed) {
      const int n = (b.jend - b.jstrV + 2) + (b.iend - b.istrU + 2);
      hipLaunchKernelGGL(k_s2d_zetabc, dim3((n + 255) / 256), dim3(256), 0, s, d, 0, c.kstp);
      hipLaunchKernelGGL(k_s2d_zetabc, dim3(1), dim3(64), 0, s, d, 1, c.kstp);
    }
    hipLaunchKernelGGL(k_s2d_mom, grid_of(RB), dim3(kBX, kBY), 0, s, d, RB, c);
  } else {
    auto fb = [&](int part) {
      const dim3 gr = grid_of(RB), bl(kBX, kBY);
#define S2D_FB(P, C, W) hipLaunchKernelGGL((k_s2d_fb<P, C, W>), gr, bl, 0, s, d, RB, c, vwrap, part)
      // the window form when roms_gpu_init set one up (ROMS_GPU_S2D_WIN=0: pointers)
#define S2D_FBW(C, W)                                                                                  \
  do {                                                                                                 \
    if (d.w2.base) hipLaunchKernelGGL((k_s2d_fb<false, C, W, 1, true>), gr, bl, 0, s, d, RB, c, vwrap, part); \
    else S2D_FB(false, C, W);                                                                          \
  } while (0)
      const bool wr = vwrap != 0;
      if (d.p.npip > 0) {
        if (cmode == 0) { if (wr) S2D_FB(true, 0, true); else S2D_FB(true, 0, false); }
        else if (cmode == 1) { if (wr) S2D_FB(true, 1, true); else S2D_FB(true, 1, false); }
        else { if (wr) S2D_FB(true, 2, true); else S2D_FB(true, 2, false); }
      } else {
        // store-flavour A/B on the two bench instances (C2: periodic, C3: closed walls folded in)
        static const int wt = [] { const char* e = getenv("ROMS_GPU_S2D_WT"); return e ? atoi(e) : 1; }();
        if (cmode == 0 && wr && wt == 0) hipLaunchKernelGGL((k_s2d_fb<false, 0, true, 0>), gr, bl, 0, s, d, RB, c, vwrap, part);
        else if (cmode == 0 && wr && wt == 2) hipLaunchKernelGGL((k_s2d_fb<false, 0, true, 2>), gr, bl, 0, s, d, RB, c, vwrap, part);
        else if (cmode == 2 && !wr && wt == 0) hipLaunchKernelGGL((k_s2d_fb<false, 2, false, 0>), gr, bl, 0, s, d, RB, c, vwrap, part);
        else if (cmode == 2 && !wr && wt == 2) hipLaunchKernelGGL((k_s2d_fb<false, 2, false, 2>), gr, bl, 0, s, d, RB, c, vwrap, part);
        else if (cmode == 0) { if (wr) S2D_FBW(0, true); else S2D_FBW(0, false); }
        else if (cmode == 1) { if (wr) S2D_FBW(1, true); else S2D_FBW(1, false); }
        else { if (wr) S2D_FBW(2, true); else S2D_FBW(2, false); }
      }
#undef S2D_FBW
#undef S2D_FB
    };
    // kernel-level timing: one interval per fast loop when nothing else runs
    // between the fused kernels (single rank, no closed edges), else one per launch
    const bool span = d.halo == nullptr && !closed;
    if (!span || t.iif == 1) ktimer_mark(s, kTimedS2dFb, 0);
    if (H && halo_pending(*H)) {
      // the previous fast step's zeta/ubar/vbar(knew) exchange is still in
      // flight on the halo stream: interior tiles first, the rim after it
      fb(1);
      halo_join(*H, s);
      fb(2);
    } else {
      fb(0);
    }
    if (!span) ktimer_mark(s, kTimedS2dFb, 1, 1);
    else if (t.iif == t.nfast) ktimer_mark(s, kTimedS2dFb, 1, t.nfast);
  }
  if (closed && !fold) {
    const int L = (b.Lm > b.Mm ? b.Lm : b.Mm) + 4 + 2 * b.gx;
    for (int ph = 0; ph < 4; ph++) {
      if (ph == 2 && !d.p.obc) continue;
      hipLaunchKernelGGL(k_s2d_edges, dim3(ph == 2 ? 1 : (4 * L + 255) / 256), dim3(ph == 2 ? 64 : 256), 0, s, d, c, ph);
    }
  }
}

}  // namespace roms
