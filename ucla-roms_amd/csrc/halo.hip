// halo.hip -- multi-rank halo exchange (mpi_exchanges.F:1-760 restated for
// one GPU per subdomain).
//
// An exchange of a list of arrays (one reference exchange_xxx(A,B,..) call)
// is pack -> transport -> unpack:
//   k_halo_pack   gathers, for each of the 8 neighbours (W,E,S,N,SW,SE,NW,NE),
//                 the 2-wide strip / 2x2 corner of every level of every array
//                 into one contiguous message (mpi_exchanges.F:533-598);
//   transport     IPC peer writes (see HaloIpc in halo.h; the default once a
//                 start-up self-test against RCCL passes), RCCL group
//                 send/recv on the library stream (capturable in a HIP graph),
//                 or, for several subdomains driven by threads of one
//                 process, device copies between their buffers;
//   k_halo_unpack scatters the received messages into the halo
//                 (mpi_exchanges.F:601-668).
// Every halo cell that has a neighbour receives that neighbour's current
// value (corners always travel), which is the superset of what the
// reference fills and equals the single-domain run's interior there.  Strips
// along a closed physical edge also carry the boundary ghost row/column, as
// the reference's jl0=0 / jl1=nyl+1 extension at the first/last jnode does.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include <unistd.h>

#include "halo.h"
#include "shim_state.h"

namespace roms {

namespace {
constexpr int kOpp[8] = {kE, kW, kN, kS, kNE, kNW, kSE, kSW};

// strips are g.w wide (2: the reference's halo; wider for the fast loop's
// exchanges); corners g.w x g.w
__host__ __device__ __forceinline__ void halo_src(const HaloGeom& g, int dir, long e, int& i, int& j) {
  const int nxs = g.i1 - g.i0 + 1, w = g.w;
  switch (dir) {
    case kW: i = 1 + (int)(e % w); j = g.j0 + (int)(e / w); break;
    case kE: i = g.Lm - w + 1 + (int)(e % w); j = g.j0 + (int)(e / w); break;
    case kS: i = g.i0 + (int)(e % nxs); j = 1 + (int)(e / nxs); break;
    case kN: i = g.i0 + (int)(e % nxs); j = g.Mm - w + 1 + (int)(e / nxs); break;
    case kSW: i = 1 + (int)(e % w); j = 1 + (int)(e / w); break;
    case kSE: i = g.Lm - w + 1 + (int)(e % w); j = 1 + (int)(e / w); break;
    case kNW: i = 1 + (int)(e % w); j = g.Mm - w + 1 + (int)(e / w); break;
    default: i = g.Lm - w + 1 + (int)(e % w); j = g.Mm - w + 1 + (int)(e / w); break;
  }
}
__host__ __device__ __forceinline__ void halo_dst(const HaloGeom& g, int h, long e, int& i, int& j) {
  const int nxs = g.i1 - g.i0 + 1, w = g.w;
  switch (h) {
    case kW: i = 1 - w + (int)(e % w); j = g.j0 + (int)(e / w); break;
    case kE: i = g.Lm + 1 + (int)(e % w); j = g.j0 + (int)(e / w); break;
    case kS: i = g.i0 + (int)(e % nxs); j = 1 - w + (int)(e / nxs); break;
    case kN: i = g.i0 + (int)(e % nxs); j = g.Mm + 1 + (int)(e / nxs); break;
    case kSW: i = 1 - w + (int)(e % w); j = 1 - w + (int)(e / w); break;
    case kSE: i = g.Lm + 1 + (int)(e % w); j = 1 - w + (int)(e / w); break;
    case kNW: i = 1 - w + (int)(e % w); j = g.Mm + 1 + (int)(e / w); break;
    default: i = g.Lm + 1 + (int)(e % w); j = g.Mm + 1 + (int)(e / w); break;
  }
}
// (array, level) of list-level index lev
__device__ __forceinline__ int list_slot(const ExchList& L, int& lev) {
  int q = 0;
  while (q < L.n - 1 && lev >= L.nlev[q]) { lev -= L.nlev[q]; q++; }
  return q;
}

// grid: x = element of the strip, y = list level, z = direction
__global__ void __launch_bounds__(256) k_halo_pack(HaloGeom g, ExchList L, double* __restrict__ sbuf, long cap) {
  const int dir = g.act_dir[blockIdx.z];
  if (!g.active[dir]) return;
  const long cnt = g.cnt[dir];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  int lev = blockIdx.y;
  const int q = list_slot(L, lev);
  if (lev >= L.nlev[q]) return;
  int i, j;
  halo_src(g, dir, e, i, j);
  sbuf[dir * cap + (long)blockIdx.y * cnt + e] = L.p[q][(long)(i + 1) + (long)(j + 1) * g.nx2 + (long)lev * g.n2];
}
__global__ void __launch_bounds__(256) k_halo_unpack(HaloGeom g, ExchList L, const double* __restrict__ rbuf, long cap) {
  const int h = g.act_dir[blockIdx.z];
  if (!g.active[h]) return;
  const long cnt = g.cnt[h];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  int lev = blockIdx.y;
  const int q = list_slot(L, lev);
  if (lev >= L.nlev[q]) return;
  int i, j;
  halo_dst(g, h, e, i, j);
  L.p[q][(long)(i + 1) + (long)(j + 1) * g.nx2 + (long)lev * g.n2] = rbuf[h * cap + (long)blockIdx.y * cnt + e];
}

// ---- IPC transport kernels (see HaloIpc in halo.h) ----
struct IpcPtrs {
  double* prbuf[8];
  unsigned long long* pflags[8];
  double* rbuf2;
  unsigned long long* flags;
  unsigned long long* seq;
  int* err_dev;     // device copy of the error state (read by every pack block)
  int* err_host;    // host-mapped copy (polled by the host entries without a sync)
  long long timeout;
};
// pack straight into the neighbour's slot opp(d) of parity seq&1.  After a
// failed wait (err_dev set) nothing more is written into a neighbour's
// buffers: a rank that gave up must not overwrite a slot the neighbour has
// not unpacked yet.
__global__ void __launch_bounds__(256) k_halo_pack_ipc(HaloGeom g, ExchList L, IpcPtrs P, long cap) {
  const int dir = g.act_dir[blockIdx.z];
  if (!g.active[dir] || *P.err_dev) return;
  const long cnt = g.cnt[dir];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long par = *P.seq & 1ull;
  int lev = blockIdx.y;
  const int q = list_slot(L, lev);
  if (e < cnt && lev < L.nlev[q]) {
    int i, j;
    halo_src(g, dir, e, i, j);
    P.prbuf[dir][((long)par * 8 + kOpp[dir]) * cap + (long)blockIdx.y * cnt + e] =
        L.p[q][(long)(i + 1) + (long)(j + 1) * g.nx2 + (long)lev * g.n2];
  }
}
// Signal + wait, one block.  The kernel boundary after k_halo_pack_ipc
// orders every block's payload stores (uncached, written through to the
// neighbour's memory) before this kernel runs; each active direction's
// neighbour then sees its arrival counter raised with a system-scope
// release.  Next, wait (acquire) until every active receive slot holds this
// exchange's message.  The wait is bounded (P.timeout; ROMS_GPU_IPC_TIMEOUT
// seconds): a timeout is fatal -- it sets the error state, which every later
// pack skips on and every host entry reports (roms_gpu_last_error) -- so a
// missing message never turns into silently stale halos.
__global__ void __launch_bounds__(64) k_halo_wait_ipc(HaloGeom g, IpcPtrs P, int nosignal) {
  const int h = threadIdx.x;
  const unsigned long long want = *P.seq + 1ull;
  const bool dead = *P.err_dev != 0;
  if (h < 8 && g.active[h] && !dead && !nosignal)
    __hip_atomic_fetch_add(P.pflags[h] + kOpp[h], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (h < 8 && g.active[h] && !dead) {
    // relaxed polls (system scope: uncached, always fresh), then ONE acquire
    // below: an acquire per poll invalidates this CU's caches every
    // iteration, and with the exchange running beside compute on the other
    // stream (deferred exchanges, enqueue_step) those polls cost the chip a
    // large share of its bandwidth (MI355X_MICROARCH.md: polling with acquire
    // loads; measured here 66.2 vs 61.4 ms per C3 step, 2 ranks on one GPU)
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(P.flags + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
      __builtin_amdgcn_s_sleep(8);
      if (wall_clock64() - t0 > P.timeout) {
        atomicExch(P.err_dev, 1);
        __hip_atomic_store(P.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: the payload the counters released
  __syncthreads();
  if (h == 0) *P.seq = want;
}
__global__ void __launch_bounds__(256) k_halo_unpack_ipc(HaloGeom g, ExchList L, IpcPtrs P, long cap) {
  const int h = g.act_dir[blockIdx.z];
  if (!g.active[h] || *P.err_dev) return;
  const long cnt = g.cnt[h];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  int lev = blockIdx.y;
  const int q = list_slot(L, lev);
  if (lev >= L.nlev[q]) return;
  const unsigned long long par = (*P.seq - 1ull) & 1ull;   // the wait kernel counted this exchange
  int i, j;
  halo_dst(g, h, e, i, j);
  L.p[q][(long)(i + 1) + (long)(j + 1) * g.nx2 + (long)lev * g.n2] =
      P.rbuf2[((long)par * 8 + h) * cap + (long)blockIdx.y * cnt + e];
}

// ---- in-process transport: subdomains driven by threads of one process ----
struct LocalGroup {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int waiting = 0;
  long gen = 0;
  std::vector<double*> sbuf;
  std::vector<std::vector<double>> red;
  long cap = 0;
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long my = gen;
    if (++waiting == n) {
      waiting = 0;
      gen++;
      cv.notify_all();
    } else if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != my; })) {
      // a rank never reached this collective: fail loudly rather than hang
      fprintf(stderr, "roms_gpu: in-process halo barrier timed out (mismatched collective calls)\n");
      std::abort();
    }
  }
};
std::mutex g_groups_m;
std::map<int, LocalGroup*> g_groups;
}  // namespace

struct RomsComm {
  int kind;  // 1 = RCCL, 2 = threads of one process, 3 = host channel (IPC halos)
  int rank, nranks;
  ncclComm_t nccl;
  LocalGroup* grp;
  int route_self;  // test hook: send self-messages through RCCL as well
  // kind 3: the host's own allgather (MPI_Allgather of bytes in a Fortran
  // host, mpi_exchanges.F's communicator); carries the IPC handles at setup
  // and the diag / area-volume gathers, never halo payloads
  roms_host_allgather_fn hfn;
  void* hctx;
};

int comm_unique_id(void* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}
RomsComm* comm_create_rccl(const void* id, int nranks, int rank, std::string& err) {
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
  if (r != ncclSuccess) {
    err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    return nullptr;
  }
  RomsComm* rc = new RomsComm{1, rank, nranks, c, nullptr, 0};
  const char* env = getenv("ROMS_GPU_RCCL_SELF");
  rc->route_self = env && env[0] == '1';
  return rc;
}
RomsComm* comm_create_host(int nranks, int rank, roms_host_allgather_fn fn, void* ctx) {
  return new RomsComm{3, rank, nranks, nullptr, nullptr, 0, fn, ctx};
}
RomsComm* comm_create_local(int group, int nranks, int rank) {
  std::lock_guard<std::mutex> lk(g_groups_m);
  LocalGroup*& gp = g_groups[group];
  if (!gp) {
    gp = new LocalGroup;
    gp->n = nranks;
    gp->sbuf.assign(nranks, nullptr);
    gp->red.assign(nranks, {});
  }
  return new RomsComm{2, rank, nranks, nullptr, gp, 0, nullptr, nullptr};
}
void comm_destroy(RomsComm* c) {
  if (!c) return;
  if (c->kind == 1) (void)ncclCommDestroy(c->nccl);
  delete c;
}
int comm_rank(const RomsComm* c) { return c ? c->rank : 0; }
int comm_size(const RomsComm* c) { return c ? c->nranks : 1; }

// neighbour table and message geometry from the processor grid (mpi_setup.F:59-139)
HaloPlan halo_plan(int Lm, int Mm, int npx, int npe, int inode, int jnode, int ewp, int nsp, int width) {
  HaloPlan P{};
  HaloGeom& g = P.g;
  g.Lm = Lm; g.Mm = Mm; g.nx2 = Lm + 4; g.n2 = (long)(Lm + 4) * (Mm + 4);
  g.w = width;
  const int w = width;
  const bool wn = ewp || inode > 0, e = ewp || inode < npx - 1;
  const bool s = nsp || jnode > 0, n = nsp || jnode < npe - 1;
  g.j0 = s ? 1 : 0; g.j1 = n ? Mm : Mm + 1;
  g.i0 = wn ? 1 : 0; g.i1 = e ? Lm : Lm + 1;
  const bool act[8] = {wn, e, s, n, s && wn, s && e, n && wn, n && e};
  const int di[8] = {-1, 1, 0, 0, -1, 1, -1, 1}, dj[8] = {0, 0, -1, 1, -1, -1, 1, 1};
  for (int d = 0; d < 8; d++) {
    g.active[d] = act[d];
    const int in = (inode + di[d] + npx) % npx, jn = (jnode + dj[d] + npe) % npe;
    P.peer[d] = act[d] ? in + jn * npx : -1;
    if (d < 2) g.cnt[d] = (long)w * (g.j1 - g.j0 + 1);
    else if (d < 4) g.cnt[d] = (long)w * (g.i1 - g.i0 + 1);
    else g.cnt[d] = (long)w * w;
    if (!act[d]) g.cnt[d] = 0;
  }
  g.nact = 0;
  for (int d = 0; d < 8; d++)
    if (act[d]) g.act_dir[g.nact++] = d;
  return P;
}

static void ipc_release(Halo& H);

// Host-staged exchange over a host-channel communicator (kind 3): the packed
// messages travel through the host's allgather (every rank's 8 messages in
// one fixed-size block of 8 x gcnt x nl doubles) and are scattered from the
// neighbours' blocks.  Only the IPC self-test uses it: it is the reference
// the peer-write transport must reproduce bitwise before it is enabled.
static int exchange_host(const Halo& H, hipStream_t s, const ExchList& L) {
  const HaloGeom& g = L.w > 2 ? H.wide.g : H.plan.g;
  RomsComm* c = H.comm;
  int nl = 0;
  for (int q = 0; q < L.n; q++) nl += L.nlev[q];
  long mx = 0;
  for (int d = 0; d < 8; d++) mx = g.cnt[d] > mx ? g.cnt[d] : mx;
  const dim3 grid((unsigned)((mx + 255) / 256), (unsigned)nl, (unsigned)(g.nact > 0 ? g.nact : 1));
  hipLaunchKernelGGL(k_halo_pack, grid, dim3(256), 0, s, g, L, H.sbuf, H.cap);
  const long m = H.gcnt * nl;
  std::vector<double> mine((size_t)8 * m, 0.0), all((size_t)8 * m * c->nranks);
  for (int d = 0; d < 8; d++)
    if (g.active[d] &&
        copy_on(mine.data() + d * m, H.sbuf + d * H.cap, (size_t)(nl * g.cnt[d]) * sizeof(double),
                hipMemcpyDeviceToHost, s) != hipSuccess)
      return -2;
  if (c->hfn(c->hctx, mine.data(), (long)((size_t)8 * m * sizeof(double)), all.data()) != 0) return -3;
  for (int h = 0; h < 8; h++)
    if (g.active[h] &&
        copy_on(H.rbuf + h * H.cap, all.data() + ((size_t)H.plan.peer[h] * 8 + kOpp[h]) * m,
                (size_t)(nl * g.cnt[h]) * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
      return -2;
  hipLaunchKernelGGL(k_halo_unpack, grid, dim3(256), 0, s, g, L, H.rbuf, H.cap);
  return hipStreamSynchronize(s) == hipSuccess ? 0 : -2;
}

// IPC transport setup: buffers, handle exchange (allgather over the RCCL
// communicator or the host channel), mapping of the neighbours' buffers, then a self-test that
// must reproduce the RCCL (host channel: host-staged) exchange bitwise on every rank (kSelfTestRounds
// exchanges of a two-level test field, alternating buffer parities, several
// exchanges queued back to back) before the transport is used.  Any failure
// anywhere leaves every rank on RCCL; every rank takes part in every
// collective whatever happened locally.
static void ipc_setup(Halo& H) {
  constexpr int kSelfTestRounds = 6;
  HaloIpc& I = H.ipc;
  RomsComm* c = H.comm;
  const int me = c->rank, nr = c->nranks;
  hipStream_t s = H.cs;   // created by halo_setup before this call
  double ok = 1.0;
  const size_t rbytes = (size_t)16 * H.cap * sizeof(double);
  if (hipExtMallocWithFlags((void**)&I.rbuf2, rbytes, hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&I.flags, 8 * sizeof(unsigned long long), hipDeviceMallocUncached) != hipSuccess ||
      hipMalloc(&I.seq, sizeof(unsigned long long)) != hipSuccess || hipMalloc(&I.err_dev, sizeof(int)) != hipSuccess ||
      hipHostMalloc((void**)&I.err_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    ok = 0.0;
  hipIpcMemHandle_t hr{}, hf{};
  if (ok != 0.0 && (hipMemset(I.rbuf2, 0, rbytes) != hipSuccess ||
                    hipMemset(I.flags, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
                    hipMemset(I.seq, 0, sizeof(unsigned long long)) != hipSuccess ||
                    hipMemset(I.err_dev, 0, sizeof(int)) != hipSuccess ||
                    hipStreamSynchronize(nullptr) != hipSuccess ||   // null-stream fills land first
                    hipIpcGetMemHandle(&hr, I.rbuf2) != hipSuccess ||
                    hipIpcGetMemHandle(&hf, I.flags) != hipSuccess))
    ok = 0.0;
  if (I.err_host) *I.err_host = 0;
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) ok = 0.0;
  double tsec = 60.0;   // ROMS_GPU_IPC_TIMEOUT: seconds a wait may take before the run fails
  {
    const char* e = getenv("ROMS_GPU_IPC_TIMEOUT");
    if (e && atof(e) > 0.0) tsec = atof(e);
  }
  I.timeout_ticks = (long long)((double)khz * 1000.0 * tsec);
  // handles of every rank: 2 x 64 B = 16 doubles, bit patterns carried as is
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  std::vector<double> mine(17), all((size_t)17 * nr);
  std::memcpy(mine.data(), &hr, 64);
  std::memcpy(mine.data() + 8, &hf, 64);
  mine[16] = ok;
  // (halo_allgather carries at most 64 doubles per rank)
  if (halo_allgather(H, s, mine.data(), 17, all.data()) != 0) ok = 0.0;
  for (int r = 0; r < nr; r++) ok = ok != 0.0 && all[(size_t)17 * r + 16] != 0.0 ? 1.0 : 0.0;
  // map each distinct neighbour once
  std::map<int, std::pair<double*, unsigned long long*>> peers;
  for (int d = 0; d < 8 && ok != 0.0; d++) {
    const int p = H.plan.peer[d];
    if (!H.plan.g.active[d] || p < 0) continue;
    if (p == me) { I.prbuf[d] = I.rbuf2; I.pflags[d] = I.flags; continue; }
    auto it = peers.find(p);
    if (it == peers.end()) {
      hipIpcMemHandle_t pr, pf;
      std::memcpy(&pr, all.data() + (size_t)17 * p, 64);
      std::memcpy(&pf, all.data() + (size_t)17 * p + 8, 64);
      void *a = nullptr, *b = nullptr;
      if (hipIpcOpenMemHandle(&a, pr, hipIpcMemLazyEnablePeerAccess) != hipSuccess) { ok = 0.0; break; }
      I.opened.push_back(a);
      if (hipIpcOpenMemHandle(&b, pf, hipIpcMemLazyEnablePeerAccess) != hipSuccess) { ok = 0.0; break; }
      I.opened.push_back(b);
      it = peers.emplace(p, std::make_pair((double*)a, (unsigned long long*)b)).first;
    }
    I.prbuf[d] = it->second.first;
    I.pflags[d] = it->second.second;
  }
  // agree on the mappings, then the self-test
  double v = ok;
  if (halo_allgather(H, s, &v, 1, all.data()) != 0) ok = 0.0;
  for (int r = 0; r < nr; r++) ok = ok != 0.0 && all[r] != 0.0 ? 1.0 : 0.0;
  if (ok != 0.0) {
    const long n2 = H.plan.g.n2, n = 2 * n2;
    std::vector<double*> A(kSelfTestRounds, nullptr), B(kSelfTestRounds, nullptr);
    std::vector<double> h(n), ha(n), hb(n);
    for (int r = 0; r < kSelfTestRounds; r++)
      if (hipMalloc(&A[r], n * sizeof(double)) != hipSuccess || hipMalloc(&B[r], n * sizeof(double)) != hipSuccess)
        ok = 0.0;
    for (int r = 0; r < kSelfTestRounds && ok != 0.0; r++) {
      for (long q = 0; q < n; q++) h[q] = 1.0e7 * (me + 1) + 1.0e3 * r + (double)q + 0.25;
      if (copy_on(A[r], h.data(), n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
          copy_on(B[r], h.data(), n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess) ok = 0.0;
    }
    if (ok != 0.0) {
      // the reference result: RCCL; then the IPC exchanges queued back to
      // back on the stream (both parities, no host sync in between)
      I.ok = 0;
      for (int r = 0; r < kSelfTestRounds; r++) {
        const ExchList LA{{A[r]}, {2}, 1};
        if (c->kind == 3) {
          if (exchange_host(H, s, LA) != 0) ok = 0.0;
        } else {
          halo_exchange(H, s, LA);
        }
      }
      I.ok = 1;
      for (int r = 0; r < kSelfTestRounds; r++) halo_exchange(H, s, ExchList{{B[r]}, {2}, 1});
      I.ok = 0;
      if (hipStreamSynchronize(s) != hipSuccess || *I.err_host != 0) ok = 0.0;
      for (int r = 0; r < kSelfTestRounds && ok != 0.0; r++) {
        if (copy_on(ha.data(), A[r], n * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
            copy_on(hb.data(), B[r], n * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
            std::memcmp(ha.data(), hb.data(), n * sizeof(double)) != 0)
          ok = 0.0;
      }
    }
    for (int r = 0; r < kSelfTestRounds; r++) {
      if (A[r]) (void)hipFree(A[r]);
      if (B[r]) (void)hipFree(B[r]);
    }
    v = ok;
    if (halo_allgather(H, s, &v, 1, all.data()) != 0) ok = 0.0;
    for (int r = 0; r < nr; r++) ok = ok != 0.0 && all[r] != 0.0 ? 1.0 : 0.0;
  }
  (void)hipStreamSynchronize(s);
  if (ok != 0.0) {
    I.ok = 1;
    const char* e = getenv("ROMS_GPU_IPC_TEST_DROP");
    I.drop_at = e ? atol(e) : -1;
    I.nexch = 0;
  } else {
    ipc_release(H);
  }
}

int halo_transport(const Halo& H) {
  if (!H.ipc.ok) return 0;
  return halo_failed(H) ? -1 : 1;
}
bool halo_failed(const Halo& H) {
  return H.ipc.ok && H.ipc.err_host && __atomic_load_n(H.ipc.err_host, __ATOMIC_ACQUIRE) != 0;
}

// every rank's (host, PCI location of its device) through the halo gather:
// distinct = 1 when no two ranks share a device
static int ranks_on_distinct_devices(const Halo& H, int& distinct) {
  distinct = 0;
  int dev = 0;
  hipDeviceProp_t p{};
  double key[2] = {-1.0, -1.0};
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
    key[0] = (double)p.pciDomainID * 65536.0 + (double)p.pciBusID * 256.0 + (double)p.pciDeviceID;
  char host[256] = {0};
  (void)gethostname(host, sizeof(host) - 1);
  unsigned h = 2166136261u;   // FNV-1a of the host name
  for (const char* c = host; *c; c++) h = (h ^ (unsigned char)*c) * 16777619u;
  key[1] = (double)h;
  const int nr = H.comm->nranks;
  std::vector<double> all((size_t)2 * nr);
  if (halo_allgather(H, H.cs, key, 2, all.data()) != 0) return -1;
  std::set<std::pair<double, double>> seen;
  for (int r = 0; r < nr; r++) {
    if (all[2 * r] < 0.0) return 0;   // a rank could not tell its device: keep the in-place order
    seen.insert({all[2 * r], all[2 * r + 1]});
  }
  distinct = (int)seen.size() == nr ? 1 : 0;
  return 0;
}

int halo_setup(Halo& H, RomsComm* comm, const HaloPlan& plan, int maxlev, const HaloPlan& wide, int wide_maxlev,
               std::string& err) {
  H.comm = comm;
  H.plan = plan;
  H.wide = wide;
  H.nexch = 0;
  long mx = 0, mxw = 0;
  for (int d = 0; d < 8; d++) mx = plan.g.cnt[d] > mx ? plan.g.cnt[d] : mx;
  if (wide.g.w > 0)
    for (int d = 0; d < 8; d++) mxw = wide.g.cnt[d] > mxw ? wide.g.cnt[d] : mxw;
  // one slot of a message buffer holds the largest message of either plan
  H.cap = mx * (long)maxlev > mxw * (long)wide_maxlev ? mx * (long)maxlev : mxw * (long)wide_maxlev;
  if (hipMalloc(&H.sbuf, (size_t)8 * H.cap * sizeof(double)) != hipSuccess ||
      hipMalloc(&H.rbuf, (size_t)8 * H.cap * sizeof(double)) != hipSuccess ||
      hipMalloc(&H.dred, (size_t)64 * (1 + (comm ? comm->nranks : 1)) * sizeof(double)) != hipSuccess) {
    err = "halo_setup: hipMalloc failed";
    return -2;
  }
  if (hipStreamCreateWithFlags(&H.cs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&H.efork, hipEventDisableTiming) != hipSuccess) {
    err = "halo_setup: stream/event creation failed";
    return -2;
  }
  for (hipEvent_t& e : H.xev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      err = "halo_setup: event creation failed";
      return -2;
    }
  H.nfork = H.njoin = 0;
  H.defer = 0;
  {
    // deferred 3-D exchanges beside the next routine (enqueue_step): on by
    // default when every rank has a GPU of its own (decided at the end of
    // this function), ROMS_GPU_XOVERLAP=1 / =0 forces either order.  Ranks
    // sharing one MI355X measured slower deferred: one
    // process exchanging with itself through IPC, C2, 7.12 vs 6.92-6.95 ms
    // per step; 2 and 4 ranks sharing the GPU, C3, 63-75 vs 57-58 ms -- there
    // the forked pack / wait / unpack kernels compete with the routine they
    // would hide behind and there is no xGMI latency to hide.  bench.py
    // --gpus N > 1 reports both orders
    const char* ex = getenv("ROMS_GPU_XOVERLAP");
    if (ex && (ex[0] == '0' || ex[0] == '1')) H.xoverlap = ex[0] == '1' && comm && comm->nranks > 1;
    else H.xoverlap = -1;   // decided below, once every rank's device is known
    const char* es = getenv("ROMS_GPU_XTEST_SKIPJOIN");
    H.xskip = es ? atoi(es) : 0;
    const char* ed = getenv("ROMS_GPU_XDELAY_US");
    H.xdelay_us = ed ? atoi(ed) : 0;
    if (H.xdelay_us < 0 || H.xdelay_us > 100000) H.xdelay_us = 0;
    int khz = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (H.xdelay_us && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
      H.xdelay_ticks = (long long)khz * H.xdelay_us / 1000;
    else
      H.xdelay_us = 0;
  }
  {
    // measured on one MI355X with every exchange routed through RCCL: the
    // overlap costs more than it hides (13.8 vs 12.9 ms/step at C2: the RCCL
    // kernel competes with the interior tiles for CUs, and the fast step
    // becomes two launches), so it is opt-in: ROMS_GPU_S2D_OVERLAP=1
    const char* e = getenv("ROMS_GPU_S2D_OVERLAP");
    H.overlap = e && e[0] == '1';
    // rim-first 3-D overlap (launch_rim_first): measured with the exchanges
    // routed through the IPC transport on one MI355X it costs more than it
    // hides (C2 9.04 -> 11.10 ms/step: the four rim launches of a column
    // kernel each take a whole column walk's latency, ~40 us, against ~20 us
    // per exchange), so it is opt-in: ROMS_GPU_OVERLAP3D=1
    const char* e3 = getenv("ROMS_GPU_OVERLAP3D");
    H.overlap3d = e3 && e3[0] == '1';
  }
  if (comm && comm->kind == 2) {
    std::lock_guard<std::mutex> lk(comm->grp->m);
    comm->grp->sbuf[comm->rank] = H.sbuf;
    comm->grp->cap = H.cap;
  }
  if (comm && comm->kind == 1) {
    const char* e = getenv("ROMS_GPU_HALO_IPC");
    if (!(e && e[0] == '0')) ipc_setup(H);
  }
  if (comm && comm->kind == 3) {
    // the host-staged self-test blocks: every rank uses the largest message of any rank
    double mine = (double)(mx > mxw ? mx : mxw);
    std::vector<double> all((size_t)comm->nranks);
    if (halo_allgather(H, H.cs, &mine, 1, all.data()) != 0) {
      err = "halo_setup: host-channel allgather failed";
      return -5;
    }
    for (double v : all) H.gcnt = (long)v > H.gcnt ? (long)v : H.gcnt;
    ipc_setup(H);
    if (!H.ipc.ok) {
      err = "halo_setup: the IPC halo transport of the host-channel communicator failed its setup or self-test "
            "(use roms_gpu_comm_create for RCCL)";
      return -5;
    }
  }
  if (H.xoverlap < 0) {
    // default: deferred exchanges when every rank drives a GPU of its own
    // (one process per GPU over xGMI: a deferred exchange's latency hides
    // behind the next routine).  Ranks that share a device (a rehearsal with
    // more ranks than GPUs) or threads of one process keep the in-place
    // order: there the forked kernels compete with the routine they would
    // hide behind, and measured slower.
    int distinct = 0;
    if (comm && comm->nranks > 1 && (comm->kind == 1 || comm->kind == 3)) {
      const int r = ranks_on_distinct_devices(H, distinct);
      if (r) {
        err = "halo_setup: device-identity gather failed";
        return -5;
      }
    }
    H.xoverlap = distinct;
  }
  H.nexch = 0;   // the self-test's exchanges do not count
  return 0;
}
static void ipc_release(Halo& H) {
  HaloIpc& I = H.ipc;
  for (void* p : I.opened) (void)hipIpcCloseMemHandle(p);
  I.opened.clear();
  if (I.rbuf2) (void)hipFree(I.rbuf2);
  if (I.flags) (void)hipFree(I.flags);
  if (I.seq) (void)hipFree(I.seq);
  if (I.err_dev) (void)hipFree(I.err_dev);
  if (I.err_host) (void)hipHostFree(I.err_host);
  I = HaloIpc{};
}
void halo_free(Halo& H) {
  ipc_release(H);
  if (H.sbuf) (void)hipFree(H.sbuf);
  if (H.rbuf) (void)hipFree(H.rbuf);
  if (H.dred) (void)hipFree(H.dred);
  H.sbuf = H.rbuf = H.dred = nullptr;
  if (H.efork) (void)hipEventDestroy(H.efork);
  for (hipEvent_t& e : H.xev) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  if (H.cs) (void)hipStreamDestroy(H.cs);
  H.efork = nullptr;
  H.cs = nullptr;
  H.nfork = H.njoin = 0;
  H.defer = 0;
}

// host copy of the pack (unpack=0) or unpack (unpack=1) index map of one direction
long halo_map(const HaloPlan& P, int dir, int unpack, int* iv, int* jv) {
  const long n = P.g.cnt[dir];
  for (long e = 0; e < n; e++) {
    if (unpack) halo_dst(P.g, dir, e, iv[e], jv[e]);
    else halo_src(P.g, dir, e, iv[e], jv[e]);
  }
  return n;
}

bool halo_graph_safe(const Halo* H) { return !H || !H->comm || H->comm->kind == 1 || H->comm->kind == 3; }

namespace {
IpcPtrs ipc_ptrs(const Halo& H) {
  IpcPtrs P;
  for (int d = 0; d < 8; d++) { P.prbuf[d] = H.ipc.prbuf[d]; P.pflags[d] = H.ipc.pflags[d]; }
  P.rbuf2 = H.ipc.rbuf2; P.flags = H.ipc.flags; P.seq = H.ipc.seq;
  P.err_dev = H.ipc.err_dev; P.err_host = H.ipc.err_host;
  P.timeout = H.ipc.timeout_ticks;
  return P;
}
// test hook (Halo::xdelay_us): one lane spins for `ticks` wall-clock ticks
// (bounded: it ends by itself), so the unpack that follows lands late
__global__ void k_halo_delay(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
// ... and before the delay every halo cell the unpack will fill is set to
// NaN, so a routine that reads the halo before its join reads NaN -- even
// where the stale and the fresh values agree -- and the run shows it
__global__ void __launch_bounds__(256) k_halo_poison(HaloGeom g, ExchList L) {
  const int h = g.act_dir[blockIdx.z];
  if (!g.active[h]) return;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.cnt[h]) return;
  int lev = blockIdx.y;
  const int q = list_slot(L, lev);
  if (lev >= L.nlev[q]) return;
  int i, j;
  halo_dst(g, h, e, i, j);
  L.p[q][(long)(i + 1) + (long)(j + 1) * g.nx2 + (long)lev * g.n2] = __builtin_nan("");
}
void xdelay(const Halo& H, hipStream_t s, const HaloGeom& g, const ExchList& L, const dim3& grid) {
  if (H.xdelay_us > 0 && s == H.cs) {
    hipLaunchKernelGGL(k_halo_poison, grid, dim3(256), 0, s, g, L);
    hipLaunchKernelGGL(k_halo_delay, dim3(1), dim3(64), 0, s, H.xdelay_ticks);
  }
}
void exchange_ipc(const Halo& H, hipStream_t s, const HaloGeom& g, const ExchList& L, const dim3& grid) {
  const IpcPtrs P = ipc_ptrs(H);
  ktimer_mark(s, kTimedHaloPack, 0);
  hipLaunchKernelGGL(k_halo_pack_ipc, grid, dim3(256), 0, s, g, L, P, H.cap);
  ktimer_mark(s, kTimedHaloPack, 1, 1);
  const int drop = H.ipc.drop_at >= 0 && H.ipc.nexch++ == H.ipc.drop_at;
  ktimer_mark(s, kTimedHaloWait, 0);
  hipLaunchKernelGGL(k_halo_wait_ipc, dim3(1), dim3(64), 0, s, g, P, drop);
  ktimer_mark(s, kTimedHaloWait, 1, 1);
  xdelay(H, s, g, L, grid);
  ktimer_mark(s, kTimedHaloUnpack, 0);
  hipLaunchKernelGGL(k_halo_unpack_ipc, grid, dim3(256), 0, s, g, L, P, H.cap);
  ktimer_mark(s, kTimedHaloUnpack, 1, 1);
}
}  // namespace

void halo_exchange(const Halo& H, hipStream_t s, const ExchList& L) {
  const HaloGeom& g = L.w > 2 ? H.wide.g : H.plan.g;
  if (L.w > 2 && g.w != L.w) {
    fprintf(stderr, "roms_gpu: %d-wide exchange without a matching halo plan (wide plan %d)\n", L.w, g.w);
    std::abort();
  }
  int nl = 0;
  for (int q = 0; q < L.n; q++) nl += L.nlev[q];
  if (nl == 0) return;
  const_cast<Halo&>(H).nexch++;
  long mx = 0;
  for (int d = 0; d < 8; d++) mx = g.cnt[d] > mx ? g.cnt[d] : mx;
  const dim3 grid((unsigned)((mx + 255) / 256), (unsigned)nl, (unsigned)(g.nact > 0 ? g.nact : 1));
  if (H.ipc.ok) {
    exchange_ipc(H, s, g, L, grid);
    return;
  }
  ktimer_mark(s, kTimedHaloPack, 0);
  hipLaunchKernelGGL(k_halo_pack, grid, dim3(256), 0, s, g, L, H.sbuf, H.cap);
  ktimer_mark(s, kTimedHaloPack, 1, 1);
  RomsComm* c = H.comm;
  const int me = c->rank;
  ktimer_mark(s, kTimedHaloWait, 0);
  if (c->kind == 1) {
    (void)ncclGroupStart();
    for (int d = 0; d < 8; d++)
      if (g.active[d] && (H.plan.peer[d] != me || c->route_self))
        (void)ncclSend(H.sbuf + d * H.cap, (size_t)(nl * g.cnt[d]), ncclDouble, H.plan.peer[d], c->nccl, s);
    // the k-th message to a peer lands in the k-th receive posted for it:
    // receive halo opp(d) in the order the peer sent direction d
    for (int d = 0; d < 8; d++) {
      const int h = kOpp[d];
      if (g.active[h] && (H.plan.peer[h] != me || c->route_self))
        (void)ncclRecv(H.rbuf + h * H.cap, (size_t)(nl * g.cnt[h]), ncclDouble, H.plan.peer[h], c->nccl, s);
    }
    (void)ncclGroupEnd();
    for (int h = 0; h < 8; h++)
      if (g.active[h] && H.plan.peer[h] == me && !c->route_self)
        (void)hipMemcpyAsync(H.rbuf + h * H.cap, H.sbuf + kOpp[h] * H.cap, (size_t)(nl * g.cnt[h]) * sizeof(double),
                             hipMemcpyDeviceToDevice, s);
  } else if (c->kind == 3) {
    (void)exchange_host(H, s, L);   // setup failed; roms_gpu_init has already returned the error
    return;
  } else {
    LocalGroup* G = c->grp;
    (void)hipStreamSynchronize(s);
    G->barrier();
    for (int h = 0; h < 8; h++)
      if (g.active[h])
        (void)hipMemcpyAsync(H.rbuf + h * H.cap, G->sbuf[H.plan.peer[h]] + kOpp[h] * G->cap,
                             (size_t)(nl * g.cnt[h]) * sizeof(double), hipMemcpyDeviceToDevice, s);
    (void)hipStreamSynchronize(s);
    G->barrier();
  }
  ktimer_mark(s, kTimedHaloWait, 1, 1);
  xdelay(H, s, g, L, grid);
  ktimer_mark(s, kTimedHaloUnpack, 0);
  hipLaunchKernelGGL(k_halo_unpack, grid, dim3(256), 0, s, g, L, H.rbuf, H.cap);
  ktimer_mark(s, kTimedHaloUnpack, 1, 1);
}

long halo_fork_exchange(Halo& H, hipStream_t s, const ExchList& L) {
  // a ring event is recorded again only after the library stream has joined
  // the exchange it marked
  if (H.nfork - H.njoin >= Halo::kRing) halo_join_to(H, s, H.nfork - Halo::kRing);
  (void)hipEventRecord(H.efork, s);
  (void)hipStreamWaitEvent(H.cs, H.efork, 0);
  halo_exchange(H, H.cs, L);
  (void)hipEventRecord(H.xev[H.nfork % Halo::kRing], H.cs);
  return H.nfork++;
}
void halo_join_to(Halo& H, hipStream_t s, long ticket) {
  if (ticket < H.njoin || ticket >= H.nfork) return;
  (void)hipStreamWaitEvent(s, H.xev[ticket % Halo::kRing], 0);
  // njoin counts the library stream's joins only: a side stream that waits
  // for an exchange does not make it joined for the library stream
  if (s == H.ls || !H.ls) H.njoin = ticket + 1;
}
void halo_join(Halo& H, hipStream_t s) { halo_join_to(H, s, H.nfork - 1); }

// out[r*n + q] = in_r[q] for every rank r (blocking)
int halo_allgather(const Halo& H, hipStream_t s, const double* in, int n, double* out) {
  RomsComm* c = H.comm;
  if (!c) {
    std::memcpy(out, in, (size_t)n * sizeof(double));
    return 0;
  }
  if (n > 64) return -1;
  if (c->kind == 3) {
    if (hipStreamSynchronize(s) != hipSuccess) return -2;
    return c->hfn(c->hctx, in, (long)((size_t)n * sizeof(double)), out) == 0 ? 0 : -3;
  }
  if (c->kind == 1) {
    double* dsend = H.dred;        // 64 doubles
    double* dall = H.dred + 64;    // 64 * nranks doubles
    if (hipMemcpyAsync(dsend, in, (size_t)n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess) return -2;
    if (ncclAllGather(dsend, dall, (size_t)n, ncclDouble, c->nccl, s) != ncclSuccess) return -3;
    if (hipMemcpyAsync(out, dall, (size_t)n * c->nranks * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess)
      return -2;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -2;
  }
  LocalGroup* G = c->grp;
  {
    std::lock_guard<std::mutex> lk(G->m);
    G->red[c->rank].assign(in, in + n);
  }
  G->barrier();
  for (int r = 0; r < c->nranks; r++) std::memcpy(out + (long)r * n, G->red[r].data(), (size_t)n * sizeof(double));
  G->barrier();
  return 0;
}

}  // namespace roms
