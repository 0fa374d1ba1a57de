// halo.h -- multi-rank halo exchange and cross-rank gathers (halo.hip).
#pragma once
#include <string>
#include <vector>

#include "../../include/roms_gpu.h"
#include "roms_dev.h"

namespace roms {

enum HaloDir : int { kW = 0, kE, kS, kN, kSW, kSE, kNW, kNE };

// message geometry of one rank; passed to the pack/unpack kernels by value
struct HaloGeom {
  int Lm, Mm, nx2;
  long n2;
  int w;           // strip width: 2 (the reference's halo), 2*s2d_k for the fast loop's wide exchanges
  int j0, j1;      // rows of the W/E strips
  int i0, i1;      // columns of the S/N strips
  int active[8];   // neighbour present in direction d
  long cnt[8];     // elements per level of the message to/from direction d
  // the active directions in order: the pack / unpack grids hold one z-slice
  // per active direction (act_dir[blockIdx.z]) instead of 8 of which most
  // exit at once -- with exchanges running beside compute (deferred
  // exchanges) every empty block still took a dispatch slot from it
  int nact;
  int act_dir[8];
};
struct HaloPlan {
  HaloGeom g;
  int peer[8];     // rank of the neighbour in direction d (-1: none)
};

struct RomsComm;  // opaque communicator handle of the C ABI

// IPC transport (one process per GPU over an RCCL communicator): the pack
// kernel writes each message straight into the neighbour's receive buffer
// (IPC-mapped, uncached, double-buffered by exchange parity); a one-block
// kernel, ordered after the pack by the kernel boundary, raises the
// neighbours' arrival counters (system-scope release) and waits for the
// counters of this rank's receive slots (acquire; a timeout is fatal); then
// unpack.  Enabled only after a start-up self-test reproduced the RCCL
// exchange bitwise on every rank.
struct HaloIpc {
  double* rbuf2 = nullptr;              // [2 parities][8 slots][cap], written by the neighbours
  unsigned long long* flags = nullptr;  // [8] messages received per slot
  unsigned long long* seq = nullptr;    // exchanges completed by this rank
  int* err_dev = nullptr;               // set when a wait timed out (device copy)
  int* err_host = nullptr;              // same, host-mapped (host entries poll it)
  double* prbuf[8] = {};                // direction d's neighbour: its rbuf2
  unsigned long long* pflags[8] = {};   // ... and its flags
  std::vector<void*> opened;            // IPC mappings to close
  long long timeout_ticks = 0;          // wall_clock64 ticks before a wait gives up
  // test hook (ROMS_GPU_IPC_TEST_DROP=n): the n-th exchange after setup does
  // not signal its neighbours, so their waits time out (eager steps only)
  mutable long nexch = 0;
  long drop_at = -1;
  int ok = 0;
};

struct Halo {
  RomsComm* comm = nullptr;
  HaloPlan plan{};
  HaloPlan wide{};         // same neighbours, w-wide strips (ExchList::w > 2; wide.g.w == 0: none)
  long nexch = 0;          // exchanges enqueued since setup (host count; roms_gpu_exchange_count)
  double* sbuf = nullptr;  // 8 x cap send messages
  double* rbuf = nullptr;  // 8 x cap receive messages
  double* dred = nullptr;  // gather staging
  long cap = 0;
  long gcnt = 0;           // host channel: largest per-level message over all ranks
  // Exchanges forked onto the halo stream `cs` (halo_fork_exchange): each
  // gets a ticket (its fork count) and an event in a ring; the library stream
  // joins them back in ticket order (halo_join_to / halo_join).  cs runs them
  // in fork order, so joining ticket t joins every earlier one too.
  static constexpr int kRing = 16;
  hipStream_t cs = nullptr;
  hipEvent_t efork = nullptr;
  hipEvent_t xev[kRing] = {};
  long nfork = 0;   // exchanges forked onto cs since setup
  long njoin = 0;   // tickets < njoin are joined into the library stream
  hipStream_t ls = nullptr;   // the library stream (the only stream whose joins advance njoin)
  HaloIpc ipc;
  int overlap = 0;  // 1: enabled (ROMS_GPU_S2D_OVERLAP=1; off by default, see halo_setup)
  int overlap3d = 0;  // rim-first overlap of the 3-D exchanges (launch_rim_first; ROMS_GPU_OVERLAP3D=1: on)
  // Deferred 3-D exchanges (enqueue_step): on multi-rank runs
  // a producer's trailing exchange runs on cs beside the next routine that
  // reads none of its halo; the step joins it before the first reader.
  // xoverlap: enabled (the default with > 1 rank when no two ranks share a
  // device; ROMS_GPU_XOVERLAP=1 forces it on, =0 off; see halo_setup);
  // defer > 0: launch_exchange_list forks instead of exchanging on the
  // caller's stream (set around one producer).
  int xoverlap = 0;
  int defer = 0;
  // test hook (ROMS_GPU_XDELAY_US): each forked exchange's destination halo
  // is set to NaN, then a bounded spin of that many microseconds on cs holds
  // back its unpack, so a reader the step forgot to join reads NaN
  // (tests/test_gpu_multirank.py, tests/test_gpu_ipc.py)
  int xdelay_us = 0;
  long long xdelay_ticks = 0;
  // test hook (ROMS_GPU_XTEST_SKIPJOIN=bits): enqueue_step leaves out the
  // joins whose bit is set (1 before omega, 2 before pre_step3d, 4 before the
  // corrector's rho_eos, 8 before its omega, 16 before step3d_uv1), so the
  // tests can show that the delay hook catches each missing join (never set
  // outside tests/test_gpu_multirank.py)
  int xskip = 0;
};

int comm_unique_id(void* out128);
RomsComm* comm_create_rccl(const void* id128, int nranks, int rank, std::string& err);
RomsComm* comm_create_local(int group, int nranks, int rank);
RomsComm* comm_create_host(int nranks, int rank, roms_host_allgather_fn fn, void* ctx);
void comm_destroy(RomsComm* c);
int comm_rank(const RomsComm* c);
int comm_size(const RomsComm* c);

HaloPlan halo_plan(int Lm, int Mm, int npx, int npe, int inode, int jnode, int ewp, int nsp, int w = 2);
// wide: the w-wide plan of the fast loop (w == 0: none), wide_maxlev its largest list
int halo_setup(Halo& H, RomsComm* comm, const HaloPlan& plan, int maxlev, const HaloPlan& wide, int wide_maxlev,
               std::string& err);
void halo_free(Halo& H);
bool halo_graph_safe(const Halo* H);
long halo_map(const HaloPlan& P, int dir, int unpack, int* iv, int* jv);
void halo_exchange(const Halo& H, hipStream_t s, const ExchList& L);
// exchange L on H.cs after the work already queued on s (fork), returns its
// ticket; halo_join makes s wait for every forked exchange, halo_join_to for
// ticket t and those before it (no-ops for exchanges already joined)
long halo_fork_exchange(Halo& H, hipStream_t s, const ExchList& L);
void halo_join(Halo& H, hipStream_t s);
void halo_join_to(Halo& H, hipStream_t s, long ticket);
inline bool halo_pending(const Halo& H) { return H.nfork > H.njoin; }
int halo_allgather(const Halo& H, hipStream_t s, const double* in, int n, double* out);
// 1 if the IPC transport is in use, 0 if RCCL; -1 if a wait timed out since setup
int halo_transport(const Halo& H);
// true once an IPC wait timed out: the exchanges since are invalid (fatal)
bool halo_failed(const Halo& H);

}  // namespace roms
