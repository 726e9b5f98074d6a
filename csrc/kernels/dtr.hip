// Device task runtime (DTR): a whole tile Cholesky as ONE persistent launch whose workgroups pull
// tasks from device-resident, priority-ordered ready lists -- the device-side counterpart of the
// reference's PTG runtime with its high_priority task classes (src/zpotrf_L.jdf:58-69, 93, 194, 306;
// PaRSEC orders ready tasks by priority when a core/stream frees up).
//
// Why: a HIP stream priority does not give a kernel CU resources that another kernel holds.  Beside
// the bulk trailing-update GEMM (2 workgroups x 72 KB LDS + 2 x 128 VGPR waves per SIMD on every CU),
// the register-resident panel solve (256-VGPR waves) is not dispatched until the GEMM has drained
// (tools/gpu/prio_probe.py, profiles/r4_prio_probe.txt: the panel TRSM takes 0.43 ms alone and 34.5 ms
// beside a 34.3 ms GEMM -- also with the GEMM capped to its resident 512 workgroups, so it is not the
// dispatch queue).
// Here the panel work runs INSIDE the GEMM's resident workgroups: every workgroup, when it finishes a
// task, takes the next ready task of the high-priority list (diagonal tile factorisation + inverse,
// panel solve, look-ahead updates) before any bulk update.
//
// Tasks (fp64, lower, NB = 512, N a multiple of 512; A column-major, ld N):
//   UPD(i, j, r, c, k0, nk): 128x128 sub-tile (r, c) of tile (i, j) -= sum_{k0 <= k < k0+nk}
//       L(i,k)[strip r] L(j,k)[strip c]^T   (gemm_tile.h, 2 x 128 VGPR waves/SIMD, 72 KB LDS)
//   TRSM(i, k, r): 128-row strip r of L(i,k) := A(i,k)[strip r] W_k, W_k = L_kk^{-T} -- four
//       sub-tile GEMMs against the upper-triangular W_k, column blocks 3, 2, 1, 0 in that order so
//       the strip is solved IN PLACE (block c reads columns < 128(c+1) only, which no later block of
//       the sequence overwrites)
//   POTRF(k, b): row block b (32 rows) of the dataflow tile Cholesky (potrf_tile.h; 16 cooperating
//       workgroups), then block column b of W_k (TRTRI below, same dataflow).
//   SEND(i, k, r, dest) / SENDW(k, c, dest) (P x Q grids, models/potrf_dtr_dist.py): strip r of the
//       solved panel tile (i, k) / column block c of W_k into rank dest's receive buffer / W, then one
//       bump of dest's counter -- a remote strip is an arrival requirement of the consumer's tasks.
// Two schedulers share the task bodies:
//  * k_dtr_q (default, DPLASMA_DTR_SCHED=queue): PUSH scheduling.  The host turns the requirement lists into
//    task edges (models/potrf_dtr.py queue_edges); a task is pushed into a ready ring -- one FIFO per (class,
//    XCD), class = its bottom level (longest path of task durations to the end) bucketed, POTRF blocks first --
//    by the workgroup that completes its last predecessor; idle workgroups scan all rings with one ballot per 64
//    and pop the best.  Across ranks a send decrements its remote consumers' pending counts and pushes them into
//    the peer's rings through the IPC mapping (system scope).  No ready task waits behind a list head
//    (profiles/r5_dtr_queue.txt: 16k 45.8 -> 48.8 TF/s; 2x4 64k emulated 17-30 % -> 74.8 %).
//  * k_dtr_potrf (DPLASMA_DTR_SCHED=lists): the static lists below.
// Dependencies of the list scheduler are tile-version counters, not successor lists: each task lists (counter, target)
// requirements (a 128x128 sub-tile's number of completed writes, a panel strip's "solved" mark, the
// number of finished W_k block columns) and bumps one counter when done.  A list's head is claimed
// (CAS on the list cursor) only when ready, so tasks start in list order and nobody ever waits
// inside a task except the 16 POTRF(k, *) workgroups, claimed in order (block b only waits on
// blocks < b, already running).  Both lists are subsequences of one topological order with the
// low lists sorted by panel block first, so the earliest unclaimed task is always the head of its
// list with every predecessor claimed: the schedule cannot deadlock (models/potrf_dtr.py).
// The bulk updates sit in one low list per XCD (consecutive sub-tiles of a tile share operand
// strips in that XCD's L2); a workgroup steals from another XCD's list only once its own is empty.
//
// Hand-offs between tasks (MI355X_MICROARCH.md, inter-workgroup visibility): producer -- every wave
// s_waitcnt vmcnt(0), barrier, lane 0 agent release fence, s_waitcnt, relaxed agent atomic add;
// consumer -- relaxed sc1 polls of the requirement counters, the claim, lane 0 agent acquire fence
// + s_waitcnt, barrier.  Every wait is bounded (info = -1000, all workgroups drain).  Between processes
// (one rank per GPU, peers' buffers IPC-mapped) the same with system scope: sc0 sc1 stores of the sent
// bytes, a system release, a system-scope counter add on the peer; system-scope polls and acquire.
//
// Multi-rank modes (DtrArgs.nranks > 1): rank >= 0 -- this launch is one rank of a P x Q grid; rank = -1
// -- EMULATION of the grid on one GPU: XCD x is rank x * nranks / 8's "GPU", every rank has its own tile
// storage, receive buffers, W and counters, and time is dilated by nranks (a task's completion becomes
// visible (nranks - 1) x its duration after it ends, through a per-counter visibility time; a send is
// visible nranks x (lat + bytes / bw) after its rank pair's link frees up), so the span / nranks models
// the grid's run on nranks GPUs (tools/emulate_potrf.py).
#include <cstddef>
#include <cstring>

#include "gemm_tile.h"
#include "potrf_tile.h"

namespace {
using namespace rbk;

enum : int { T_UPD = 0, T_TRSM = 1, T_POTRF = 2, T_SEND = 3, T_SENDW = 4 };
constexpr int MAXR = 8;     // ranks of one launch (emulation) / of a grid (process mode)

struct DtrTask {      // 32 bytes
  int type;
  int i, j;           // UPD: tile (i, j); TRSM: tile (i, k0); POTRF: -; SEND: tile row i, j = destination rank
  int k0;             // first panel (TRSM / POTRF / SEND / SENDW: the panel)
  int req_beg;        // requirements [req_beg, req_beg + nreq): (counter, target) pairs
  int inc;            // counter bumped on completion (-1: none); SEND / SENDW: on the destination rank
  short r, c;         // UPD: sub-tile; TRSM / SEND: strip r; POTRF: block row r; SENDW: column block r
  short nk, nreq;     // UPD: panels in the run
};
static_assert(sizeof(DtrTask) == 32, "DtrTask layout");

struct DtrArgs {
  long long ld;             // leading dimension of every tile (local, received) -- 512: TILE storage
  int nt;
  int nranks;               // 1: one process, one rank; > 1: grid (process mode or emulation)
  int rank;                 // >= 0: this launch's rank; -1: emulation (rank from the XCD)
  int epoch;
  int flags;                // bit 0: steal a ready head of another XCD's list when the own head is not ready;
                            // bits 8-15 / 16-23: how long a ticket holder polls before helping (see below);
                            // bits 24-27: high-list segments scanned per claim (0: 8)
  int dil;                  // emulation: time dilation (= nranks); 1 otherwise
  long long ncnt;           // counters per rank
  const DtrTask* tasks;
  const int2* reqs;
  const long long* tab;     // per rank nt x nt: element offset (from the rank's A) of tile (i, j) at i + j nt
  const long long* xoff;    // per task: SEND / SENDW destination element offset (receive buffer / W)
  int* cur;                 // cursors: [r] step low-water mark of rank r, [MAXR + x] low list of XCD x; PSTRIDE apart
  const int* hi;            // high lists (task ids), rank r's at [hi_off[r], hi_off[r + 1])
  int hi_off[MAXR + 1];
  int nsteps;               // each rank's high list is nsteps FIFO segments (list order "step": one per panel)
  const int* hs_off;        // per rank nsteps + 1 segment offsets (relative to hi_off[r])
  int* scur;                // per rank x segment ticket cursors, PSTRIDE ints apart
  const int* lo;            // low lists, XCD x's at [lo_off[x], lo_off[x + 1])
  int lo_off[9];
  double* A[MAXR];          // rank r's tile storage base (process mode: [rank] only)
  double* recv[MAXR];       // rank r's receive buffer (process mode: IPC-mapped peers)
  double* W[MAXR];          // rank r's W: nt x (512 x 512), W_k = L_kk^{-T}
  int* cnt[MAXR];           // rank r's version / arrival counters (zeroed per launch)
  unsigned long long* vis;  // emulation: per rank ncnt visibility times (100 MHz ticks)
  unsigned long long* link; // emulation: MAXR x MAXR "link free at" times
  long long bw_bpt;         // emulation: link bytes per tick (GB/s x 10)
  long long lat_t;          // emulation: link latency (ticks)
  double* Mw;               // nt x MAXB x BLK     (M_k of the 32-blocks, potrf_tile.h)
  double* Sw;               // nt x MAXB x RB
  double* Lp;               // nt x MAXB x MAXB x BLK  (published L(b, m) blocks, T-layout)
  double* Wp;               // nt x MAXB x MAXB x BLK  (published W blocks, T-layout)
  int* prog;                // nt x 2 x MAXB x PSTRIDE: tile-step flags, then W-column flags
  int* info;
  long long* trace;         // optional (DPLASMA_DTR_TRACE): per task {start, end, wg << 8 | xcd, visible}, 100 MHz ticks
  // ---- push scheduling (k_dtr_q): per-task pending-predecessor counts, successor lists, ready rings
  int ntask;                // tasks this launch runs (this rank's)
  int nclass;               // priority classes (ring r = class * 8 + XCD; lower class first)
  int* pend[MAXR];          // rank r's per-task (global ids) predecessors not yet complete (reset per launch)
  const int* succ_off;      // global task ids: successors [succ_off[t], succ_off[t + 1])
  const int* succ;
  const int* ring_of;       // per task: the ready ring it is pushed to (on its owner)
  const int* town;          // per task: owner rank (null: one rank)
  const int* qbase;         // per rank nclass * 8 + 1 slot offsets
  int* qctl[MAXR];          // rank r's rings: head at [2 q PSTRIDE], tail at [(2 q + 1) PSTRIDE] (reset per launch)
  int* qslot[MAXR];         // rank r's ring slots: task id + 1, 0 = reserved but not yet written (reset per launch)
  int* done;                // tasks completed by this launch
  unsigned long long* rdy;  // emulation: per task, when its last input becomes visible (max over predecessors)
  // optional hazard probe (DPLASMA_DTR_PROBE=1, the two-workgroups-per-CU hunt, profiles/r6_dtr_probe.txt):
  // [0] record count, [8, 8 + 4 nt * nt) per strip (4 i + r, k) the epoch stamped by its TRSM before its release,
  // then 8-word records of every diagonal-tile update that saw a strip operand stale (see probe_strips)
  long long* probe;
  double* snap;             // optional (with probe): nt x 512 x 512 copy of every diagonal tile's POTRF input
};

constexpr int NBT = 512;    // tile size
constexpr int LDS_D = 2 * 2 * GBK * FLS;   // doubles of LDS: the GEMM image (>= 2 x BLK of the tile body)
static_assert(LDS_D >= 2 * BLK, "LDS overlay");
// One LDS image for every task body (file scope: the non-inlined bodies below all address the same
// allocation, so the kernel holds 72 KB, not the sum of its task kinds' needs)
__shared__ double g_lds[LDS_D];

__device__ inline int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}

__device__ inline bool emul(const DtrArgs& g) { return g.rank < 0; }
__device__ inline bool sysmode(const DtrArgs& g) { return g.rank >= 0 && g.nranks > 1; }
template <typename T> __device__ inline T ld_sys(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline unsigned long long now_t() { return __builtin_amdgcn_s_memrealtime(); }

// readiness of task t on rank rk, checked by a whole wave: lane q tests requirements q, q + 64, ... (one
// round trip for the requirement records and one for the counters per 64 of them, instead of nreq serial
// ones on one lane; an update by a run of nk panels has 1 + 2 nk requirements, so deep runs take several
// rounds).  Emulation: a counter AT its target also needs that version's visibility time to have passed.
__device__ inline bool ready_wave(const DtrArgs& g, int t, int rk) {
  const int l = threadIdx.x & 63;
  const int rb = __builtin_amdgcn_readfirstlane(g.tasks[t].req_beg);
  const int nr = __builtin_amdgcn_readfirstlane((int)g.tasks[t].nreq);
  const int* cnt = g.cnt[rk];
  const bool em = emul(g), sy = sysmode(g);
  const unsigned long long now = em ? now_t() : 0;
  for (int q0 = 0; q0 < nr; q0 += 64) {
    bool ok = true;
    if (q0 + l < nr) {
      const int2 rq = g.reqs[rb + q0 + l];
      const int v = sy ? ld_sys(cnt + rq.x) : ld_sc1(cnt + rq.x);
      ok = v >= rq.y;
      if (ok && em && v == rq.y) ok = ld_sc1(g.vis + (size_t)rk * g.ncnt + rq.x) <= now;
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
  }
  return true;
}

// one CAS claim attempt on a low list (wave 0): the task, -1 (head not ready), -2 (list exhausted)
__device__ inline int try_list(const DtrArgs& g, int* cur, const int* list, int n, int rk) {
  for (int tries = 0; tries < 4; ++tries) {
    const int h = __builtin_amdgcn_readfirstlane(ld_sc1(cur));
    if (h >= n) return -2;
    const int t = __builtin_amdgcn_readfirstlane(list[h]);
    if (!ready_wave(g, t, rk)) return -1;
    int won = 0;
    if ((threadIdx.x & 63) == 0) won = atomicCAS(cur, h, h + 1) == h;
    if (__builtin_amdgcn_readfirstlane(won)) return t;
  }
  return -1;
}

__device__ inline int try_xcd(const DtrArgs& g, int x, int rk) {
  return try_list(g, g.cur + PSTRIDE * (MAXR + x), g.lo + g.lo_off[x], g.lo_off[x + 1] - g.lo_off[x], rk);
}

// wave 0: a ready task of the rank's low lists -- its own XCD's list, another of the rank's XCDs' only once
// its own is exhausted (-1 none ready yet, -2 every low list of the rank exhausted).  x0, nx: the rank's XCDs.
__device__ inline int claim_low(const DtrArgs& g, int xcd, int x0, int nx, int rk) {
  const int own = try_xcd(g, xcd, rk);
  if (own >= 0) return own;
  if (own == -1) {
    if (!(g.flags & 1)) return -1;
    // flags bit 0: the own head waits on a dependency -- take a READY head of another XCD's list instead
    // (any claimed task is ready, so the deadlock-freedom argument is unchanged; L2 locality is traded away)
    for (int d = 1; d < nx; ++d) {
      const int t = try_xcd(g, x0 + (xcd - x0 + d) % nx, rk);
      if (t >= 0) return t;
    }
    return -1;
  }
  bool all_done = true;
  for (int d = 1; d < nx; ++d) {
    const int t = try_xcd(g, x0 + (xcd - x0 + d) % nx, rk);
    if (t >= 0) return t;
    if (t == -1) all_done = false;
  }
  return all_done ? -2 : -1;
}

// tile offsets of rank rk (element offsets from g.A[rk]): local tiles and received copies
// (wave-uniform: the loaded value is made scalar again, or every buffer resource built from it -- the GEMM's
// operand and C addresses -- would be wrapped in a waterfall loop inside the software pipeline)
__device__ inline long long tile_at(const long long* tab, int nt, int i, int j) {
  const long long v = tab[i + (long long)j * nt];
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}

struct UpdKs {   // k-run of an update: L(i,k) strip r, L(j,k) strip c, k in [k0, k0+nk)
  // the first four panels' operand offsets are looked up once, before the GEMM (scalar registers, selected
  // by the uniform run index): a table load inside the software pipeline would stall it at every k-tile
  // switch; deeper runs read the table for the rest
  long long a0, a1, a2, a3, b0, b1, b2, b3;
  const long long* tab;
  int nt, i, j, r, c, k0;
  __device__ void init(int nk) {
    const long long ra = 128 * r, rb = 128 * c;
    a0 = tile_at(tab, nt, i, k0) + ra;
    b0 = tile_at(tab, nt, j, k0) + rb;
    a1 = nk > 1 ? tile_at(tab, nt, i, k0 + 1) + ra : 0;
    b1 = nk > 1 ? tile_at(tab, nt, j, k0 + 1) + rb : 0;
    a2 = nk > 2 ? tile_at(tab, nt, i, k0 + 2) + ra : 0;
    b2 = nk > 2 ? tile_at(tab, nt, j, k0 + 2) + rb : 0;
    a3 = nk > 3 ? tile_at(tab, nt, i, k0 + 3) + ra : 0;
    b3 = nk > 3 ? tile_at(tab, nt, j, k0 + 3) + rb : 0;
    a0 = rfl64_(a0), a1 = rfl64_(a1), a2 = rfl64_(a2), a3 = rfl64_(a3);
    b0 = rfl64_(b0), b1 = rfl64_(b1), b2 = rfl64_(b2), b3 = rfl64_(b3);
  }
  static __device__ long long rfl64_(long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
  }
  __device__ KPair operator()(int t) const {
    KPair p;
    if (t < 4) {
      // (readfirstlane: the functor may live in memory, which makes its fields look divergent)
      p.a_off = rfl64_(t == 0 ? a0 : t == 1 ? a1 : t == 2 ? a2 : a3);
      p.b_off = rfl64_(t == 0 ? b0 : t == 1 ? b1 : t == 2 ? b2 : b3);
    } else {
      p.a_off = tile_at(tab, nt, i, k0 + t) + 128 * r;
      p.b_off = tile_at(tab, nt, j, k0 + t) + 128 * c;
    }
    p.k = NBT;
    p.pad = 0;
    return p;
  }
};

struct TrsmKs {  // strip r of tile (i, k) times column block c of W_k (rows [0, 128(c+1)))
  long long a_off;
  int c;
  __device__ KPair operator()(int) const {
    KPair p;
    p.a_off = a_off;
    p.b_off = (long long)c * 128 * NBT;
    p.k = 128 * (c + 1);
    p.pad = 0;
    return p;
  }
};

// Block column b of W_k = L_kk^{-T} (upper triangular, 32-blocks W_{j,b}, j <= b), by the workgroup
// that factored row block b of the tile:  W_{b,b} = Z_b^T,  W_{j,b} = -(sum_{m=j}^{b-1} W_{j,m} L(b,m)^T) Z_b^T
// for j = b-1 .. 0  (rows of L^{-1}: R_b = Z_b (E_b - sum_{m<b} L(b,m) R_m), transposed), Z_b = diag(S_b) M_b.
// W_{j,m} comes from workgroup m, which publishes its block column in the order j = m, m-1, ..
// (flag = epoch * 64 + blocks published), so the 16 workgroups run as a wavefront.
__device__ void w_column(const DtrArgs& g, double* Wr, int k, int b, double* Vb) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int a = w >> 1, bh = w & 1;        // this wave's quadrant (row half a, column half bh)
  const int base = g.epoch * 64;
  const double* Mb = g.Mw + ((size_t)k * MAXB + b) * BLK;
  const double* Sb = g.Sw + ((size_t)k * MAXB + b) * RB;
  double* Lpk = g.Lp + (size_t)k * MAXB * MAXB * BLK;
  double* Wpk = g.Wp + (size_t)k * MAXB * MAXB * BLK;
  int* wprog = g.prog + ((size_t)k * 2 + 1) * MAXB * PSTRIDE;
  double* Wk = Wr + (size_t)k * NBT * NBT;
  const int rho = 16 * a + (l & 15);
  // Z_b^T operand rows (M_b rows of the bh half) and the column scale S_b
  double ym[8], sc[4];
#pragma unroll
  for (int u = 0; u < 8; ++u) ym[u] = ld_sc1(Mb + (4 * u + (l >> 4)) * RB + 16 * bh + (l & 15));
#pragma unroll
  for (int r = 0; r < 4; ++r) sc[r] = ld_sc1(Sb + 16 * bh + (l >> 4) + 4 * r);
  // W_{b,b} = Z_b^T: element (rho, gam) = S_b[gam] M_b[gam + 32 rho]
  {
    double* dst = Wpk + ((size_t)b * MAXB + b) * BLK;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gam = 16 * bh + (l >> 4) + 4 * r;
      const double v = sc[r] * ld_sc1(Mb + gam + RB * rho);
      st_sc1(dst + (w * 4 + r) * 64 + l, v);
      Wk[(32 * b + rho) + (long long)NBT * (32 * b + gam)] = v;
    }
  }
  drain_stores();
  __syncthreads();
  if (tid == 0) st_sc1(wprog + b * PSTRIDE, base + 1);
  for (int j = b - 1; j >= 0; --j) {
    // W_{j,m}, m in [j, b): workgroup m has published blocks m, m-1, .., j (m - j + 1 of them)
    if (l == 0)
      for (int m = j; m < b; ++m) spin_until(wprog + m * PSTRIDE, base + (m - j + 1), g.info);
    __builtin_amdgcn_wave_barrier();
    d4_t acc = {0, 0, 0, 0};
    for (int m = j; m < b; ++m) {
      double x[8], y[8];
      const double* Wjm = Wpk + ((size_t)j * MAXB + m) * BLK;
      const double* Lbm = Lpk + ((size_t)b * MAXB + m) * BLK;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = ld_sc1(Wjm + qoff(a, u, l));
        y[u] = ld_sc1(Lbm + qoff(bh, u, l));
      }
      acc = mfma_chunks<8>(y, x, acc);   // (W_{j,m} L(b,m)^T) quadrant (a, bh)
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Vb[(w * 4 + r) * 64 + l] = acc[r];
    __syncthreads();
    double xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xv[u] = -Vb[qoff(a, u, l)];
    d4_t o = {0, 0, 0, 0};
    o = mfma_chunks<8>(ym, xv, o);        // -(V M_b^T) quadrant (a, bh)
    double* dst = Wpk + ((size_t)j * MAXB + b) * BLK;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gam = 16 * bh + (l >> 4) + 4 * r;
      const double v = o[r] * sc[r];
      st_sc1(dst + (w * 4 + r) * 64 + l, v);
      Wk[(32 * j + rho) + (long long)NBT * (32 * b + gam)] = v;
    }
    drain_stores();
    __syncthreads();                      // (also: Vb is rewritten next step)
    if (tid == 0) st_sc1(wprog + b * PSTRIDE, base + (b - j + 1));
  }
}


// function arguments arrive in VGPRs: make the (uniform) task id and argument pointer scalar again,
// or every buffer resource derived from them needs a waterfall loop
__device__ inline const DtrArgs* uni(const DtrArgs* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const DtrArgs*)(((unsigned long long)hi << 32) | lo);
}

__device__ inline int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline long long rfl64(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}
template <typename P> __device__ inline P* rflp(P* p) { return (P*)rfl64((long long)p); }

// the task record and the argument fields a body uses, as wave-uniform (SGPR) values
struct TaskU {
  int i, j, k0, r, c, nk, nt;
  double* A;
  const long long* tab;
  long long ld;
  __device__ TaskU(const DtrArgs& g, int t, int rk) {
    const DtrTask tk = g.tasks[t];
    i = rfl(tk.i);
    j = rfl(tk.j);
    k0 = rfl(tk.k0);
    r = rfl(tk.r);
    c = rfl(tk.c);
    nk = rfl(tk.nk);
    nt = rfl(g.nt);
    A = rflp(g.A[rk]);
    tab = rflp(g.tab) + (size_t)rk * nt * nt;
    ld = rfl64(g.ld);
  }
};

// Hazard probe of one strip operand (thread 0): its TRSM's stamp must be this launch's epoch, and two elements of it
// -- row 0 of the strip in column 511 (the in-place TRSM's first-written block) and column 0 (its last) -- must
// read the same through this CU's caches (a plain load) and from memory (a system-scope load).  A mismatch is
// recorded: {task, k << 16 | strip << 8 | phase << 4 | kind, wg << 8 | xcd, stamp, plain511, mem511, plain0, mem0},
// kind 1 = stamp not this epoch (the task started before the TRSM's release), 2 = stale cache line.
__device__ __attribute__((noinline)) void probe_strip(const DtrArgs* __restrict__ gp, int t, int rk, int ti, int k,
                                                      int strip, int phase) {
  const DtrArgs& g = *gp;
  long long* pr = g.probe;
  const int nt = g.nt;
  const long long st = __hip_atomic_load(pr + 8 + (long long)(4 * ti + strip) * nt + k, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  const long long* tab = g.tab + (size_t)rk * nt * nt;
  const double* base = g.A[rk] + tab[ti + (long long)k * nt] + 128 * strip;
  const double* p511 = base + 511LL * g.ld;
  const double n511 = *(volatile const double*)p511, n0 = *(volatile const double*)base;
  const double m511 = __hip_atomic_load(const_cast<double*>(p511), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const double m0 = __hip_atomic_load(const_cast<double*>(base), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int kind = st != g.epoch ? 1 : ((__double_as_longlong(n511) != __double_as_longlong(m511) ||
                                         __double_as_longlong(n0) != __double_as_longlong(m0)) ? 2 : 0);
  if (!kind) return;
  const long long q = atomicAdd((unsigned long long*)pr, 1ULL);
  if (q >= 4096) return;
  long long* rec = pr + 8 + 4LL * nt * nt + 8 * q;
  rec[0] = t;
  rec[1] = ((long long)k << 16) | (strip << 8) | (phase << 4) | kind;
  rec[2] = ((long long)blockIdx.x << 8) | xcc_id();
  rec[3] = st;
  rec[4] = __double_as_longlong(n511);
  rec[5] = __double_as_longlong(m511);
  rec[6] = __double_as_longlong(n0);
  rec[7] = __double_as_longlong(m0);
}

// sub-tile (r, c) of diagonal tile (i, i): its stamp (epoch << 12 | panel the last update run ended at) and one element
// through the caches vs memory.  want: the expected stamp (< 0: no check); kinds 3 / 4 (an update's C operand) and
// 5 / 6 (a POTRF block's input), stamp / cache.
__device__ __attribute__((noinline)) void probe_sub(const DtrArgs* __restrict__ gp, int t, int rk, int i, int r, int c,
                                                    long long want, int row, int kst) {
  const DtrArgs& g = *gp;
  long long* pr = g.probe;
  const int nt = g.nt;
  long long* sst = pr + 8 + 4LL * nt * nt;
  const long long st = __hip_atomic_load(sst + ((long long)i * nt + i) * 16 + 4 * r + c, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  const long long* tab = g.tab + (size_t)rk * nt * nt;
  const double* e = g.A[rk] + tab[i + (long long)i * nt] + row + 128LL * c * g.ld;
  const double n0 = *(volatile const double*)e;
  const double m0 = __hip_atomic_load(const_cast<double*>(e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int kind = (want >= 0 && st != want) ? kst : (__double_as_longlong(n0) != __double_as_longlong(m0) ? kst + 1 : 0);
  if (!kind) return;
  const long long q = atomicAdd((unsigned long long*)pr, 1ULL);
  if (q >= 4096) return;
  long long* rec = pr + 8 + 20LL * nt * nt + 8 * q;
  rec[0] = t;
  rec[1] = ((long long)i << 16) | ((4 * r + c) << 8) | kind;
  rec[2] = ((long long)blockIdx.x << 8) | xcc_id();
  rec[3] = st;
  rec[4] = __double_as_longlong(n0);
  rec[5] = __double_as_longlong(m0);
  rec[6] = want;
  rec[7] = row;
}

__device__ inline void probe_upd(const DtrArgs* __restrict__ gp, int t, int rk, int i, int j, int r, int c, int k0,
                                 int nk, int phase) {
  if (threadIdx.x != 0) return;
  for (int q = 0; q < nk; ++q) {
    probe_strip(gp, t, rk, i, k0 + q, r, phase);
    if (c != r) probe_strip(gp, t, rk, j, k0 + q, c, phase);
  }
  if (phase == 0) probe_sub(gp, t, rk, i, r, c, k0 > 0 ? ((long long)gp->epoch << 12) + k0 : -1, 128 * r, 3);
}

// Task bodies: each is a separate (non-inlined) function, so its registers are allocated on its own
// -- the GEMM body inlined into the task loop spilled (the capped persistent k_gemm_full spills the
// same way: hipcc -Rpass-analysis=kernel-resource-usage, profiles/r4_dtr_regs.txt).
__device__ __attribute__((noinline)) void run_upd(const DtrArgs* __restrict__ gp, int t, int rk) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t), rfl(rk));
  __builtin_amdgcn_s_setprio(0);
  UpdKs ks;
  ks.tab = u.tab;
  ks.nt = u.nt, ks.i = u.i, ks.j = u.j, ks.r = u.r, ks.c = u.c, ks.k0 = u.k0;
  ks.init(u.nk);
  const int uplo = (u.i == u.j && u.r == u.c) ? 1 : 0;
  const bool prb = g.probe != nullptr && u.i == u.j;
  if (prb) probe_upd(gp, rfl(t), rfl(rk), u.i, u.j, u.r, u.c, u.k0, u.nk, 0);
  gemm_subtile<double, false, true>(g_lds, ks, u.nk, 0, 0, uplo, -1.0, u.A, (int)u.ld, u.A, (int)u.ld, 1.0,
                                    u.A + tile_at(u.tab, u.nt, u.i, u.j) + 128 * u.r + 128LL * u.c * u.ld, (int)u.ld,
                                    -1, (rfl(g.flags) & 16) != 0);
  if (prb) probe_upd(gp, rfl(t), rfl(rk), u.i, u.j, u.r, u.c, u.k0, u.nk, 1);
}

__device__ __attribute__((noinline)) void run_trsm(const DtrArgs* __restrict__ gp, int t, int rk) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t), rfl(rk));
  __builtin_amdgcn_s_setprio(2);
  const long long ao = tile_at(u.tab, u.nt, u.i, u.k0) + 128 * u.r;
  const double* Wk = rflp(g.W[rfl(rk)]) + (size_t)u.k0 * NBT * NBT;
  for (int c = 3; c >= 0; --c) {
    const TrsmKs ks{ao, c};
    gemm_subtile<double, false, false>(g_lds, ks, 1, 0, 0, 0, 1.0, u.A, (int)u.ld, Wk, NBT, 0.0,
                                       u.A + ao + 128LL * c * u.ld, (int)u.ld, -1, (rfl(g.flags) & 16) != 0);
    __syncthreads();   // LDS image reuse (block c-1 never reads the columns block c wrote)
  }
}

__device__ __attribute__((noinline)) void run_potrf(const DtrArgs* __restrict__ gp, int t, int rk) {
  const DtrArgs& g = *uni(gp);
  t = __builtin_amdgcn_readfirstlane(t);
  rk = __builtin_amdgcn_readfirstlane(rk);
  const DtrTask tk = g.tasks[t];
  __builtin_amdgcn_s_setprio(RB_PRIO);
  const int k = tk.k0, b = tk.r;
  RbWork ws;
  ws.M = g.Mw + (size_t)k * MAXB * BLK;
  ws.S = g.Sw + (size_t)k * MAXB * RB;
  ws.Lp = g.Lp + (size_t)k * MAXB * MAXB * BLK;
  ws.prog = g.prog + (size_t)k * 2 * MAXB * PSTRIDE;
  ws.ticket = nullptr;
  ws.tbase = 0;
  const long long* tab = g.tab + (size_t)rk * g.nt * g.nt;
  if (g.probe && threadIdx.x == 0)   // hazard probe: the row block's input sub-tiles (final versions, fresh)
    for (int c = 0; c <= b / 4; ++c)
      probe_sub(gp, t, rk, k, b / 4, c, k > 0 ? ((long long)g.epoch << 12) + k : -1, 32 * b, 5);
  if (g.snap) {   // ... and a copy of the row block's input as this workgroup reads it (host: chol(input) vs output)
    const double* src = g.A[rk] + tile_at(tab, g.nt, k, k);
    double* dst = g.snap + (size_t)k * NBT * NBT;
    for (int e = threadIdx.x; e < 32 * (32 * b + 32); e += 256) {
      const int rr = 32 * b + e % 32, cc = e / 32;
      dst[rr + (long long)cc * NBT] = src[rr + (long long)cc * g.ld];
    }
    __syncthreads();
  }
  // with the task trace on: the tile body's phase stamps of every block (64 per block, after the task records)
  unsigned long long* ph = g.trace ? (unsigned long long*)(g.trace + 4LL * g.ntask) + (size_t)k * MAXB * 64 : nullptr;
  rb_tile_body<true>(g.A[rk] + tile_at(tab, g.nt, k, k), NBT, (int)g.ld, g.info, k * NBT, ws, g.epoch, ph, b,
                     g_lds, g_lds + BLK);
  __syncthreads();
  if (ph && threadIdx.x == 0) ph[64 * b + 52] = __builtin_amdgcn_s_memrealtime();
  w_column(g, g.W[rk], k, b, g_lds);
  if (ph && threadIdx.x == 0) ph[64 * b + 53] = __builtin_amdgcn_s_memrealtime();
}

// system-scope stores (sc0 sc1: written through to the peer's memory), two 8-byte ones -- compiler-generated, not
// inline asm (an inline-asm dwordx4 store hides its VGPR operands from the hazard recognizer: see st_sc1_x2 in
// potrf_tile.h and profiles/r6_dtr_coresidency_rootcause.txt)
__device__ inline void st_sys_x2(double* p, double a, double b) {
  __hip_atomic_store(p, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(p + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// copy rows x cols (column-major, both ld 512) from src to dst with the whole workgroup: 16-byte loads /
// stores, 4 x 16 B in flight per thread; system-scope stores when the destination is a peer's memory
__device__ inline void copy_block(double* __restrict__ dst, const double* __restrict__ src, int rows, int cols,
                                  bool sys) {
  typedef double d2_t __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x;
  const int hr = rows >> 1;                 // 16-byte pairs per column
  const int n = hr * cols;
  for (int e0 = tid; e0 < n; e0 += 4 * 256) {
    d2_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      if (e < n) {
        const int cc = e / hr, rr = 2 * (e % hr);
        v[u] = *(const d2_t*)(src + rr + (long long)cc * NBT);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      if (e < n) {
        const int cc = e / hr, rr = 2 * (e % hr);
        double* d = dst + rr + (long long)cc * NBT;
        if (sys) st_sys_x2(d, v[u][0], v[u][1]);
        else *(d2_t*)d = v[u];
      }
    }
  }
}

// SEND: strip r (128 x 512) of the solved panel tile (i, k0) into the destination's receive slot
__device__ __attribute__((noinline)) void run_send(const DtrArgs* __restrict__ gp, int t, int rk) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t), rfl(rk));
  __builtin_amdgcn_s_setprio(2);
  const double* src = u.A + tile_at(u.tab, u.nt, u.i, u.k0) + 128 * u.r;
  double* dst = rflp(g.recv[u.j]) + rfl64(g.xoff[rfl(t)]);
  copy_block(dst, src, 128, NBT, sysmode(g));
}

// SENDW: column block c of W_k (rows [0, 128 (c + 1)), upper triangle + the zeros below it in the
// diagonal block) into the destination's W
__device__ __attribute__((noinline)) void run_sendw(const DtrArgs* __restrict__ gp, int t, int rk) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t), rfl(rk));
  __builtin_amdgcn_s_setprio(2);
  const long long o = rfl64(g.xoff[rfl(t)]);
  const double* src = rflp(g.W[rfl(rk)]) + o;
  double* dst = rflp(g.W[u.j]) + o;
  copy_block(dst, src, 128 * (u.r + 1), 128, sysmode(g));
}

// Emulation: when the completion of task t (ran [t0, t1)) becomes visible -- (dil - 1) x its duration after
// it ended; a send: dil x (lat + bytes / bw) after the (src, dst) link frees up (FIFO per ordered pair)
__device__ inline unsigned long long emul_due(const DtrArgs& g, const DtrTask& tk, int rk, unsigned long long t0,
                                              unsigned long long t1) {
  if (tk.type != T_SEND && tk.type != T_SENDW)
    return t1 + (unsigned long long)(g.dil - 1) * (t1 - t0);
  const long long bytes = tk.type == T_SEND ? 128LL * NBT * 8 : 128LL * 128 * (tk.r + 1) * 8;
  const unsigned long long dur = (unsigned long long)g.dil * (unsigned long long)(g.lat_t + bytes / g.bw_bpt);
  unsigned long long* lk = g.link + rk * MAXR + tk.j;
  unsigned long long old = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const unsigned long long st = old > t1 ? old : t1;
    const unsigned long long fin = st + dur;
    if (__hip_atomic_compare_exchange_strong(lk, &old, fin, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return fin;
  }
}

// The arguments live in device memory and are re-read through a laundered pointer every iteration:
// hoisting all of DtrArgs into SGPRs across the task loop (what a by-value kernel argument invites)
// leaves the GEMM body too few SGPRs and spills it to scratch.
// The high list is handed out by TICKET (one atomic add per workgroup, no compare-and-swap retries on a
// cursor that 512 workgroups contend for): a workgroup takes the next ticket when the list's head is
// ready, and while a ticket's task is not ready yet (a race) it runs ready low-list tasks (a POTRF ticket only after 50 us: its 16 cooperating workgroups
// should start together) -- the high list's claim rate no longer bounds the critical path (profiles/
// r4_dtr_trace.txt: one CAS cursor gave ~4 us per claim, 86k claims).  Progress: tickets go out in list
// order, so the earliest unfinished task in the topological order is ready and either held by a ticket
// (its holder comes back to it) or the head of its low list (claimable by every workgroup that has
// waited 50 us).
__global__ __launch_bounds__(256, 2) void k_dtr_potrf(const DtrArgs* __restrict__ gargs) {
  __shared__ int s_task;
  const int tid = threadIdx.x;
  const int xcd = xcc_id();
  unsigned long long idle0 = 0;
  int nap = 1;        // idle back-off (s_sleep units of 64 clocks), doubled up to ~1 us
  int ticket = -1;    // held high-list position (wave 0's copy)
  unsigned long long ticket_t0 = 0;
  bool hi_done = false, lo_done = false;
  // this workgroup's rank and that rank's XCDs [x0, x0 + nx)
  int rk, x0, nx;
  {
    const DtrArgs* gp = gargs;
    asm volatile("" : "+s"(gp));
    const int nr = gp->nranks, rr = gp->rank;
    if (rr >= 0) {
      rk = nr > 1 ? rr : 0;
      x0 = 0;
      nx = 8;
    } else {
      rk = xcd * nr / 8;
      nx = 8 / nr;
      x0 = rk * nx;
    }
  }
  for (;;) {
    const DtrArgs* gp = gargs;
    asm volatile("" : "+s"(gp));
    const DtrArgs& g = *gp;
    if (tid < 64) {
      int t = -1;
      if (ld_sc1(g.info) == -1000) {
        t = -2;
      } else {
        const int hbeg = g.hi_off[rk];
        if (ticket < 0 && !hi_done) {
          // the high list is nsteps FIFO segments (one per panel step with the "step" order, else one): a
          // ticket goes out for a READY head of one of the first STEPW segments not yet handed out completely
          // (lowest first) -- a task of step k+1 (POTRF(k+1)) is not held up behind step k's updates that wait
          // for remote strips.  A ticket only for a ready head: a workgroup holding a not-yet-ready critical
          // task would run low-list tasks meanwhile and come back up to one bulk task late -- the 16 POTRF
          // workgroups of a tile would then start spread over ~0.4 ms and wait for each other.
          // Progress: the earliest unclaimed task of the (step-major) topological order is the head of the
          // lowest segment that is not handed out, which every scan looks at first.
          const int stepw = ((unsigned)g.flags >> 24) & 15u ? (((unsigned)g.flags >> 24) & 15u) : 8;
          const int ns = g.nsteps;
          const int* so = g.hs_off + (size_t)rk * (ns + 1);
          int* lw = g.cur + PSTRIDE * rk;
          const int s0 = __builtin_amdgcn_readfirstlane(ld_sc1(lw));
          if (s0 >= ns) {
            hi_done = true;
          } else {
            const int s1 = s0 + stepw < ns ? s0 + stepw : ns;
            for (int sg = s0; sg < s1; ++sg) {
              int* sc = g.scur + ((size_t)rk * ns + sg) * PSTRIDE;
              const int b = so[sg], n = so[sg + 1] - b;
              const int h = __builtin_amdgcn_readfirstlane(ld_sc1(sc));
              if (h >= n) {
                if (sg == s0 && tid == 0) atomicCAS(lw, s0, s0 + 1);   // segment handed out: raise the mark
                continue;
              }
              if (ready_wave(g, __builtin_amdgcn_readfirstlane(g.hi[hbeg + b + h]), rk)) {
                int tk = 0;
                if (tid == 0) tk = atomicAdd(sc, 1);
                tk = __builtin_amdgcn_readfirstlane(tk);
                if (tk < n) {
                  ticket = b + tk;
                  ticket_t0 = now_t();
                  break;
                }
              }
            }
          }
        }
        bool help = true;
        if (ticket >= 0) {
          const int th = __builtin_amdgcn_readfirstlane(g.hi[hbeg + ticket]);
          if (ready_wave(g, th, rk)) {
            t = th;
            ticket = -1;
          } else {
            // a ticket whose task is not ready yet polls for a while before it helps with a low-list task
            // (which can hold it for a whole bulk update): POTRF tickets 50 us by default (the group starts
            // together), other tickets not at all; flags bits 16-23 / 8-15 override (units of 10 us)
            const unsigned fl = (unsigned)g.flags;
            const bool is_potrf = __builtin_amdgcn_readfirstlane(g.tasks[th].type) == T_POTRF;
            unsigned long long hold = is_potrf ? ((fl >> 16) & 255u) : ((fl >> 8) & 255u);
            if (is_potrf && hold == 0) hold = 5;
            if (now_t() - ticket_t0 < hold * 1000ULL * (unsigned long long)g.dil) help = false;
          }
        }
        if (t < 0 && help && !lo_done) {
          t = claim_low(g, xcd, x0, nx, rk);
          if (t == -2) {
            lo_done = true;
            t = -1;
          }
        }
        if (t < 0) t = (hi_done && lo_done && ticket < 0) ? -2 : -1;
      }
      if (t >= 0) {
        // the predecessors' bytes, fresh in this CU (system scope: a peer process wrote some of them)
        // (flags bit 2: the system-scope acquire also in one process -- a measurement knob: it invalidates the
        // XCD's L2 as well, see profiles/r5_dtr_dist_emulation.txt)
        if (tid == 0) {
          if (sysmode(g) || (g.flags & 4)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        idle0 = 0;
      } else if (t == -1 && tid == 0) {
        const unsigned long long now = now_t();
        if (idle0 == 0) idle0 = now;
        else if (now - idle0 > 400000000ULL * (unsigned long long)g.dil) {   // 4 s (dilated) without a ready task: drain
          atomicExch(g.info, -1000);
          t = -2;
        }
      }
      if (tid == 0) s_task = t;
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);   // wave-uniform: task fields load to SGPRs
    __syncthreads();
    if (t == -2) break;
    if (t == -1) {
      for (int q = 0; q < nap; ++q) __builtin_amdgcn_s_sleep(1);
      nap = nap < 32 ? 2 * nap : 32;
      continue;
    }
    nap = 1;
    const unsigned long long t_start = now_t();
    const DtrTask tk = g.tasks[t];
    if (tk.type == T_UPD) run_upd(gp, t, rk);
    else if (tk.type == T_TRSM) run_trsm(gp, t, rk);
    else if (tk.type == T_POTRF) run_potrf(gp, t, rk);
    else if (tk.type == T_SEND) run_send(gp, t, rk);
    else run_sendw(gp, t, rk);
    // release: every wave's stores drained, then one agent-scope release and the counter bump
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned long long due = 0;
    if (tid == 0 && tk.inc >= 0 && emul(g)) due = emul_due(g, tk, rk, t_start, now_t());
    if (tid == 0 && g.trace) {
      long long* tr = g.trace + 4 * (size_t)t;
      tr[0] = (long long)t_start;
      tr[1] = (long long)now_t();
      tr[2] = ((long long)blockIdx.x << 8) | xcd;
      // emulation: when the completion becomes visible; otherwise the number of times the task ran (1)
      if (emul(g)) tr[3] = (long long)due;
      else atomicAdd((unsigned long long*)(tr + 3), 1ULL);
    }
    if (tid == 0 && g.probe && tk.type == T_TRSM)   // hazard probe: the strip's stamp, ordered by the release below
      __hip_atomic_store(g.probe + 8 + (long long)(4 * tk.i + tk.r) * g.nt + tk.k0, (long long)g.epoch,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && g.probe && tk.type == T_UPD && tk.i == tk.j)   // ... and a diagonal sub-tile's version stamp
      __hip_atomic_store(g.probe + 8 + 4LL * g.nt * g.nt + ((long long)tk.i * g.nt + tk.i) * 16 + 4 * tk.r + tk.c,
                         ((long long)g.epoch << 12) + tk.k0 + tk.nk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && tk.inc >= 0) {
      const bool remote = tk.type == T_SEND || tk.type == T_SENDW;
      const int tr_ = remote ? tk.j : rk;
      if (emul(g))
        __hip_atomic_fetch_max(g.vis + (size_t)tr_ * g.ncnt + tk.inc, due, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // (flags bit 3: the system-scope release for every task -- a measurement knob, DPLASMA_DTR_SYSREL; it
      // does not remove the two-workgroups-per-CU failure, profiles/r5_dtr_coresidency.txt)
      if ((remote && sysmode(g)) || (g.flags & 8)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(g.cnt[tr_] + tk.inc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(g.cnt[tr_] + tk.inc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

// ---------------------------------------------------------------------------------------------------------
// Push scheduling: a task becomes READY when its last predecessor completes -- that predecessor's workgroup
// decrements the pending count of each successor (64 lanes at once) and pushes the one it brought to zero into
// a ready ring: one FIFO per (priority class, XCD), sized for every task that will ever enter it (pushes
// never wrap).  Workers pop the lowest non-empty class, own XCD first: the ready critical-path task (a POTRF
// block, a panel TRSM, a look-ahead update) is the next one any idle workgroup takes, with no list position to
// wait behind -- what the reference's priority-ordered ready queues do on every rank (src/zpotrf_L.jdf:58-69).
// The lists + version counters of k_dtr_potrf make a ready task wait behind its list's head; its traces showed
// that wait as the critical path (profiles/r5_dtr_queue.txt).
// A push reserves a slot (tail atomic) and then stores the id (sc1): a popper that finds the reserved slot still
// 0 treats the ring as empty for now.  Completion order: release (every wave's stores drained, agent release)
// before the decrements, so a pushed task's inputs are visible to the popper's acquire.
template <typename T> __device__ inline T ld_q(const T* p, bool sy) { return sy ? ld_sys(p) : ld_sc1(p); }

__device__ inline int q_pop(const DtrArgs& g, int r, int rk, bool sy) {
  int* head = g.qctl[rk] + (size_t)(2 * r) * PSTRIDE;
  int* tail = head + PSTRIDE;
  const int* qb = g.qbase + (size_t)rk * (g.nclass * 8 + 1);
  for (int tries = 0; tries < 2; ++tries) {
    const int h = __builtin_amdgcn_readfirstlane(ld_q(head, sy));
    const int tl = __builtin_amdgcn_readfirstlane(ld_q(tail, sy));
    if (h >= tl) return -1;
    const int s = __builtin_amdgcn_readfirstlane(ld_q(g.qslot[rk] + qb[r] + h, sy));
    if (s == 0) return -1;
    int won = 0;
    if ((threadIdx.x & 63) == 0) {
      int e = h;
      won = sy ? __hip_atomic_compare_exchange_strong(head, &e, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM)
               : atomicCAS(head, h, h + 1) == h;
    }
    if (__builtin_amdgcn_readfirstlane(won)) return s - 1;
  }
  return -1;
}

// push task t into its ring on rank d (one lane); process mode: the peer's rings through its IPC mapping
__device__ inline void q_push(const DtrArgs& g, int t, int d, bool sy) {
  const int r = g.ring_of[t];
  int* tail = g.qctl[d] + (size_t)(2 * r + 1) * PSTRIDE;
  const int* qb = g.qbase + (size_t)d * (g.nclass * 8 + 1);
  if (sy) {
    const int pos = __hip_atomic_fetch_add(tail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(g.qslot[d] + qb[r] + pos, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    const int pos = atomicAdd(tail, 1);
    st_sc1(g.qslot[d] + qb[r] + pos, t + 1);
  }
}

__global__ __launch_bounds__(256, 2) void k_dtr_q(const DtrArgs* __restrict__ gargs) {
  __shared__ int s_task;
  const int tid = threadIdx.x;
  const int xcd = xcc_id();
  unsigned long long idle0 = 0;
  int nap = 1;
  int seen_done = -1;   // g.done read before this workgroup's last empty scan (-1: none)
  int rk, x0, nx;
  bool sy, em;
  {
    const DtrArgs* gp = gargs;
    asm volatile("" : "+s"(gp));
    sy = sysmode(*gp);
    em = emul(*gp);
    // emulation: XCD x runs rank x nr / 8 (its rings live on that rank's XCDs [x0, x0 + nx))
    nx = em ? 8 / gp->nranks : 8;
    rk = sy ? gp->rank : em ? xcd / nx : 0;
    x0 = em ? rk * nx : 0;
  }
  for (;;) {
    const DtrArgs* gp = gargs;
    asm volatile("" : "+s"(gp));
    const DtrArgs& g = *gp;
    if (tid < 64) {
      int t = -1;
      // one process: a task is pushed only by a completion, and every completion bumps g.done after its pushes --
      // so when g.done has not moved since this workgroup's last empty scan, no ring can have gained a task and
      // the 2 x nclass x 8 coherent loads of a scan are skipped (with ~160 idle workgroups rescanning, the early
      // steps' POTRF hand-offs ran 2x slower: profiles/r6_dtr16k_analysis.txt).  Not with remote pushes (peers)
      // or emulated visibility times.  DPLASMA_DTR_SCANSKIP=0 (flags bit 5) turns it off.
      const bool can_skip = !sy && !em && !(g.flags & 32);
      const int dnow = can_skip ? __builtin_amdgcn_readfirstlane(ld_sc1(g.done)) : 0;
      if (ld_sc1(g.info) == -1000) {
        t = -2;
      } else if (can_skip && dnow == seen_done) {
        if (dnow >= g.ntask) t = -2;
      } else {
        // every ring's emptiness at once (lane l: scan position l + 64 w, class-major, own XCD first inside a
        // class), then a pop of the first non-empty one in that order; a lost race rescans
        const int nr = g.nclass * nx;
        const int l = tid & 63;
        const unsigned long long now = em ? now_t() : 0;
        for (int tries = 0; tries < 4 && t < 0; ++tries) {
          int best = -1;
          for (int w0 = 0; w0 < nr && best < 0; w0 += 64) {
            const int pos = w0 + l;
            bool ne = false;
            int r = 0;
            if (pos < nr) {
              r = (pos / nx) * 8 + x0 + (xcd - x0 + pos) % nx;
              const int* hd = g.qctl[rk] + (size_t)(2 * r) * PSTRIDE;
              const int h = ld_q(hd, sy);
              ne = h < ld_q(hd + PSTRIDE, sy);
              if (ne && em) {   // emulation: a head whose inputs are not visible yet does not count
                const int sx = ld_sc1(g.qslot[rk] + g.qbase[(size_t)rk * (g.nclass * 8 + 1) + r] + h);
                ne = sx != 0 && ld_sc1(g.rdy + sx - 1) <= now;
              }
            }
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(ne);
            if (bal) {
              const int first = __builtin_ctzll(bal);
              best = __builtin_amdgcn_readlane(r, first);
            }
          }
          if (best < 0) break;
          t = q_pop(g, best, rk, sy);
        }
        if (t >= 0 && em && ld_sc1(g.rdy + t) > now_t()) {
          // (a race: the popped head was replaced by one not visible yet) -- wait for it, it is ours now
          while (ld_sc1(g.rdy + t) > now_t()) __builtin_amdgcn_s_sleep(2);
        }
        seen_done = (t < 0 && can_skip) ? dnow : -1;
        if (t < 0 && __builtin_amdgcn_readfirstlane(ld_sc1(g.done)) >= g.ntask) t = -2;
      }
      if (t >= 0) {
        if (tid == 0) {
          if (sy) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // a peer's strips / W may be among the inputs
          else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        idle0 = 0;
      } else if (t == -1 && tid == 0) {
        const unsigned long long now = now_t();
        if (idle0 == 0) idle0 = now;
        else if (now - idle0 > 400000000ULL) {   // 4 s without a ready task: drain
          atomicExch(g.info, -1000);
          t = -2;
        }
      }
      if (tid == 0) s_task = t;
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();
    if (t == -2) break;
    if (t == -1) {
      // idle back-off: every scan is 2 x nclass x 8 coherent loads, and ~150 idle workgroups rescanning after 1-16
      // sleeps slowed the POTRF blocks' hand-offs in the early steps (POTRF(1..3) 814-919 us against ~380: phase
      // stamps, dtr_trace_run.py 16k); cap = 2^(flags >> 28) sleeps (DPLASMA_DTR_NAP; 0: 16)
      const unsigned napl = ((unsigned)g.flags >> 28) & 15u;
      const int napmax = napl ? (1 << napl) : 16;
      for (int q = 0; q < nap; ++q) __builtin_amdgcn_s_sleep(1);
      nap = nap < napmax ? 2 * nap : napmax;
      continue;
    }
    nap = 1;
    const unsigned long long t_start = now_t();
    const DtrTask tk = g.tasks[t];
    if (tk.type == T_UPD) run_upd(gp, t, rk);
    else if (tk.type == T_TRSM) run_trsm(gp, t, rk);
    else if (tk.type == T_POTRF) run_potrf(gp, t, rk);
    else if (tk.type == T_SEND) run_send(gp, t, rk);
    else run_sendw(gp, t, rk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && g.trace) {
      long long* tr = g.trace + 4 * (size_t)t;
      tr[0] = (long long)t_start;
      tr[1] = (long long)now_t();
      tr[2] = ((long long)blockIdx.x << 8) | xcd;
      atomicAdd((unsigned long long*)(tr + 3), 1ULL);
    }
    unsigned long long due = 0;
    if (tid == 0 && em) due = emul_due(g, tk, rk, t_start, now_t());
    if (em) {   // (unsigned words: a signed low word would sign-extend into the high one)
      const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)due), hi = __builtin_amdgcn_readfirstlane((unsigned)(due >> 32));
      due = ((unsigned long long)hi << 32) | lo;
    }
    if (tid == 0 && g.probe && tk.type == T_TRSM)   // hazard probe: the strip's stamp, ordered by the release below
      __hip_atomic_store(g.probe + 8 + (long long)(4 * tk.i + tk.r) * g.nt + tk.k0, (long long)g.epoch,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && g.probe && tk.type == T_UPD && tk.i == tk.j)   // ... and a diagonal sub-tile's version stamp
      __hip_atomic_store(g.probe + 8 + 4LL * g.nt * g.nt + ((long long)tk.i * g.nt + tk.i) * 16 + 4 * tk.r + tk.c,
                         ((long long)g.epoch << 12) + tk.k0 + tk.nk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 64) {
      if (sy) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int sb = g.succ_off[t], se = g.succ_off[t + 1];
      for (int q = sb + tid; q < se; q += 64) {
        const int sx = g.succ[q];
        const int d = g.town ? g.town[sx] : 0;
        if (em) {   // the successor's visibility: the latest of its predecessors' (before the decrement)
          __hip_atomic_fetch_max(g.rdy + sx, due, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const int left = sy ? __hip_atomic_fetch_sub(g.pend[d] + sx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                            : atomicSub(g.pend[d] + sx, 1);
        if (left == 1) q_push(g, sx, d, sy);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) atomicAdd(g.done, 1);
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

}  // namespace

// One DTR Cholesky launch (see the header).  args: a DtrArgs image built by the host (models/potrf_dtr.py
// fills it through dpl_dtr_args_size / the field offsets below), grid = 2 x #CUs workgroups.
DPL_API int dpl_dtr_args_size() { return (int)sizeof(DtrArgs); }
// the push-scheduled launch (k_dtr_q): one process, one rank
DPL_API int dpl_dtr_potrf_q(const void* args_dev, int nwg, hipStream_t st) {
  if (nwg <= 0 || !args_dev) return -3;
  hipLaunchKernelGGL(k_dtr_q, dim3(nwg), dim3(256), 0, st, (const DtrArgs*)args_dev);
  return (int)hipGetLastError();
}
DPL_API int dpl_dtr_lds_doubles() { return LDS_D; }
// args_dev: the DtrArgs image in device memory (uploaded by the host before the launch)
DPL_API int dpl_dtr_potrf(const void* args_dev, int nwg, hipStream_t st) {
  if (nwg <= 0 || !args_dev) return -3;
  hipLaunchKernelGGL(k_dtr_potrf, dim3(nwg), dim3(256), 0, st, (const DtrArgs*)args_dev);
  return (int)hipGetLastError();
}
// offsets of DtrArgs fields by name (the host packs the struct without a C compiler): returns the offset of
// field `name`, sizeof(DtrArgs) for "size", the layout constants for "MAXB" / "BLK" / "RB" / "PSTRIDE" /
// "MAXR" / "task", or -1
#define DTR_FIELD(f) if (!std::strcmp(name, #f)) return (long long)offsetof(DtrArgs, f);
DPL_API long long dpl_dtr_field(const char* name) {
  DTR_FIELD(ld) DTR_FIELD(nt) DTR_FIELD(nranks) DTR_FIELD(rank) DTR_FIELD(epoch) DTR_FIELD(flags) DTR_FIELD(dil)
  DTR_FIELD(ncnt) DTR_FIELD(tasks) DTR_FIELD(reqs) DTR_FIELD(tab) DTR_FIELD(xoff) DTR_FIELD(cur) DTR_FIELD(hi)

  DTR_FIELD(hi_off) DTR_FIELD(nsteps) DTR_FIELD(hs_off) DTR_FIELD(scur) DTR_FIELD(lo) DTR_FIELD(lo_off) DTR_FIELD(A) DTR_FIELD(recv) DTR_FIELD(W) DTR_FIELD(cnt)
  DTR_FIELD(vis) DTR_FIELD(link) DTR_FIELD(bw_bpt) DTR_FIELD(lat_t) DTR_FIELD(Mw) DTR_FIELD(Sw) DTR_FIELD(Lp)
  DTR_FIELD(Wp) DTR_FIELD(prog) DTR_FIELD(info) DTR_FIELD(trace) DTR_FIELD(ntask) DTR_FIELD(nclass) DTR_FIELD(pend)
  DTR_FIELD(succ_off) DTR_FIELD(succ) DTR_FIELD(ring_of) DTR_FIELD(town) DTR_FIELD(qbase) DTR_FIELD(qctl)
  DTR_FIELD(qslot) DTR_FIELD(done) DTR_FIELD(rdy) DTR_FIELD(probe) DTR_FIELD(snap)
  if (!std::strcmp(name, "size")) return (long long)sizeof(DtrArgs);
  if (!std::strcmp(name, "task")) return (long long)sizeof(DtrTask);
  if (!std::strcmp(name, "MAXB")) return MAXB;
  if (!std::strcmp(name, "BLK")) return BLK;
  if (!std::strcmp(name, "RB")) return RB;
  if (!std::strcmp(name, "PSTRIDE")) return PSTRIDE;
  if (!std::strcmp(name, "MAXR")) return MAXR;
  return -1;
}
