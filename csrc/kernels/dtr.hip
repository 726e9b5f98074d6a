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
// Dependencies are tile-version counters, not successor lists: each task lists (counter, target)
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
// + s_waitcnt, barrier.  Every wait is bounded (info = -1000, all workgroups drain).
#include "gemm_tile.h"
#include "potrf_tile.h"

namespace {
using namespace rbk;

enum : int { T_UPD = 0, T_TRSM = 1, T_POTRF = 2 };

struct DtrTask {      // 32 bytes
  int type;
  int i, j;           // UPD: tile (i, j); TRSM: tile (i, k0); POTRF: -
  int k0;             // first panel (TRSM / POTRF: the panel)
  int req_beg;        // requirements [req_beg, req_beg + nreq): (counter, target) pairs
  int inc;            // counter bumped on completion (-1: none)
  short r, c;         // UPD: sub-tile; TRSM: strip r; POTRF: block row r
  short nk, nreq;     // UPD: panels in the run
};
static_assert(sizeof(DtrTask) == 32, "DtrTask layout");

struct DtrArgs {
  double* A;
  long long ld;             // leading dimension of the tiles
  long long si, sj;         // element offset of tile (i, j) = i * si + j * sj (LAPACK or TILE storage)
  int nt;
  const DtrTask* tasks;
  const int2* reqs;
  int* cnt;                 // version counters (zeroed per launch)
  int* cur;                 // list cursors: [0] high, [1 + x] low list of XCD x; PSTRIDE ints apart
  const int* hi;            // high list (task ids)
  int nhi;
  const int* lo;            // low lists, concatenated
  int lo_off[9];
  double* W;                // nt x (512 x 512): W_k = L_kk^{-T}
  double* Mw;               // nt x MAXB x BLK     (M_k of the 32-blocks, potrf_tile.h)
  double* Sw;               // nt x MAXB x RB
  double* Lp;               // nt x MAXB x MAXB x BLK  (published L(b, m) blocks, T-layout)
  double* Wp;               // nt x MAXB x MAXB x BLK  (published W blocks, T-layout)
  int* prog;                // nt x 2 x MAXB x PSTRIDE: tile-step flags, then W-column flags
  int epoch;
  int flags;                // bit 0: steal a ready head of another XCD's list when the own head is not ready
  int* info;
  long long* trace;         // optional (DPLASMA_DTR_TRACE): per task {start, end, wg << 8 | xcd}, 100 MHz ticks
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

__device__ inline long long toff(long long si, long long sj, int i, int j) { return (long long)i * si + (long long)j * sj; }

// readiness of task t, checked by a whole wave: lane q tests requirements q, q + 64, ... (one round trip
// for the requirement records and one for the counters per 64 of them, instead of nreq serial ones on one
// lane; an update by a run of nk panels has 1 + 2 nk requirements, so deep runs take several rounds)
__device__ inline bool ready_wave(const DtrArgs& g, int t) {
  const int l = threadIdx.x & 63;
  const int rb = __builtin_amdgcn_readfirstlane(g.tasks[t].req_beg);
  const int nr = __builtin_amdgcn_readfirstlane((int)g.tasks[t].nreq);
  for (int q0 = 0; q0 < nr; q0 += 64) {
    bool ok = true;
    if (q0 + l < nr) {
      const int2 rq = g.reqs[rb + q0 + l];
      ok = ld_sc1(g.cnt + rq.x) >= rq.y;
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
  }
  return true;
}

// one CAS claim attempt on a low list (wave 0): the task, -1 (head not ready), -2 (list exhausted)
__device__ inline int try_list(const DtrArgs& g, int* cur, const int* list, int n) {
  for (int tries = 0; tries < 4; ++tries) {
    const int h = __builtin_amdgcn_readfirstlane(ld_sc1(cur));
    if (h >= n) return -2;
    const int t = __builtin_amdgcn_readfirstlane(list[h]);
    if (!ready_wave(g, t)) return -1;
    int won = 0;
    if ((threadIdx.x & 63) == 0) won = atomicCAS(cur, h, h + 1) == h;
    if (__builtin_amdgcn_readfirstlane(won)) return t;
  }
  return -1;
}

// wave 0: a ready task of the low lists -- its own XCD's list, another XCD's only once its own is
// exhausted (-1 none ready yet, -2 every low list exhausted)
__device__ inline int claim_low(const DtrArgs& g, int xcd) {
  const int own = try_list(g, g.cur + PSTRIDE * (1 + xcd), g.lo + g.lo_off[xcd], g.lo_off[xcd + 1] - g.lo_off[xcd]);
  if (own >= 0) return own;
  if (own == -1) {
    if (!(g.flags & 1)) return -1;
    // flags bit 0: the own head waits on a dependency -- take a READY head of another XCD's list instead
    // (any claimed task is ready, so the deadlock-freedom argument is unchanged; L2 locality is traded away)
    for (int d = 1; d < 8; ++d) {
      const int x = (xcd + d) & 7;
      const int t = try_list(g, g.cur + PSTRIDE * (1 + x), g.lo + g.lo_off[x], g.lo_off[x + 1] - g.lo_off[x]);
      if (t >= 0) return t;
    }
    return -1;
  }
  bool all_done = true;
  for (int d = 1; d < 8; ++d) {
    const int x = (xcd + d) & 7;
    const int t = try_list(g, g.cur + PSTRIDE * (1 + x), g.lo + g.lo_off[x], g.lo_off[x + 1] - g.lo_off[x]);
    if (t >= 0) return t;
    if (t == -1) all_done = false;
  }
  return all_done ? -2 : -1;
}

struct UpdKs {   // k-run of an update: L(i,k) strip r, L(j,k) strip c, k in [k0, k0+nk)
  long long si, sj;
  int i, j, r, c, k0;
  __device__ KPair operator()(int t) const {
    KPair p;
    p.a_off = toff(si, sj, i, k0 + t) + 128 * r;
    p.b_off = toff(si, sj, j, k0 + t) + 128 * c;
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
__device__ void w_column(const DtrArgs& g, int k, int b, double* Vb) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int a = w >> 1, bh = w & 1;        // this wave's quadrant (row half a, column half bh)
  const int base = g.epoch * 64;
  const double* Mb = g.Mw + ((size_t)k * MAXB + b) * BLK;
  const double* Sb = g.Sw + ((size_t)k * MAXB + b) * RB;
  double* Lpk = g.Lp + (size_t)k * MAXB * MAXB * BLK;
  double* Wpk = g.Wp + (size_t)k * MAXB * MAXB * BLK;
  int* wprog = g.prog + ((size_t)k * 2 + 1) * MAXB * PSTRIDE;
  double* Wk = g.W + (size_t)k * NBT * NBT;
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
  int i, j, k0, r, c, nk;
  double* A;
  long long ld, si, sj;
  __device__ TaskU(const DtrArgs& g, int t) {
    const DtrTask tk = g.tasks[t];
    i = rfl(tk.i);
    j = rfl(tk.j);
    k0 = rfl(tk.k0);
    r = rfl(tk.r);
    c = rfl(tk.c);
    nk = rfl(tk.nk);
    A = rflp(g.A);
    ld = rfl64(g.ld);
    si = rfl64(g.si);
    sj = rfl64(g.sj);
  }
};

// Task bodies: each is a separate (non-inlined) function, so its registers are allocated on its own
// -- the GEMM body inlined into the task loop spilled (the capped persistent k_gemm_full spills the
// same way: hipcc -Rpass-analysis=kernel-resource-usage, profiles/r4_dtr_regs.txt).
__device__ __attribute__((noinline)) void run_upd(const DtrArgs* __restrict__ gp, int t) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t));
  __builtin_amdgcn_s_setprio(0);
  const UpdKs ks{u.si, u.sj, u.i, u.j, u.r, u.c, u.k0};
  const int uplo = (u.i == u.j && u.r == u.c) ? 1 : 0;
  gemm_subtile<double, false, true>(g_lds, ks, u.nk, 0, 0, uplo, -1.0, u.A, (int)u.ld, u.A, (int)u.ld, 1.0,
                                    u.A + toff(u.si, u.sj, u.i, u.j) + 128 * u.r + 128LL * u.c * u.ld, (int)u.ld);
}

__device__ __attribute__((noinline)) void run_trsm(const DtrArgs* __restrict__ gp, int t) {
  const DtrArgs& g = *uni(gp);
  const TaskU u(g, rfl(t));
  __builtin_amdgcn_s_setprio(2);
  const long long ao = toff(u.si, u.sj, u.i, u.k0) + 128 * u.r;
  const double* Wk = rflp(g.W) + (size_t)u.k0 * NBT * NBT;
  for (int c = 3; c >= 0; --c) {
    const TrsmKs ks{ao, c};
    gemm_subtile<double, false, false>(g_lds, ks, 1, 0, 0, 0, 1.0, u.A, (int)u.ld, Wk, NBT, 0.0,
                                       u.A + ao + 128LL * c * u.ld, (int)u.ld);
    __syncthreads();   // LDS image reuse (block c-1 never reads the columns block c wrote)
  }
}

__device__ __attribute__((noinline)) void run_potrf(const DtrArgs* __restrict__ gp, int t) {
  const DtrArgs& g = *uni(gp);
  t = __builtin_amdgcn_readfirstlane(t);
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
  rb_tile_body<true>(g.A + toff(g.si, g.sj, k, k), NBT, (int)g.ld, g.info, k * NBT, ws, g.epoch, nullptr, b, g_lds,
                     g_lds + BLK);
  __syncthreads();
  w_column(g, k, b, g_lds);
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
  for (;;) {
    const DtrArgs* gp = gargs;
    asm volatile("" : "+s"(gp));
    const DtrArgs& g = *gp;
    if (tid < 64) {
      int t = -1;
      if (ld_sc1(g.info) == -1000) {
        t = -2;
      } else {
        if (ticket < 0 && !hi_done) {
          // a ticket only for a ready head: a workgroup holding a not-yet-ready critical task would run
          // low-list tasks meanwhile and come back up to one bulk task late -- the 16 POTRF workgroups of
          // a tile would then start spread over ~0.4 ms and wait for each other
          const int h = __builtin_amdgcn_readfirstlane(ld_sc1(g.cur));
          if (h >= g.nhi) {
            hi_done = true;
          } else if (ready_wave(g, __builtin_amdgcn_readfirstlane(g.hi[h]))) {
            int tk = 0;
            if (tid == 0) tk = atomicAdd(g.cur, 1);
            tk = __builtin_amdgcn_readfirstlane(tk);
            if (tk < g.nhi) {
              ticket = tk;
              ticket_t0 = __builtin_amdgcn_s_memrealtime();
            } else {
              hi_done = true;
            }
          }
        }
        bool help = true;
        if (ticket >= 0) {
          const int th = __builtin_amdgcn_readfirstlane(g.hi[ticket]);
          if (ready_wave(g, th)) {
            t = th;
            ticket = -1;
          } else if (__builtin_amdgcn_readfirstlane(g.tasks[th].type) == T_POTRF &&
                     __builtin_amdgcn_s_memrealtime() - ticket_t0 < 5000ULL) {
            help = false;   // a POTRF ticket polls for its first 50 us (the group starts together), then helps
          }
        }
        if (t < 0 && help && !lo_done) {
          t = claim_low(g, xcd);
          if (t == -2) {
            lo_done = true;
            t = -1;
          }
        }
        if (t < 0) t = (hi_done && lo_done && ticket < 0) ? -2 : -1;
      }
      if (t >= 0) {
        if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the predecessors' bytes, fresh in this CU
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        idle0 = 0;
      } else if (t == -1 && tid == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (idle0 == 0) idle0 = now;
        else if (now - idle0 > 400000000ULL) {   // 4 s without a ready task: broken schedule, drain
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
    long long t_start = 0;
    if (g.trace && tid == 0) t_start = (long long)__builtin_amdgcn_s_memrealtime();
    const DtrTask tk = g.tasks[t];
    if (tk.type == T_UPD) run_upd(gp, t);
    else if (tk.type == T_TRSM) run_trsm(gp, t);
    else run_potrf(gp, t);
    // release: every wave's stores drained, then one agent-scope release and the counter bump
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && g.trace) {
      long long* tr = g.trace + 3 * (size_t)t;
      tr[0] = t_start;
      tr[1] = (long long)__builtin_amdgcn_s_memrealtime();
      tr[2] = ((long long)blockIdx.x << 8) | xcd;
    }
    if (tid == 0 && tk.inc >= 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(g.cnt + tk.inc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

}  // namespace

// One DTR Cholesky launch (see the header).  args: a DtrArgs image built by the host (models/potrf_dtr.py
// fills it through dpl_dtr_args_size / the field offsets below), grid = 2 x #CUs workgroups.
DPL_API int dpl_dtr_args_size() { return (int)sizeof(DtrArgs); }
DPL_API int dpl_dtr_lds_doubles() { return LDS_D; }
// args_dev: the DtrArgs image in device memory (uploaded by the host before the launch)
DPL_API int dpl_dtr_potrf(const void* args_dev, int nwg, hipStream_t st) {
  if (nwg <= 0 || !args_dev) return -3;
  hipLaunchKernelGGL(k_dtr_potrf, dim3(nwg), dim3(256), 0, st, (const DtrArgs*)args_dev);
  return (int)hipGetLastError();
}
// offsets of DtrArgs fields (the host packs the struct without a C compiler)
DPL_API int dpl_dtr_args_layout(long long* off, int n) {
  const long long v[] = {
      (long long)offsetof(DtrArgs, A),      (long long)offsetof(DtrArgs, ld),     (long long)offsetof(DtrArgs, si),
      (long long)offsetof(DtrArgs, sj),     (long long)offsetof(DtrArgs, nt),
      (long long)offsetof(DtrArgs, tasks),  (long long)offsetof(DtrArgs, reqs),   (long long)sizeof(DtrTask),
      (long long)offsetof(DtrArgs, cnt),    (long long)offsetof(DtrArgs, cur),    (long long)offsetof(DtrArgs, hi),
      (long long)offsetof(DtrArgs, nhi),    (long long)offsetof(DtrArgs, lo),     (long long)offsetof(DtrArgs, lo_off),
      (long long)offsetof(DtrArgs, W),      (long long)offsetof(DtrArgs, Mw),     (long long)offsetof(DtrArgs, Sw),
      (long long)offsetof(DtrArgs, Lp),     (long long)offsetof(DtrArgs, Wp),     (long long)offsetof(DtrArgs, prog),
      (long long)offsetof(DtrArgs, epoch),  (long long)offsetof(DtrArgs, info),   (long long)offsetof(DtrArgs, trace),
      (long long)sizeof(DtrArgs),
      (long long)MAXB, (long long)BLK, (long long)RB, (long long)PSTRIDE, (long long)offsetof(DtrArgs, flags)};
  const int m = (int)(sizeof(v) / sizeof(v[0]));
  for (int q = 0; q < n && q < m; ++q) off[q] = v[q];
  return m;
}
