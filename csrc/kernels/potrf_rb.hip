// Dataflow Cholesky of one diagonal tile over several workgroups (fp64, n <= 512).
//
// Reference role: the potrf_zpotrf task body (src/zpotrf_L.jdf:93-188; its GPU incarnation calls
// cusolverDnZpotrf, its CPU one CORE_zpotrf -> LAPACKE_zpotrf_work, src/cores/core_zpotrf.c:68-74)
// with the reference's info convention *INFO = k*mb + iinfo (src/zpotrf_L.jdf:180-182).
//
// Why a new kernel: the single-workgroup left-looking k_potrf_ll (potrf_trsm.hip) re-streams the
// whole left panel through ONE CU for every 16-column step (~n^3/6 doubles through one CU's L1/L2
// port) and is latency-bound at ~625 us for a 512 tile.  This kernel spreads the tile over
// ceil(n/32) workgroups, one 32-row block each, with the block row RESIDENT IN LDS for the whole
// factorisation (block 15 of a 512 tile = 16 x 8 KB), and runs a right-looking dataflow schedule:
//
//   WG i, step k < i:  wait Z_k = inv(L(k,k)) (published by WG k)
//                      L(i,k) = A(i,k) Z_k^T              (MFMA, 4 waves = 4 16x16 quadrants)
//                      publish L(i,k) (one wave, write-through stores + flag)
//                      A(i,j) -= L(i,k) L(j,k)^T, j = k+1..i  (L(j,k) from WG j's publication)
//   WG i, step i:      Cholesky + inverse of the 32x32 diagonal block on one wave, publish Z_i.
//
// Only 15 hand-offs sit on the critical path (Z_k -> WG k+1), each followed by one 32x32 TRSM,
// one SYRK and one 32x32 factorisation.  Workgroups only ever wait on workgroups with a SMALLER
// LOGICAL index, and the logical index is a ticket taken with one atomic when the workgroup
// starts (not blockIdx.x): every workgroup a waiter depends on has therefore already started, so
// forward progress does not rest on the hardware dispatching blockIdx in order across the 8 XCDs
// or beside other queues' kernels.  Every spin is bounded anyway (info = -1000 after ~2 s).
//
// Flag initialisation is stream-ordered: a workspace slot's flags and ticket are zeroed with
// hipMemsetAsync on the stream that first launches into it.  (Round 3 zeroed them with
// hipMemset on the null stream + hipDeviceSynchronize; a rocprofv3 trace of the headline bench,
// gpurun_out/b4_prof, shows six of those fills executing AFTER the first k_potrf_rb had started
// on a non-blocking stream -- the kernel's first flags were wiped and its waiters timed out.)
//
// Data layout ("T-layout"): a 32x32 block is stored as 4 quadrants x 4 registers x 64 lanes;
// lane l, register r of quadrant q = (rh, ch) holds element
//     (16 rh + (l & 15), 16 ch + (l >> 4) + 4 r).
// It is simultaneously (a) the accumulator layout of v_mfma_f64_16x16x4 when the product is formed
// as D = Y X^T-transposed (A operand = Y, B operand = X), and (b) the A/B operand layout of the same
// instruction for k-chunk u = 4 ch + r.  Every LDS and workspace access is therefore one
// lane-contiguous 8-byte access (conflict-free, coalesced), and MFMA results are stored without
// any shuffle.
//
// Hand-off protocol (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility",
// first row of the sc1 table): payload stored with agent-scope relaxed atomics (sc1, write-through),
// s_waitcnt vmcnt(0) in every storing wave, one lane's sc1 flag store; consumers poll the flag with
// sc1 loads and read every handed-off byte with sc1 loads.  Flags carry a per-launch epoch, so no
// reset is needed between launches.
#include <mutex>

#include "common.h"
#include "grid_sync.h"

#include "potrf_tile.h"

namespace {
using namespace rbk;

template <bool LOWER>
__global__ __launch_bounds__(256) void k_potrf_rb(double* __restrict__ A, int n, int lda, int* __restrict__ info,
                                                  int info_base, RbWork ws, int epoch,
                                                  unsigned long long* __restrict__ trace) {
  __shared__ double Tb[BLK], Xb[BLK];
  rb_tile_body<LOWER>(A, n, lda, info, info_base, ws, epoch, trace, wg_ticket(ws), Tb, Xb);
}

std::mutex g_mu;
RbWork g_ws[64][NSLOT];
bool g_have[64] = {};
unsigned int g_launch = 0;
hipStream_t g_slot_stream[64][NSLOT] = {};
bool g_slot_used[64][NSLOT] = {};
bool g_slot_zeroed[64][NSLOT] = {};    // flags + ticket zeroed on the slot's current stream
unsigned int g_slot_tick[64][NSLOT] = {};
unsigned int g_slot_wgs[64][NSLOT] = {};  // tickets handed out so far (= next launch's tbase)

// nwg: workgroups of the launch that will use the workspace (advances the slot's ticket base)
int get_ws(RbWork* out, int* epoch, hipStream_t st, int nwg) {
  int dev = 0;
  HIP_CHECK_RET(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return -4;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_have[dev]) {
    for (int s = 0; s < NSLOT; ++s) {
      RbWork& w = g_ws[dev][s];
      HIP_CHECK_RET(hipMalloc((void**)&w.M, sizeof(double) * MAXB * BLK));
      HIP_CHECK_RET(hipMalloc((void**)&w.S, sizeof(double) * MAXB * RB));
      HIP_CHECK_RET(hipMalloc((void**)&w.Lp, sizeof(double) * MAXB * MAXB * BLK));
      // flags, then one 128-byte line for the ticket counter
      HIP_CHECK_RET(hipMalloc((void**)&w.prog, sizeof(int) * (MAXB + 1) * PSTRIDE));
      w.ticket = (unsigned*)(w.prog + MAXB * PSTRIDE);
      g_slot_zeroed[dev][s] = false;
    }
    g_have[dev] = true;
  }
  ++g_launch;
  if ((g_launch & 0x1ffffff) == 0) {  // epoch wrap (every 2^25 launches): every slot re-zeroed on its next use
    HIP_CHECK_RET(hipDeviceSynchronize());
    for (int s = 0; s < NSLOT; ++s) g_slot_zeroed[dev][s] = false;
    ++g_launch;
  }
  // One workspace per stream: launches on one stream are serialised, so they can share it; launches
  // on different streams (which may run concurrently, the whole program being enqueued ahead) never
  // do.  Beyond NSLOT streams the least recently used stream's slot is recycled after that stream
  // has drained (a host wait, only when more than NSLOT streams launch tile kernels).
  int slot = -1, lru = 0;
  for (int s = 0; s < NSLOT; ++s) {
    if (g_slot_stream[dev][s] == st && g_slot_used[dev][s]) slot = s;
    if (!g_slot_used[dev][s] || (g_slot_used[dev][lru] && g_slot_tick[dev][s] < g_slot_tick[dev][lru])) lru = s;
  }
  if (slot < 0) {
    slot = lru;
    if (g_slot_used[dev][slot]) (void)hipStreamSynchronize(g_slot_stream[dev][slot]);  // may be destroyed: ignore
    g_slot_stream[dev][slot] = st;
    g_slot_used[dev][slot] = true;
  }
  RbWork& w = g_ws[dev][slot];
  if (!g_slot_zeroed[dev][slot]) {  // ordered before this launch by the stream itself
    HIP_CHECK_RET(hipMemsetAsync(w.prog, 0, sizeof(int) * (MAXB + 1) * PSTRIDE, st));
    g_slot_wgs[dev][slot] = 0;
    g_slot_zeroed[dev][slot] = true;
  }
  g_slot_tick[dev][slot] = g_launch;
  w.tbase = g_slot_wgs[dev][slot];
  g_slot_wgs[dev][slot] += (unsigned)nwg;
  *out = w;
  *epoch = (int)(g_launch & 0x1ffffff);
  return 0;
}
unsigned long long* g_trace = nullptr;
}  // namespace

// debug: record per-workgroup phase timestamps of the next launches into buf (64 x 8 B per WG)
DPL_API int dpl_potrf_rb_set_trace(void* buf) {
  g_trace = (unsigned long long*)buf;
  return 0;
}

// Cholesky of one n x n fp64 tile (n <= 512) in place; returns -3 when the shape is not supported.
// zbuf (optional, ZBUF doubles): receives (M_k, S_k) of every diagonal 32-block for dpl_trsm_rb.
DPL_API int dpl_potrf_tile_rbz(int uplo, int n, double* A, int lda, int* info, int info_base, double* zbuf,
                               hipStream_t st) {
  if (n <= 0) return 0;
  if (n > RB * MAXB) return -3;
  const int nblk = cdiv(n, RB);
  RbWork ws;
  int epoch = 0;
  const int rc = get_ws(&ws, &epoch, st, nblk);
  if (rc) return rc;
  if (zbuf) {
    ws.M = zbuf;
    ws.S = zbuf + MAXB * BLK;
  }
  if (uplo == DPL_LOWER)
    hipLaunchKernelGGL((k_potrf_rb<true>), dim3(nblk), dim3(256), 0, st, A, n, lda, info, info_base, ws, epoch, g_trace);
  else
    hipLaunchKernelGGL((k_potrf_rb<false>), dim3(nblk), dim3(256), 0, st, A, n, lda, info, info_base, ws, epoch, g_trace);
  return (int)hipGetLastError();
}

DPL_API int dpl_potrf_tile_rb(int uplo, int n, double* A, int lda, int* info, int info_base, hipStream_t st) {
  return dpl_potrf_tile_rbz(uplo, n, A, lda, info, info_base, nullptr, st);
}

// Fused tile Cholesky + panel solve (k_potrf_trsm_rb): the tile at A, the panel strips in B
// (device RbItem[nrb], offsets relative to B); zbuf (optional) receives (M, S) as in dpl_potrf_tile_rbz.
DPL_API int dpl_potrf_trsm_rb(int uplo, int n, double* A, int lda, int* info, int info_base, double* zbuf, int nrb,
                              const void* items, double* B, int ldb, hipStream_t st);

// ================================================================== panel TRSM on the (M, S) blocks
// B := B L^{-T} for every 16-row strip of the panel tiles below a diagonal tile factored by
// k_potrf_rb (or prepared by k_trsm_rb_prep): the right-looking block substitution of the same
// dataflow, without waiting -- every (M_k, S_k) and L(j,k) is final when this launch starts.
// One wave per 16-row strip and no barrier at all: the strip (16 x 512) stays in the wave's
// registers for the whole solve, as the T-layout quadrants of its <= 16 column blocks -- the
// accumulator layout of the MFMA products is also the B-operand layout of the next ones, so
// L(R,k) = C(R,k) M_k^T diag(S_k) feeds the updates C(R,j) -= L(R,k) L(j,k)^T straight from
// registers.  L(j,k) is read from the factored tile (L2-resident, shared by every strip).
// Reference role: the potrf_ztrsm tasks (src/zpotrf_L.jdf:194-243).
constexpr int TR_ROWS = 16;
#ifndef TR_GRP
#define TR_GRP 3  // update blocks whose operands are fetched together
#endif
struct RbItem {
  long long b_off;  // element offset of the strip in B
  int rows;         // <= TR_ROWS
  int pad;
};

template <bool LOWER, int NBLK>  // NBLK = ceil(n / 32): static, so the strip never needs runtime guards
__global__ __launch_bounds__(64) void k_trsm_rb(const RbItem* __restrict__ items, int n,
                                                const double* __restrict__ Lt, int ldl,
                                                const double* __restrict__ zb, double* __restrict__ B, int ldb) {
  __builtin_amdgcn_s_setprio(RB_PRIO);
  const RbItem it = items[blockIdx.x];
  const int l = threadIdx.x;
  const long long sib = LOWER ? 1 : ldb, sjb = LOWER ? ldb : 1;
  const long long sil = LOWER ? 1 : ldl, sjl = LOWER ? ldl : 1;
  const int row = l & 15;
  const bool rok = row < it.rows;
  double* Bb = B + it.b_off;
  const double* Sz = zb + MAXB * BLK;
  // operands of the next solve / update are fetched one operation ahead (software pipeline)
  auto load_m = [&](int k, double* m) {  // M_k rows of both halves (12 chunks) + the 8 S values
    const double* Mk = zb + (size_t)k * BLK;
#pragma unroll
    for (int u = 0; u < 4; ++u) m[u] = Mk[(4 * u + (l >> 4)) * RB + (l & 15)];
#pragma unroll
    for (int u = 0; u < 8; ++u) m[4 + u] = Mk[(4 * u + (l >> 4)) * RB + 16 + (l & 15)];
#pragma unroll
    for (int q = 0; q < 8; ++q) m[12 + q] = Sz[k * RB + 16 * (q >> 2) + (l >> 4) + 4 * (q & 3)];
  };
  auto load_y = [&](int k, int jb, double* y) {  // L(jb, k), both row halves, T-layout chunks
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lr = RB * jb + 16 * h + (l & 15);
#pragma unroll
      for (int u = 0; u < 8; ++u) y[8 * h + u] = (lr < n) ? Lt[lr * sil + (RB * k + 4 * u + (l >> 4)) * sjl] : 0.0;
    }
  };
  d4_t C[NBLK][2];
  // Upper: a strip row is a COLUMN of U(k, i) (contiguous in memory) and the T-layout's 16 row lanes
  // would stride by ldb (32-byte segments).  Stage each 16 x 32 block through LDS instead: lane l
  // moves 8 consecutive elements of strip row l / 4 (4 lanes = one 256-byte run), then reads its
  // T-layout values back (row stride 33 doubles: conflict-free).
  __shared__ double stg[LOWER ? 1 : TR_ROWS * 33];
  const int srow = l >> 2, scol = (l & 3) * 8;
  const bool sok = srow < it.rows;
  if constexpr (LOWER) {
#pragma unroll
    for (int jb = 0; jb < NBLK; ++jb)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = RB * jb + 16 * h + (l >> 4) + 4 * r;
          C[jb][h][r] = (rok && col < n) ? Bb[row * sib + col * sjb] : 0.0;
        }
  } else {
#pragma unroll
    for (int jb = 0; jb < NBLK; ++jb) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = RB * jb + scol + e;
        stg[srow * 33 + scol + e] = (sok && col < n) ? Bb[(long long)srow * ldb + col] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) C[jb][h][r] = rok ? stg[row * 33 + 16 * h + (l >> 4) + 4 * r] : 0.0;
      __syncthreads();
    }
  }
  double mc[20];
#pragma unroll
  for (int k = 0; k < NBLK; ++k) {
    load_m(k, mc);
    // L(R,k) = C(R,k) M_k^T diag(S_k)
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = C[k][u >> 2][u & 3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      d4_t acc = {0, 0, 0, 0};
      if (h == 0) acc = mfma_chunks<4>(mc, x, acc);
      else acc = mfma_chunks<8>(mc + 4, x, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * h + (l >> 4) + 4 * r;
        acc[r] *= mc[12 + 4 * h + r];
        if constexpr (LOWER) {
          if (rok && RB * k + c < n) Bb[row * sib + (RB * k + c) * sjb] = acc[r];  // final L(R,k)
        } else {
          stg[row * 33 + c] = acc[r];
        }
      }
      C[k][h] = acc;
    }
    if constexpr (!LOWER) {  // final U(k, R) columns: back through LDS, 256-byte runs per strip row
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = RB * k + scol + e;
        if (sok && col < n) Bb[(long long)srow * ldb + col] = stg[srow * 33 + scol + e];
      }
      __syncthreads();
    }
    double xm[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xm[u] = -C[k][u >> 2][u & 3];
    // updates in groups of TR_GRP blocks: the group's operand loads are all in flight together
#pragma unroll
    for (int j0 = k + 1; j0 < NBLK; j0 += TR_GRP) {
      double y[TR_GRP][16];
#pragma unroll
      for (int g = 0; g < TR_GRP; ++g)
        if (j0 + g < NBLK) load_y(k, j0 + g, y[g]);
#pragma unroll
      for (int g = 0; g < TR_GRP; ++g)
        if (j0 + g < NBLK) {
          C[j0 + g][0] = mfma_chunks<8>(y[g], xm, C[j0 + g][0]);
          C[j0 + g][1] = mfma_chunks<8>(y[g] + 8, xm, C[j0 + g][1]);
        }
    }
  }
}

// ================================================================== fused tile POTRF + panel TRSM
// One launch: workgroups 0..NBLK-1 factor the diagonal tile exactly as k_potrf_rb; every further
// workgroup solves four 16-row strips of the panel (one per wave) *along the factorisation
// wavefront*: strip step k starts as soon as (M_k, S_k) and the blocks L(j,k), j > k, are published
// (the same epoch-tagged flags the tile workgroups hand off with), reading them write-through from
// the workspace.  The panel solve therefore overlaps the tile factorisation instead of following
// it, and its workgroups are dispatched while the tile is still being factored -- beside a bulk
// GEMM the separate TRSM launch waited ~1 ms for free slots (profiles/r2_potrf16k_timeline.txt).
// Deadlock-free for the same reason as the tile kernel: a workgroup only ever waits on workgroups
// with a smaller index (in-order dispatch); every spin is bounded.
#ifndef TR_GRP_FUSED
#define TR_GRP_FUSED 2  // fewer operand registers than k_trsm_rb: the fused kernel also holds the tile path
#endif
// one step k of a strip (compile-time k: the register arrays are indexed statically, and the
// bounded flag spin cannot keep the compiler from unrolling the step sequence)
template <bool LOWER, int NBLK, int K>
__device__ __forceinline__ void rb_strip_step(d4_t (&C)[NBLK][2], const RbWork& ws, int base, int* __restrict__ info,
                                              double* __restrict__ Bb, long long sib, long long sjb, bool rok,
                                              int row, int n, int l) {
  if constexpr (K < NBLK) {
    // (M_K, S_K) and every L(j,K), j > K, published
    if (l == 0) {
#pragma nounroll
      for (int j = K; j < NBLK; ++j) spin_until(ws.prog + j * PSTRIDE, base + K + 1, info);
    }
    __builtin_amdgcn_wave_barrier();
    double mc[20];
    const double* Mk = ws.M + (size_t)K * BLK;
#pragma unroll
    for (int u = 0; u < 4; ++u) mc[u] = ld_sc1(Mk + (4 * u + (l >> 4)) * RB + (l & 15));
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[4 + u] = ld_sc1(Mk + (4 * u + (l >> 4)) * RB + 16 + (l & 15));
#pragma unroll
    for (int q = 0; q < 8; ++q) mc[12 + q] = ld_sc1(ws.S + (size_t)K * RB + 16 * (q >> 2) + (l >> 4) + 4 * (q & 3));
    // L(R,K) = C(R,K) M_K^T diag(S_K)
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = C[K][u >> 2][u & 3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      d4_t acc = {0, 0, 0, 0};
      if (h == 0) acc = mfma_chunks<4>(mc, x, acc);
      else acc = mfma_chunks<8>(mc + 4, x, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * h + (l >> 4) + 4 * r;
        acc[r] *= mc[12 + 4 * h + r];
        if (rok && RB * K + c < n) Bb[row * sib + (RB * K + c) * sjb] = acc[r];  // final L(R,K)
      }
      C[K][h] = acc;
    }
    double xm[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xm[u] = -C[K][u >> 2][u & 3];
    // C(R,j) -= L(R,K) L(j,K)^T: L(j,K) from the workspace (T-layout, both row halves)
#pragma unroll
    for (int j0 = K + 1; j0 < NBLK; j0 += TR_GRP_FUSED) {
      double y[TR_GRP_FUSED][16];
#pragma unroll
      for (int g = 0; g < TR_GRP_FUSED; ++g)
        if (j0 + g < NBLK) {
          const double* Yp = ws.Lp + ((size_t)(j0 + g) * MAXB + K) * BLK;
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int u = 0; u < 8; ++u) y[g][8 * h + u] = ld_sc1(Yp + qoff(h, u, l));
        }
#pragma unroll
      for (int g = 0; g < TR_GRP_FUSED; ++g)
        if (j0 + g < NBLK) {
          C[j0 + g][0] = mfma_chunks<8>(y[g], xm, C[j0 + g][0]);
          C[j0 + g][1] = mfma_chunks<8>(y[g] + 8, xm, C[j0 + g][1]);
        }
    }
    rb_strip_step<LOWER, NBLK, K + 1>(C, ws, base, info, Bb, sib, sjb, rok, row, n, l);
  }
}

template <bool LOWER, int NBLK>
__device__ inline void rb_strip_dataflow(const RbItem it, int n, const RbWork& ws, int base, int* __restrict__ info,
                                         double* __restrict__ B, int ldb) {
  const int l = threadIdx.x & 63;
  const long long sib = LOWER ? 1 : ldb, sjb = LOWER ? ldb : 1;
  const int row = l & 15;
  const bool rok = row < it.rows;
  double* Bb = B + it.b_off;
  d4_t C[NBLK][2];
#pragma unroll
  for (int jb = 0; jb < NBLK; ++jb)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = RB * jb + 16 * h + (l >> 4) + 4 * r;
        C[jb][h][r] = (rok && col < n) ? Bb[row * sib + col * sjb] : 0.0;
      }
  rb_strip_step<LOWER, NBLK, 0>(C, ws, base, info, Bb, sib, sjb, rok, row, n, l);
}

template <bool LOWER, int NBLK>
__global__ __launch_bounds__(256) void k_potrf_trsm_rb(double* __restrict__ A, int n, int lda, int* __restrict__ info,
                                                       int info_base, RbWork ws, int epoch,
                                                       const RbItem* __restrict__ items, int nrb,
                                                       double* __restrict__ B, int ldb) {
  const int id = wg_ticket(ws);
  if (id < NBLK) {
    __shared__ double Tb[BLK], Xb[BLK];
    rb_tile_body<LOWER>(A, n, lda, info, info_base, ws, epoch, nullptr, id, Tb, Xb);
    return;
  }
  __builtin_amdgcn_s_setprio(RB_PRIO);
  const int strip = (id - NBLK) * 4 + (threadIdx.x >> 6);
  if (strip >= nrb) return;
  rb_strip_dataflow<LOWER, NBLK>(items[strip], n, ws, epoch * 64, info, B, ldb);
}

// (M_k, S_k) of every 32x32 diagonal block of a factored tile L (for ranks that received L):
// row elimination of L_kk applied to I (M L_kk = diag(L_kk)), so inv(L_kk) = diag(1 / L_kk(p,p)) M.
template <bool LOWER>
__global__ __launch_bounds__(64) void k_trsm_rb_prep(int n, const double* __restrict__ Lt, int ldl,
                                                     double* __restrict__ zb) {
  __builtin_amdgcn_s_setprio(RB_PRIO);
  const int k = blockIdx.x, l = threadIdx.x;
  const long long sil = LOWER ? 1 : ldl, sjl = LOWER ? ldl : 1;
  const int j = l & 31;
  const bool mhalf = l >= RB;
  double col[RB];
#pragma unroll
  for (int p = 0; p < RB; ++p) {
    const int gr = RB * k + p, gc = RB * k + j;
    const double v = (gr < n && gc < n) ? Lt[gr * sil + gc * sjl] : (gr == gc ? 1.0 : 0.0);
    col[p] = mhalf ? ((p == j) ? 1.0 : 0.0) : ((p >= j) ? v : 0.0);
  }
#pragma unroll
  for (int c = 0; c < RB; ++c) {
    const double d = readlane_d(col[c], c);
    double akc[RB];
#pragma unroll
    for (int p = c + 1; p < RB; ++p) akc[p] = readlane_d(col[p], c);
    const double t = col[c] * rcp_d(d);
    if (mhalf) {
#pragma unroll
      for (int p = c + 1; p < RB; ++p) col[p] = fma(-akc[p], t, col[p]);
    }
  }
  double dj = 1.0;
#pragma unroll
  for (int p = 0; p < RB; ++p)
    if (p == j) dj = col[p];
  if (mhalf) {
    double* Mk = zb + (size_t)k * BLK + j * RB;
#pragma unroll
    for (int p = 0; p < RB; ++p) Mk[p] = col[p];
  } else {
    zb[MAXB * BLK + k * RB + j] = rcp_d(dj);
  }
}

DPL_API int dpl_potrf_zbuf_size() { return ZBUF; }

DPL_API int dpl_trsm_rb_prep(int uplo, int n, const double* L, int ldl, double* zbuf, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > RB * MAXB) return -3;
  const int nblk = cdiv(n, RB);
  if (uplo == DPL_LOWER)
    hipLaunchKernelGGL((k_trsm_rb_prep<true>), dim3(nblk), dim3(64), 0, st, n, L, ldl, zbuf);
  else
    hipLaunchKernelGGL((k_trsm_rb_prep<false>), dim3(nblk), dim3(64), 0, st, n, L, ldl, zbuf);
  return (int)hipGetLastError();
}

// items: device RbItem[nrb] (16-row strips of the panel tiles, offsets relative to B)
DPL_API int dpl_trsm_rb(int uplo, int n, const double* L, int ldl, const double* zbuf, int nrb, const void* items,
                        double* B, int ldb, hipStream_t st) {
  if (n <= 0 || nrb <= 0) return 0;
  if (n > RB * MAXB) return -3;
  const int nblk = cdiv(n, RB);
  const RbItem* it = (const RbItem*)items;
#define TRSM_RB_CASE(NB_)                                                                              \
  case NB_:                                                                                            \
    if (uplo == DPL_LOWER)                                                                             \
      hipLaunchKernelGGL((k_trsm_rb<true, NB_>), dim3(nrb), dim3(64), 0, st, it, n, L, ldl, zbuf, B, ldb);  \
    else                                                                                               \
      hipLaunchKernelGGL((k_trsm_rb<false, NB_>), dim3(nrb), dim3(64), 0, st, it, n, L, ldl, zbuf, B, ldb); \
    break;
  switch (nblk) {
    TRSM_RB_CASE(1) TRSM_RB_CASE(2) TRSM_RB_CASE(3) TRSM_RB_CASE(4) TRSM_RB_CASE(5) TRSM_RB_CASE(6)
    TRSM_RB_CASE(7) TRSM_RB_CASE(8) TRSM_RB_CASE(9) TRSM_RB_CASE(10) TRSM_RB_CASE(11) TRSM_RB_CASE(12)
    TRSM_RB_CASE(13) TRSM_RB_CASE(14) TRSM_RB_CASE(15) TRSM_RB_CASE(16)
    default: return -3;
  }
#undef TRSM_RB_CASE
  return (int)hipGetLastError();
}

DPL_API int dpl_potrf_trsm_rb(int uplo, int n, double* A, int lda, int* info, int info_base, double* zbuf, int nrb,
                              const void* items, double* B, int ldb, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > RB * MAXB) return -3;
  if (nrb <= 0) return dpl_potrf_tile_rbz(uplo, n, A, lda, info, info_base, zbuf, st);
  const int nblk = cdiv(n, RB);
  const dim3 grid(nblk + cdiv(nrb, 4));
  RbWork ws;
  int epoch = 0;
  const int rc = get_ws(&ws, &epoch, st, (int)grid.x);
  if (rc) return rc;
  if (zbuf) {
    ws.M = zbuf;
    ws.S = zbuf + MAXB * BLK;
  }
  const RbItem* it = (const RbItem*)items;
#define POTRF_TRSM_CASE(NB_)                                                                              \
  case NB_:                                                                                               \
    if (uplo == DPL_LOWER)                                                                                \
      hipLaunchKernelGGL((k_potrf_trsm_rb<true, NB_>), grid, dim3(256), 0, st, A, n, lda, info, info_base, ws, \
                         epoch, it, nrb, B, ldb);                                                         \
    else                                                                                                  \
      hipLaunchKernelGGL((k_potrf_trsm_rb<false, NB_>), grid, dim3(256), 0, st, A, n, lda, info, info_base, ws, \
                         epoch, it, nrb, B, ldb);                                                         \
    break;
  switch (nblk) {
    POTRF_TRSM_CASE(1) POTRF_TRSM_CASE(2) POTRF_TRSM_CASE(3) POTRF_TRSM_CASE(4) POTRF_TRSM_CASE(5)
    POTRF_TRSM_CASE(6) POTRF_TRSM_CASE(7) POTRF_TRSM_CASE(8) POTRF_TRSM_CASE(9) POTRF_TRSM_CASE(10)
    POTRF_TRSM_CASE(11) POTRF_TRSM_CASE(12) POTRF_TRSM_CASE(13) POTRF_TRSM_CASE(14) POTRF_TRSM_CASE(15)
    POTRF_TRSM_CASE(16)
    default: return -3;
  }
#undef POTRF_TRSM_CASE
  return (int)hipGetLastError();
}
