// Device-resident partial-pivoting LU building blocks (no host round trip per step).
//
// Reference roles: CORE_zgetrf_rectil / _reclap -- the recursive, multithreaded panel of
// src/cores/core_zgetrf_rectil.c:120-279 (spin barriers + shared amax arrays between
// threads), the GETRF_MAX / GETRF_RDC / GETRF_SND pivot search of
// src/zgetrf_ptgpanel.jdf:206-590, and CORE_zlaswp / zlaswp_ontile (core_zlaswp.c:62-224).
//
// MI355X design:
//  * The tall panel (m up to 64k rows x NB columns, column-major, one buffer) is factored by a
//    recursive LU (host-side recursion in dplasma_amd.ops: halves -> laswp + TRSM + MFMA GEMM);
//    its base case is a column block of <= 64 columns handled by dpl_lu_block.  Real precisions run
//    it as ONE persistent launch with the block's rows in LDS and the per-column pivot chosen through
//    tagged granules (k_lu_block_tag, the default -- see there; the grid-barrier and register variants
//    stay selectable).  The fallback (complex, or panels taller than 256 rows x #CU) issues one launch
//    per column.  Launch j, over every row of the panel (256 rows per workgroup, one row per thread,
//    coalesced column-major reads):
//      1. applies column j-1: l = a(r, j-1) / a(j-1, j-1); a(r, j-1) = l;
//         a(r, c) -= l * a(j-1, c) for the block's columns c > j-1   (rank-1 update)
//      2. computes the workgroup's |max| of column j over its rows,
//      3. the LAST workgroup to finish (agent-scope release / ticket / acquire, per
//         cdna_hip_programming.md G16) reduces the partial maxima, records the pivot and swaps
//         the two rows across the block -- so the pivot search never leaves the GPU and the
//         next launch sees the swapped rows (kernel boundary).
//  * Trailing interchanges: dpl_piv_moves turns the sequential swaps (LAPACK ipiv) into the
//    net list of moved rows on the device (one thread, LDS hash of displaced rows), and
//    dpl_rows_gather / dpl_rows_scatter move those rows across any set of local tile columns
//    through a staging buffer (the rows' owners contribute, others write zeros, so on a P x Q
//    grid one all-reduce of the staging buffer inside the process column completes the
//    exchange -- SWAP_COLLECT / SWAP_SND of the reference without host planning).
#include "common.h"
#include "grid_sync.h"

#define LUR 256        // rows per workgroup (one per thread)
#define LU_MAXBW 64    // widest base block

template <typename T>
__device__ inline void last_wg_fence_ticket(int* cnt, int nwg, bool& last) {
  __shared__ int s_last;
  // every wave's stores are issued and drained before the workgroup's ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nwg - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  last = s_last;
}

// One column step of the blocked panel LU (see header).  Rows [row0, m) take part; row0 = j
// (rows above j are final).  Block columns [c0, cend); j in [c0, cend]:
//   j > c0   : apply column j-1 (scale + rank-1 update of columns j..cend-1)
//   j < cend : pivot search on column j, last workgroup swaps rows j <-> p over [c0, cend)
template <typename T>
__global__ __launch_bounds__(LUR) void k_lu_col(T* __restrict__ A, int ld, int m, int c0, int cend, int j,
                                                int* __restrict__ ipiv, typename ST<T>::real* __restrict__ wsv,
                                                int* __restrict__ wsi, int* __restrict__ cnt, int* __restrict__ info,
                                                int info_base, int pivot) {
  typedef typename ST<T>::real R;
  const int tid = threadIdx.x;
  const int r = j + blockIdx.x * LUR + tid;
  const bool in = r < m;
  // ---- 1. rank-1 update with column j-1 (pivot row j-1 is final)
  if (j > c0 && in) {
    const int jp = j - 1;
    const T d = A[jp + (long long)jp * ld];
    T l = A[r + (long long)jp * ld];
    if (!is_zero(d)) l = divv(l, d);
    A[r + (long long)jp * ld] = l;
    for (int c = j; c < cend; ++c) {
      const T u = A[jp + (long long)c * ld];
      A[r + (long long)c * ld] = sub(A[r + (long long)c * ld], mul(l, u));
    }
  }
  if (j >= cend || !pivot) {
    if (j < cend && !pivot && blockIdx.x == 0 && tid == 0) {
      ipiv[j] = j;
      if (is_zero(A[j + (long long)j * ld]) && info) atomicCAS(info, 0, info_base + j + 1);
    }
    return;
  }
  // ---- 2. workgroup |max| of column j (ties -> smallest row, LAPACK i?amax)
  __shared__ R sv[LUR];
  __shared__ int si[LUR];
  sv[tid] = in ? piv_mag(abs1(A[r + (long long)j * ld])) : R(-1);
  si[tid] = in ? r : 0x7fffffff;
  __syncthreads();
  for (int s = LUR / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const R a = sv[tid], b = sv[tid + s];
      if (b > a || (b == a && si[tid + s] < si[tid])) { sv[tid] = b; si[tid] = si[tid + s]; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    wsv[blockIdx.x] = sv[0];
    wsi[blockIdx.x] = si[0];
  }
  // ---- 3. last workgroup: global pivot, swap rows over the block
  bool last;
  last_wg_fence_ticket<T>(cnt, gridDim.x, last);
  if (!last) return;
  R best = R(-1);
  int bi = 0x7fffffff;
  for (int b = tid; b < (int)gridDim.x; b += LUR) {
    const R v = wsv[b];   // plain loads after the agent-scope acquire
    const int i = wsi[b];
    if (v > best || (v == best && i < bi)) { best = v; bi = i; }
  }
  sv[tid] = best;
  si[tid] = bi;
  __syncthreads();
  for (int s = LUR / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const R a = sv[tid], b = sv[tid + s];
      if (b > a || (b == a && si[tid + s] < si[tid])) { sv[tid] = b; si[tid] = si[tid + s]; }
    }
    __syncthreads();
  }
  const int p = si[0];
  if (p != j) {
    for (int c = c0 + tid; c < cend; c += LUR) {
      const T t = A[j + (long long)c * ld];
      A[j + (long long)c * ld] = A[p + (long long)c * ld];
      A[p + (long long)c * ld] = t;
    }
  }
  if (tid == 0) {
    ipiv[j] = p;
    if (sv[0] == R(0) && info) atomicCAS(info, 0, info_base + j + 1);
    *cnt = 0;  // ready for the next launch (kernel boundary orders it)
  }
}

// Net effect of the sequential LAPACK interchanges r <-> pv[r - i0] (r in [i0, i0 + k), pv[.] >= r):
// afterwards row dst[t] holds the former row src[t], t < return value (<= 2k moves).
// Content-parallel replay: every involved row's CONTENT (rows i0..i0+k-1 and each distinct
// pv[j] >= i0 + k) is tracked by its own thread through all k swaps -- k steps of a few VALU ops
// per content with the swap pair read as an LDS broadcast, instead of one lane chasing the swaps
// through LDS / global memory (a dependent-latency chain of ~k * 4 round trips).
// NT threads, CPT contents per thread (2k <= NT * CPT); pv is in LDS; wtot = NT/64 LDS ints.
template <int NT, int CPT>
__device__ int net_moves(const int* pv, int i0, int k, int* dst, int* src, int* wtot) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int start[CPT], pos[CPT];
  bool act[CPT];
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int c = u * NT + tid;
    start[u] = -1;
    act[u] = false;
    if (c < k) {
      start[u] = i0 + c;
      act[u] = true;
    } else if (c < 2 * k) {
      const int p = pv[c - k];
      if (p >= i0 + k) { start[u] = p; act[u] = true; }
    }
    pos[u] = start[u];
  }
  for (int i = 0; i < k; ++i) {
    const int p = pv[i], r = i0 + i;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      if (u * NT >= 2 * k) break;       // uniform: no contents left in this slot
      const int j = u * NT + tid - k;   // content index among the pivot rows (>= 0 for those)
      if (j > i && p == start[u]) act[u] = false;   // row p is already tracked by an earlier pivot
      pos[u] = pos[u] == r ? p : (pos[u] == p ? r : pos[u]);
    }
  }
  const unsigned long long below = (1ull << lane) - 1ull;
  int n = 0;
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    if (u * NT >= 2 * k) break;
    const bool mv = act[u] && pos[u] != start[u];
    const unsigned long long m = __ballot(mv);
    if (lane == 0) wtot[w] = __popcll(m);
    __syncthreads();
    int off = n, tot = 0;
#pragma unroll
    for (int v = 0; v < NT / 64; ++v) {
      const int x = wtot[v];
      off += v < w ? x : 0;
      tot += x;
    }
    if (mv) {
      const int t = off + __popcll(m & below);
      dst[t] = pos[u];
      src[t] = start[u];
    }
    n += tot;
    __syncthreads();
  }
  return n;
}

// An out-of-range pivot (a corrupt or stale ipiv entry) is never dereferenced: the launch that sees it
// moves nothing and reports DPL_INFO_BAD_PIVOT through info (over 0 or a positive singular-column index,
// never over another failure code) -- a silently skipped row would give a wrong factor with info 0.
#define DPL_INFO_BAD_PIVOT (-1001)
__device__ inline void report_bad_pivot(int* info) {
  if (!info) return;
  int old = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (old >= 0) {
    const int prev = atomicCAS(info, old, DPL_INFO_BAD_PIVOT);
    if (prev == old) break;
    old = prev;
  }
}

// Sequential interchanges (fallback for i1 - i0 > 512): one thread per column replays the swaps.
template <typename T>
__global__ __launch_bounds__(64) void k_laswp_seq(T* __restrict__ A, int ld, int m, int ca, int cb,
                                                  const int* __restrict__ ipiv, int i0, int i1, int* __restrict__ info) {
  // every pivot is validated (i <= ipiv[i] < m) before any column moves: one bad entry -> no moves at all
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int i = i0 + threadIdx.x; i < i1; i += 64) {
    const int p = ipiv[i];
    if (p < i || p >= m) bad = 1;
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0 && blockIdx.x == 0) report_bad_pivot(info);
    return;
  }
  const int c = ca + blockIdx.x * 64 + threadIdx.x;
  if (c >= cb) return;
  T* col = A + (long long)c * ld;
  for (int i = i0; i < i1; ++i) {
    const int p = ipiv[i];
    if (p != i) {
      const T t = col[i];
      col[i] = col[p];
      col[p] = t;
    }
  }
}

// Interchanges rows i <-> ipiv[i], i in [i0, i1) (i1 - i0 <= 512), on columns [ca, cb) of the
// panel: every workgroup derives the net moves in LDS (net_moves), then each wave moves its
// columns -- all reads of a column land in LDS before its writes (no chain through memory).
// Rows: [0, m); a pivot outside [i, m) stops the launch (report_bad_pivot).
#define LSW_COLS 16
template <typename T>
__global__ __launch_bounds__(512) void k_laswp_panel(T* __restrict__ A, int ld, int m, int ca, int cb,
                                                     const int* __restrict__ ipiv, int i0, int i1,
                                                     int* __restrict__ info) {
  __shared__ int pv[512], mdst[1024], msrc[1024], wtot[8];
  __shared__ T vals[4][1024];
  const int k = i1 - i0, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int badl = 0;
  for (int i = threadIdx.x; i < k; i += 512) {
    const int p = ipiv[i0 + i];
    pv[i] = p;
    badl |= (p < i0 + i || p >= m);
  }
  if (__syncthreads_or(badl)) {
    if (threadIdx.x == 0 && blockIdx.x == 0) report_bad_pivot(info);
    return;
  }
  const int n = net_moves<512, 2>(pv, i0, k, mdst, msrc, wtot);
  if (w >= 4) return;
  for (int cc = w; cc < LSW_COLS; cc += 4) {
    const int c = ca + blockIdx.x * LSW_COLS + cc;
    if (c >= cb) break;
    T* col = A + (long long)c * ld;
    for (int t = lane; t < n; t += 64) vals[w][t] = col[msrc[t]];
    for (int t = lane; t < n; t += 64) col[mdst[t]] = vals[w][t];
  }
}

// Net row moves of the sequential interchanges ipiv[0..kb) (panel-relative rows, kb <= 1024):
// row dst[t] holds the former row src[t]; cnt[0] = number of moved rows (<= 2 kb).  Pivots must lie in
// [i, mrel) (mrel: the rows below the panel's first one); otherwise cnt[0] = 0 (no moves) and info reports it.
__global__ __launch_bounds__(1024) void k_piv_moves(const int* __restrict__ ipiv, int kb, int mrel,
                                                    int* __restrict__ dst, int* __restrict__ src,
                                                    int* __restrict__ cnt, int* __restrict__ info) {
  __shared__ int pv[1024], wtot[16];
  int badl = 0;
  for (int i = threadIdx.x; i < kb; i += 1024) {
    const int p = ipiv[i];
    pv[i] = p;
    badl |= (p < i || p >= mrel);
  }
  if (__syncthreads_or(badl)) {
    if (threadIdx.x == 0) {
      cnt[0] = 0;
      report_bad_pivot(info);
    }
    return;
  }
  const int n = net_moves<1024, 2>(pv, 0, kb, dst, src, wtot);
  if (threadIdx.x == 0) cnt[0] = n;
}

// Row moves across local tile columns of a tiled matrix.  Global view row R = r0 + rel lives in
// view tile-row R / mb at local offset rowoff[R / mb] (+ R % mb); -1 = not on this rank.
// Column c of the flattened set: tile t = c / nb (coloff[t], ncols[t]), element c % nb.
// gather : buf[t_row * ldb + c] = A[src row] (0 if the row is not local)
// scatter: A[dst row] = buf[...] (only if the row is local)
template <typename T, bool GATHER>
__global__ __launch_bounds__(256) void k_rows_move(T* __restrict__ A, int ld, int mb, int r0,
                                                   const long long* __restrict__ rowoff, int nrt,
                                                   const long long* __restrict__ coloff, const int* __restrict__ ncols,
                                                   int nct, int nb, const int* __restrict__ rows,
                                                   const int* __restrict__ cnt, T* __restrict__ buf, int ldb,
                                                   int* __restrict__ info) {
  // lanes run along the move list (64 moves per wave): the staging buffer is column-major in t
  // and the moved rows are mostly runs of consecutive rows (the top kb rows), so both sides of
  // the copy coalesce; the 4 waves of a workgroup take different columns.
  const int n = cnt[0];
  const int t = blockIdx.y * 64 + (threadIdx.x & 63);
  if (blockIdx.y * 64 >= n) return;
  const bool tin = t < n;
  int R = 0, rt = 0;
  long long ro = -1;
  if (tin) {
    R = r0 + rows[t];
    rt = R / mb;
    // a row outside the view (a corrupt or stale pivot) is never dereferenced, and reported
    const bool inview = R >= 0 && rt < nrt;
    ro = inview ? rowoff[rt] : -1;
    if (!inview && blockIdx.x == 0) report_bad_pivot(info);
  }
  const long long rbase = ro + (R % mb);
  const int W = nct * nb;
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < W; c += gridDim.x * 4) {
    const int ct = c / nb, cc = c % nb;
    if (!tin || cc >= ncols[ct]) continue;
    const long long a = rbase + coloff[ct] + (long long)cc * ld;
    if (GATHER) {
      buf[(long long)c * ldb + t] = (ro >= 0) ? A[a] : ST<T>::zero();
    } else if (ro >= 0) {
      A[a] = buf[(long long)c * ldb + t];
    }
  }
}

// In-place row permutation on one process (P == 1): row r0 + dst[t] := former row r0 + src[t] over
// every local tile column, without the staging buffer of k_rows_move (no gather/scatter round trip
// through HBM, one launch).  Each wave owns whole columns: it reads all moved elements of its column
// into LDS before writing any of them (the moves form a permutation of the involved rows).
template <typename T>
__global__ __launch_bounds__(256) void k_rows_permute(T* __restrict__ A, int ld, int mb, int r0,
                                                      const long long* __restrict__ rowoff, int nrt,
                                                      const long long* __restrict__ coloff,
                                                      const int* __restrict__ ncols, int nct, int nb,
                                                      const int* __restrict__ dst, const int* __restrict__ src,
                                                      const int* __restrict__ cnt, int* __restrict__ info) {
  __shared__ long long so[1024], dof[1024];
  __shared__ T vals[4][1024];
  const int n = min(cnt[0], 1024);
  int badl = 0;
  for (int t = threadIdx.x; t < n; t += 256) {
    const int Rs = r0 + src[t], Rd = r0 + dst[t];
    const int ts = Rs / mb, td = Rd / mb;
    const long long bs = (Rs >= 0 && ts < nrt) ? rowoff[ts] : -1, bd = (Rd >= 0 && td < nrt) ? rowoff[td] : -1;
    const bool ok = bs >= 0 && bd >= 0;
    badl |= !ok;
    so[t] = ok ? bs + Rs % mb : -1;
    dof[t] = ok ? bd + Rd % mb : -1;
  }
  // one process: every moved row is local, so a missing one is a corrupt move list -- nothing moves
  if (__syncthreads_or(badl)) {
    if (threadIdx.x == 0 && blockIdx.x == 0) report_bad_pivot(info);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int W = nct * nb;
  for (int c = blockIdx.x * 4 + w; c < W; c += gridDim.x * 4) {
    const int ct = c / nb, cc = c % nb;
    if (cc >= ncols[ct]) continue;
    const long long co = coloff[ct] + (long long)cc * ld;
    for (int t = lane; t < n; t += 64)
      if (so[t] >= 0) vals[w][t] = A[so[t] + co];
    for (int t = lane; t < n; t += 64)
      if (dof[t] >= 0) A[dof[t] + co] = vals[w][t];
  }
}

// ---------------------------------------------------------------- persistent block LU
// Same block factorisation as k_lu_col, in ONE launch with the block's rows resident in LDS:
// G workgroups (<= one per CU), workgroup w owns panel rows [c0 + w R, c0 + (w+1) R) x the
// block's BW columns (R <= 256 rows, one per thread; R x BW x 8 B <= 128 KiB of LDS).
// Per column j, ONE grid barrier: before it every workgroup publishes its local |max| with
// that row's BW values (the candidate pivot row) and the owner of row j publishes row j;
// after it every workgroup reduces the G candidates (same answer everywhere), takes the winner
// as the new row j and the owner of the pivot row takes the old row j -- the interchange needs
// no second hand-off.  Barrier: monotonic agent-scope counter (release fence -> arrive ->
// relaxed poll with s_sleep -> acquire fence; MI355X_MICROARCH.md barrier-counter), published
// data double-buffered by column parity.  Rank-1 updates run on the LDS copy.
#define PLR 256
#define PBW 64
// wave-level argmax (|v| desc, row asc) with DPP-free shuffles, then across the 4 waves in LDS
__device__ inline void wave_argmax(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
}

// Pivot of one column across the G workgroups: every workgroup has published its local winner (v at
// pval[par G + w], row at pidx[par G + w]) and its candidate row; returns the global winner (largest
// magnitude, lowest row on ties) in every thread.
//  HIER (default): XCD-sharded fan-in -- workgroup w arrives on the counter of group w % 8 (the hardware
//    dispatches blockIdx round-robin over the 8 XCDs, so a group is an XCD; correctness never depends on it),
//    the group's LAST arriver (told by the value its add returned) reduces the group's candidates, publishes
//    the group winner and arrives on the top counter; every workgroup polls the top counter and reduces <= 8
//    group winners.  ~32 + 8 serialised atomics and 8 candidate loads per workgroup instead of 256 + 256
//    (MI355X_MICROARCH.md barrier-counter 7.4 us vs barrier-xcd 4.1 us at 256 workgroups).
//  flat: one counter, every workgroup reduces all G candidates (the former path; dpl_lu_block_set_kind(2)).
// ctr: 9 counters, 32 ints apart (zeroed before the launch); gval / gidx: [2][8] group winners.
// sv / si: >= 13 LDS slots.  Everything crossing workgroups is an sc1 store drained before the arrival and
// an sc1 load after the poll (grid_sync.h).
template <bool HIER>
__device__ inline void lu_pick(double v, int vi, int par, int cj, int G, int w, double* pval, int* pidx, int* ctr,
                               double* gval, int* gidx, int* info, double* sv, int* si, double& best, int& bi) {
  const int tid = threadIdx.x;
  if (!HIER) {
    grid_sync_counter(ctr, (cj + 1) * G, info);
    best = -1.0;
    bi = 0x7fffffff;
    for (int b = tid; b < G; b += PLR) {
      const double pv_ = ld_sc1(&pval[par * G + b]);
      const int pi_ = ld_sc1(&pidx[par * G + b]);
      if (pv_ > best || (pv_ == best && pi_ < bi)) { best = pv_; bi = pi_; }
    }
    wave_argmax(best, bi);
    if ((tid & 63) == 0) { sv[8 + (tid >> 6)] = best; si[8 + (tid >> 6)] = bi; }
    __syncthreads();
    best = sv[8];
    bi = si[8];
#pragma unroll
    for (int q = 1; q < PLR / 64; ++q)
      if (sv[8 + q] > best || (sv[8 + q] == best && si[8 + q] < bi)) { best = sv[8 + q]; bi = si[8 + q]; }
    return;
  }
  (void)v;
  (void)vi;
  const int ng = G < 8 ? G : 8;
  const int x = w % ng;
  const int gx = (G - x + ng - 1) / ng;        // workgroups of group x: x, x + ng, ...
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(&ctr[32 * x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    si[12] = (old + 1 == (cj + 1) * gx);
  }
  __syncthreads();
  if (si[12]) {                                 // uniform: the group's last arriver reduces it
    double gv = -1.0;
    int gi = 0x7fffffff;
    for (int t = tid; t < gx; t += PLR) {
      const int b = x + t * ng;
      const double pv_ = ld_sc1(&pval[par * G + b]);
      const int pi_ = ld_sc1(&pidx[par * G + b]);
      if (pv_ > gv || (pv_ == gv && pi_ < gi)) { gv = pv_; gi = pi_; }
    }
    wave_argmax(gv, gi);
    if ((tid & 63) == 0) { sv[8 + (tid >> 6)] = gv; si[8 + (tid >> 6)] = gi; }
    __syncthreads();
    if (tid == 0) {
      gv = sv[8];
      gi = si[8];
#pragma unroll
      for (int q = 1; q < PLR / 64; ++q)
        if (sv[8 + q] > gv || (sv[8 + q] == gv && si[8 + q] < gi)) { gv = sv[8 + q]; gi = si[8 + q]; }
      st_sc1(&gval[par * 8 + x], gv);
      st_sc1(&gidx[par * 8 + x], gi);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&ctr[32 * 8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0) {
    const int target = (cj + 1) * ng;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&ctr[32 * 8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ULL) {  // 100 MHz clock: 2 s (grid not co-resident)
        if (info) atomicExch(info, -1000);
        break;
      }
    }
  }
  __syncthreads();
  if (tid < 64) {
    best = tid < ng ? ld_sc1(&gval[par * 8 + tid]) : -1.0;
    bi = tid < ng ? ld_sc1(&gidx[par * 8 + tid]) : 0x7fffffff;
    wave_argmax(best, bi);
    if (tid == 0) { sv[12] = best; si[13] = bi; }
  }
  __syncthreads();
  best = sv[12];
  bi = si[13];
}

// BWT: the widest block this instantiation holds (64: 128 KiB LDS tile for fp64; 32: 64 KiB, which leaves
// room on the CU for one trailing-update GEMM workgroup -- DPLASMA_LU_BW=32, the recursion's base width)
template <typename T, int BWT, bool HIER>
__global__ __launch_bounds__(PLR) void k_lu_block_persist(T* __restrict__ A, int ld, int m, int c0, int cend, int R,
                                                          int* __restrict__ ipiv, T* __restrict__ cand,
                                                          double* __restrict__ pval, int* __restrict__ pidx,
                                                          int* __restrict__ cnt, double* __restrict__ gval,
                                                          int* __restrict__ gidx, int* __restrict__ info,
                                                          int info_base) {
  __shared__ T tile[BWT * PLR];      // column-major: tile[c * R + r]
  __shared__ T prow[PBW], oldj[PBW];
  __shared__ double sv[PLR];
  __shared__ int si[PLR];
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
  // the panel is the critical path: its waves win VALU issue over a co-resident trailing-update GEMM wave
  // (a 32-column block leaves room on a CU for one GEMM workgroup beside it; MI355X_MICROARCH.md, wave priority)
  __builtin_amdgcn_s_setprio(3);
  const int BW = cend - c0;
  const int rbase = c0 + w * R;
  const int nr = max(0, min(R, m - rbase));   // rows owned
  // ---- load the block rows
  for (int e = tid; e < BW * R; e += PLR) {
    const int c = e / R, r = e % R;
    if (r < nr) tile[c * R + r] = A[(rbase + r) + (long long)(c0 + c) * ld];
  }
  __syncthreads();
  const int r = tid, g = rbase + tid;
  const bool own = r < nr;
  for (int cj = 0; cj < BW; ++cj) {
    const int j = c0 + cj;
    const int par = cj & 1;
    // ---- 1. apply column cj-1 (pivot row in prow); each thread touches only its own row, so the local
    //         pivot search below needs no barrier after it
    if (cj > 0 && own && g >= j) {
      const T d = prow[cj - 1];
      T l = tile[(cj - 1) * R + r];
      if (!is_zero(d)) l = divv(l, d);
      tile[(cj - 1) * R + r] = l;
      for (int c = cj; c < BW; ++c) tile[c * R + r] = sub(tile[c * R + r], mul(l, prow[c]));
    }
    // ---- 2. local |max| of column cj over rows >= j; publish it with its row, and row j.  The four waves'
    //         winners meet in LDS and every thread reduces them itself (one barrier, no second round).
    double v = (own && g >= j) ? piv_mag((double)abs1(tile[cj * R + r])) : -1.0;
    int vi = (own && g >= j) ? g : 0x7fffffff;
    wave_argmax(v, vi);
    if ((tid & 63) == 0) { sv[(tid >> 6) + 4 * par] = v; si[(tid >> 6) + 4 * par] = vi; }
    __syncthreads();
    v = sv[4 * par];
    vi = si[4 * par];
#pragma unroll
    for (int q = 1; q < PLR / 64; ++q) {
      const double v2 = sv[q + 4 * par];
      const int i2 = si[q + 4 * par];
      if (v2 > v || (v2 == v && i2 < vi)) { v = v2; vi = i2; }
    }
    const int lw = vi;
    if (tid == 0) {
      st_sc1(&pval[par * G + w], v);
      st_sc1(&pidx[par * G + w], lw);
    }
    if (lw != 0x7fffffff && tid < BW) st_sc1(&cand[((long long)par * G + w) * PBW + tid], tile[tid * R + (lw - rbase)]);
    if (j >= rbase && j < rbase + nr && tid < BW)
      st_sc1(&cand[((long long)2 * G + par) * PBW + tid], tile[tid * R + (j - rbase)]);
    // ---- 3. global pivot (the winning workgroup travels with the row index: row -> owner is rbase
    //         arithmetic; LDS slots 8..13 are the exchange's, 0..7 hold this and the previous column's search)
    {
      double best;
      int bi;
      lu_pick<HIER>(v, lw, par, cj, G, w, pval, pidx, cnt, gval, gidx, info, sv, si, best, bi);
      const int p = bi, pw = (p - c0) / R;
      if (tid < BW) {
        prow[tid] = ld_sc1(&cand[((long long)par * G + pw) * PBW + tid]);
        oldj[tid] = ld_sc1(&cand[((long long)2 * G + par) * PBW + tid]);
      }
      __syncthreads();
      // interchange rows j <-> p on the LDS copies
      if (tid < BW) {
        if (j >= rbase && j < rbase + nr) tile[tid * R + (j - rbase)] = prow[tid];
        if (p != j && p >= rbase && p < rbase + nr) tile[tid * R + (p - rbase)] = oldj[tid];
      }
      if (w == 0 && tid == 0) {
        ipiv[j] = p;
        if (best == 0.0 && info) atomicCAS(info, 0, info_base + j + 1);
      }
      __syncthreads();
    }
  }
  // ---- last column: scale below the diagonal
  if (own && g >= cend) {
    const T d = prow[BW - 1];
    T l = tile[(BW - 1) * R + r];
    if (!is_zero(d)) l = divv(l, d);
    tile[(BW - 1) * R + r] = l;
  }
  __syncthreads();
  for (int e = tid; e < BW * R; e += PLR) {
    const int c = e / R, rr = e % R;
    if (rr < nr) A[(rbase + rr) + (long long)(c0 + c) * ld] = tile[c * R + rr];
  }
}

// ---------------------------------------------------------------- tagged-granule block LU (default)
// k_lu_block_persist with the pivot exchange done through self-validating granules instead of a counter:
// every value that crosses workgroups travels as one 8-byte {32-bit payload, 32-bit tag} word written by ONE
// sc1 store, tag = launch epoch << 7 | (column + 1).  A reader polls the words themselves until every tag
// matches -- no drain before an arrival, no counter round trip, no poll on a separate flag (MI355X_MICROARCH.md
// handoff-1to1 ~0.8-1 us vs barrier-counter 7.4 us): one column costs the local search, one record read
// (value hi / lo, row) of every workgroup, and one read of the winning row and the old row j.
// Records, candidate rows and row j are double-buffered by column parity: a workgroup publishes column cj + 2
// only after it has read every workgroup's column cj + 1, which each of them published after reading cj.
// Layout (8-byte words): rec[2][G][4] = {value hi, value lo, row}, rows[2][G][PBW * NW], jrow[2][PBW * NW]
// (NW = 32-bit words per element).
template <typename T, int BWT>
__global__ __launch_bounds__(PLR) void k_lu_block_tag(T* __restrict__ A, int ld, int m, int c0, int cend, int R,
                                                      int* __restrict__ ipiv, unsigned long long* __restrict__ rec,
                                                      unsigned long long* __restrict__ rows,
                                                      unsigned long long* __restrict__ jrow, unsigned tag0,
                                                      int* __restrict__ info, int info_base) {
  constexpr int NW = sizeof(T) / 4;
  __shared__ T tile[BWT * PLR];      // column-major: tile[c * R + r]
  __shared__ T prow[PBW], oldj[PBW];
  __shared__ double sv[16];
  __shared__ int si[16];
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
  __builtin_amdgcn_s_setprio(3);
  const int BW = cend - c0;
  const int rbase = c0 + w * R;
  const int nr = max(0, min(R, m - rbase));
  for (int e = tid; e < BW * R; e += PLR) {
    const int c = e / R, r = e % R;
    if (r < nr) tile[c * R + r] = A[(rbase + r) + (long long)(c0 + c) * ld];
  }
  __syncthreads();
  const int r = tid, g = rbase + tid;
  const bool own = r < nr;
  for (int cj = 0; cj < BW; ++cj) {
    const int j = c0 + cj;
    const int par = cj & 1;
    const unsigned tag = tag0 | (unsigned)(cj + 1);
    // ---- 1. apply column cj-1 (pivot row in prow) to column cj only: the search needs nothing more, and the
    //         rest of the rank-1 update (3b) runs while the record travels
    const bool upd = cj > 0 && own && g >= j;
    T l = ST<T>::zero();
    if (upd) {
      const T d = prow[cj - 1];
      l = tile[(cj - 1) * R + r];
      if (!is_zero(d)) l = divv(l, d);
      tile[(cj - 1) * R + r] = l;
      tile[cj * R + r] = sub(tile[cj * R + r], mul(l, prow[cj]));
    }
    // ---- 2. local |max| of column cj over rows >= j
    double v = (own && g >= j) ? piv_mag((double)abs1(tile[cj * R + r])) : -1.0;
    int vi = (own && g >= j) ? g : 0x7fffffff;
    wave_argmax(v, vi);
    if ((tid & 63) == 0) { sv[(tid >> 6) + 4 * par] = v; si[(tid >> 6) + 4 * par] = vi; }
    __syncthreads();
    v = sv[4 * par];
    vi = si[4 * par];
#pragma unroll
    for (int q = 1; q < PLR / 64; ++q) {
      const double v2 = sv[q + 4 * par];
      const int i2 = si[q + 4 * par];
      if (v2 > v || (v2 == v && i2 < vi)) { v = v2; vi = i2; }
    }
    // ---- publish: record, candidate row, and row j by its owner (tagged words, no drain, no counter)
    if (tid == 0) {
      const unsigned long long vb = (unsigned long long)__double_as_longlong(v);
      unsigned long long* rc = rec + ((long long)par * G + w) * 4;
      st_sc1(&rc[0], ((vb >> 32) << 32) | tag);
      st_sc1(&rc[1], (vb << 32) | tag);
      st_sc1(&rc[2], ((unsigned long long)(unsigned)vi << 32) | tag);
    }
    // ---- 3b. the rest of column cj-1's rank-1 update (own row only), then the rows are complete
    if (upd)
      for (int c = cj + 1; c < BW; ++c) tile[c * R + r] = sub(tile[c * R + r], mul(l, prow[c]));
    __syncthreads();
    // candidate row by threads [0, 64), row j by threads [64, 128): one element (NW words) per thread
    if (tid < BW && vi != 0x7fffffff)
      tag_put<T>(&rows[((long long)par * G + w) * (PBW * NW) + tid * NW], tile[tid * R + (vi - rbase)], tag);
    if (tid >= 64 && tid - 64 < BW && j >= rbase && j < rbase + nr)
      tag_put<T>(&jrow[(long long)par * (PBW * NW) + (tid - 64) * NW], tile[(tid - 64) * R + (j - rbase)], tag);
    // ---- 3. every workgroup's record -> global pivot (same answer everywhere)
    double best = -1.0;
    int bi = 0x7fffffff;
    for (int b = tid; b < G; b += PLR) {
      const unsigned long long* rc = rec + ((long long)par * G + b) * 4;
      // the three words issued together; only a stale one is polled again
      unsigned long long x0 = ld_sc1(&rc[0]), x1 = ld_sc1(&rc[1]), x2 = ld_sc1(&rc[2]);
      if ((unsigned)x0 != tag) tag_poll(&rc[0], tag, x0, info);
      if ((unsigned)x1 != tag) tag_poll(&rc[1], tag, x1, info);
      if ((unsigned)x2 != tag) tag_poll(&rc[2], tag, x2, info);
      const double pv_ = __longlong_as_double((long long)(((x0 >> 32) << 32) | (x1 >> 32)));
      const int pi_ = (int)(unsigned)(x2 >> 32);
      if (pv_ > best || (pv_ == best && pi_ < bi)) { best = pv_; bi = pi_; }
    }
    wave_argmax(best, bi);
    if ((tid & 63) == 0) { sv[8 + (tid >> 6)] = best; si[8 + (tid >> 6)] = bi; }
    __syncthreads();
    best = sv[8];
    bi = si[8];
#pragma unroll
    for (int q = 1; q < PLR / 64; ++q)
      if (sv[8 + q] > best || (sv[8 + q] == best && si[8 + q] < bi)) { best = sv[8 + q]; bi = si[8 + q]; }
    const bool any = bi != 0x7fffffff;           // no eligible row (j >= m): nothing to pivot
    const int p = bi, pw = any ? (p - c0) / R : 0;
    // ---- 4. the winning row (threads [0, 64)) and the old row j (threads [64, 128))
    if (any && tid < BW) prow[tid] = tag_get<T>(&rows[((long long)par * G + pw) * (PBW * NW) + tid * NW], tag, info);
    if (j < m && tid >= 64 && tid - 64 < BW)
      oldj[tid - 64] = tag_get<T>(&jrow[(long long)par * (PBW * NW) + (tid - 64) * NW], tag, info);
    __syncthreads();
    if (any && tid < BW) {
      if (j >= rbase && j < rbase + nr) tile[tid * R + (j - rbase)] = prow[tid];
      if (p != j && p >= rbase && p < rbase + nr) tile[tid * R + (p - rbase)] = oldj[tid];
    }
    if (w == 0 && tid == 0 && any) {
      ipiv[j] = p;
      if (best == 0.0 && info) atomicCAS(info, 0, info_base + j + 1);
    }
    __syncthreads();
  }
  if (own && g >= cend) {
    const T d = prow[BW - 1];
    T l = tile[(BW - 1) * R + r];
    if (!is_zero(d)) l = divv(l, d);
    tile[(BW - 1) * R + r] = l;
  }
  __syncthreads();
  for (int e = tid; e < BW * R; e += PLR) {
    const int c = e / R, rr = e % R;
    if (rr < nr) A[(rbase + rr) + (long long)(c0 + c) * ld] = tile[c * R + rr];
  }
}

// ---------------------------------------------------------------- register-resident block LU
// Same algorithm and hand-offs as k_lu_block_persist, but every thread keeps ITS ROW of the block in
// registers (v[c], c < 64, the column loop fully unrolled so every index is static) instead of a
// 128 KiB LDS tile.  A workgroup then needs ~2 KiB of LDS and <= 256 VGPRs per lane, so it can share
// a CU with a trailing-update GEMM workgroup (72 KiB LDS, 256 VGPRs): with look-ahead the panel no
// longer waits for whole CUs to drain of GEMM waves before its grid barrier can complete.
template <typename T>
__global__ __launch_bounds__(PLR) void k_lu_block_reg(T* __restrict__ A, int ld, int m, int c0, int cend, int R,
                                                      int* __restrict__ ipiv, T* __restrict__ cand,
                                                      double* __restrict__ pval, int* __restrict__ pidx,
                                                      int* __restrict__ cnt, double* __restrict__ gval,
                                                      int* __restrict__ gidx, int* __restrict__ info, int info_base) {
  __shared__ T prow[PBW], oldj[PBW];
  __shared__ double sv[16];
  __shared__ int si[16];
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
  const int BW = cend - c0;
  const int rbase = c0 + w * R;
  const int nr = max(0, min(R, m - rbase));
  const int g = rbase + tid;
  const bool own = tid < nr;
  T v[PBW];
#pragma unroll
  for (int c = 0; c < PBW; ++c) v[c] = (own && c < BW) ? A[g + (long long)(c0 + c) * ld] : ST<T>::zero();
#pragma clang loop unroll(full)
  for (int cj = 0; cj < PBW; ++cj) {
    if (cj < BW) {   // uniform; no break, so the loop unrolls and every v[] index is static
    const int j = c0 + cj;
    const int par = cj & 1;
    // ---- 1. apply column cj-1 (pivot row in prow)
    if (cj > 0 && own && g >= j) {
      const T d = prow[cj - 1];
      T l = v[cj - 1];
      if (!is_zero(d)) l = divv(l, d);
      v[cj - 1] = l;
#pragma unroll
      for (int c = cj; c < PBW; ++c)
        if (c < BW) v[c] = sub(v[c], mul(l, prow[c]));
    }
    // ---- 2. workgroup |max| of column cj over rows >= j
    double val = (own && g >= j) ? piv_mag((double)abs1(v[cj])) : -1.0;
    int vi = (own && g >= j) ? g : 0x7fffffff;
    wave_argmax(val, vi);
    if ((tid & 63) == 0) { sv[tid >> 6] = val; si[tid >> 6] = vi; }
    __syncthreads();
    double bv = sv[0];
    int bi = si[0];
#pragma unroll
    for (int q = 1; q < PLR / 64; ++q)
      if (sv[q] > bv || (sv[q] == bv && si[q] < bi)) { bv = sv[q]; bi = si[q]; }
    if (tid == 0) {
      st_sc1(&pval[par * G + w], bv);
      st_sc1(&pidx[par * G + w], bi);
    }
    if (own && g == bi) {
#pragma unroll
      for (int c = 0; c < PBW; ++c)
        if (c < BW) st_sc1(&cand[((long long)par * G + w) * PBW + c], v[c]);
    }
    if (own && g == j) {
#pragma unroll
      for (int c = 0; c < PBW; ++c)
        if (c < BW) st_sc1(&cand[((long long)2 * G + par) * PBW + c], v[c]);
    }
    // ---- 3. global pivot
    double best;
    int bix;
    lu_pick<true>(bv, bi, par, cj, G, w, pval, pidx, cnt, gval, gidx, info, sv, si, best, bix);
    const int p = bix, pw = (p - c0) / R;
    if (tid < BW) {
      prow[tid] = ld_sc1(&cand[((long long)par * G + pw) * PBW + tid]);
      oldj[tid] = ld_sc1(&cand[((long long)2 * G + par) * PBW + tid]);
    }
    __syncthreads();
    if (own && g == j) {
#pragma unroll
      for (int c = 0; c < PBW; ++c) v[c] = prow[c];
    } else if (own && g == p) {
#pragma unroll
      for (int c = 0; c < PBW; ++c) v[c] = oldj[c];
    }
    if (w == 0 && tid == 0) {
      ipiv[j] = p;
      if (best == 0.0 && info) atomicCAS(info, 0, info_base + j + 1);
    }
    }
  }
  // ---- last column: scale below the diagonal, then the rows go home
  if (own && g >= cend) {
    const T d = prow[BW - 1];
#pragma unroll
    for (int c = 0; c < PBW; ++c)
      if (c == BW - 1 && !is_zero(d)) v[c] = divv(v[c], d);
  }
#pragma unroll
  for (int c = 0; c < PBW; ++c)
    if (own && c < BW) A[g + (long long)(c0 + c) * ld] = v[c];
}

// block kernel choice for the pivoting persistent path: 0 = LDS tile, tagged-granule exchange (default),
// 1 = register-resident rows, 2 = LDS tile with the flat one-counter exchange (the former default), 3 = LDS tile
// with the XCD-sharded counter exchange (profiles/r5_lu_pivot_exchange.txt).
// Measured on one MI355X (profiles/r3_lu_block_reg.txt): the register variant is 30 % slower per column
// (64 fully unrolled column steps: ~100 KiB of code per launch, instruction-cache bound) and look-ahead
// does not recover it -- kept opt-in (DPLASMA_LU_BLOCK=reg) as the measured alternative.
static int g_lu_kind = 0;
DPL_API int dpl_lu_block_set_kind(int k) {
  const int old = g_lu_kind;
  g_lu_kind = k;
  return old;
}

#define DISPATCH(prec, CALL)                                          \
  switch (prec) {                                                     \
    case DPL_S: { typedef float T; CALL; } break;                     \
    case DPL_D: { typedef double T; CALL; } break;                    \
    case DPL_C: { typedef hipFloatComplex T; CALL; } break;           \
    case DPL_Z: { typedef hipDoubleComplex T; CALL; } break;          \
    default: return -2;                                               \
  }

// Factor block columns [c0, cend) of the panel A (m rows, ld) with partial pivoting (or none):
// cend - c0 + 1 launches of k_lu_col.  ws: >= 2*ceil(m/256) 8-byte words + 1 int counter
// (zero on first use; each launch leaves it zero).
static int g_num_cus = 0;

// ws layout (bytes): [0, 8*2*G) pval, then 4*2*G pidx, then 8-aligned candidate rows
// (3 * G * PBW * sizeof(T) <= 3 * 256 * 64 * 16 B); callers size it with dpl_lu_block_ws_bytes.
// + the tagged-exchange area (k_lu_block_tag) at LU_TAG_OFF: rec 2 x 256 x 32 B, rows 2 x 256 x PBW x 2 x 8 B,
// jrow 2 x PBW x 2 x 8 B.
#define LU_TAG_OFF (1LL << 20)
DPL_API long long dpl_lu_block_ws_bytes(int m) {
  const int maxwg = (m + LUR - 1) / LUR;
  long long a = 16LL * (maxwg > 256 ? maxwg : 256) + 64;
  a += 3LL * 256 * PBW * 16 + 64;
  const long long tag_end = LU_TAG_OFF + 2LL * 256 * 32 + 2LL * 256 * PBW * 2 * 8 + 2LL * PBW * 2 * 8;
  return a > tag_end ? a : tag_end;
}

// ------------------------------------------------------------------ no-pivot block LU
// Columns [c0, cend) (<= 64), rows [c0, m) of P, without pivoting (CORE_zgetrf_nopiv's role): the
// bw x bw top block is tiny, so every workgroup factors it redundantly in LDS (bw dependent steps on
// 256 threads) and then solves its own 256 rows as L21 = A21 U11^-1 by forward substitution, one
// row per thread -- no grid-wide synchronisation at all (the pivoting path needs one grid barrier per
// column for the pivot search; without pivots the rows are independent given U11).
constexpr int NPB = 64;
template <typename T>
__global__ __launch_bounds__(256) void k_lu_nopiv_block(T* __restrict__ A, int ld, int m, int c0, int cend,
                                                        int* __restrict__ info, int info_base) {
  __shared__ T U[NPB][NPB + 1];
  const int tid = threadIdx.x;
  const int bw = cend - c0;
  const int top = min(bw, m - c0);
  for (int e = tid; e < top * bw; e += 256) {
    const int r = e % top, c = e / top;
    U[r][c] = A[(long long)(c0 + r) + (long long)(c0 + c) * ld];
  }
  __syncthreads();
  int bad = 0;
  for (int j = 0; j < top; ++j) {
    const T d = U[j][j];
    if (is_zero(d)) {
      if (!bad) bad = j + 1;
      __syncthreads();
      continue;
    }
    for (int e = tid; e < (top - j - 1) * (bw - j); e += 256) {
      const int r = j + 1 + e % (top - j - 1), c = j + e / (top - j - 1);
      if (c == j) U[r][j] = divv(U[r][j], d);
    }
    __syncthreads();
    for (int e = tid; e < (top - j - 1) * (bw - j - 1); e += 256) {
      const int r = j + 1 + e % (top - j - 1), c = j + 1 + e / (top - j - 1);
      U[r][c] = sub(U[r][c], mul(U[r][j], U[j][c]));
    }
    __syncthreads();
  }
  if (blockIdx.x == 0) {
    for (int e = tid; e < top * bw; e += 256) {
      const int r = e % top, c = e / top;
      A[(long long)(c0 + r) + (long long)(c0 + c) * ld] = U[r][c];
    }
    if (tid == 0 && bad && info && *info == 0) *info = info_base + c0 + bad;
  }
  // rows below the top block: x := x U11^-1
  const int r = c0 + top + blockIdx.x * 256 + tid;
  if (r >= m) return;
  T x[NPB];
#pragma unroll
  for (int c = 0; c < NPB; ++c) x[c] = (c < bw) ? A[(long long)r + (long long)(c0 + c) * ld] : ST<T>::zero();
#pragma unroll
  for (int c = 0; c < NPB; ++c) {
    if (c < bw) {
      T v = x[c];
#pragma unroll
      for (int i = 0; i < c; ++i) v = sub(v, mul(x[i], U[i][c]));
      x[c] = (c < top && !is_zero(U[c][c])) ? divv(v, U[c][c]) : v;
    }
  }
#pragma unroll
  for (int c = 0; c < NPB; ++c)
    if (c < bw) A[(long long)r + (long long)(c0 + c) * ld] = x[c];
}

DPL_API int dpl_lu_block(int prec, void* A, int ld, int m, int c0, int cend, int* ipiv, void* ws, int* cnt,
                         int* info, int info_base, int pivot, hipStream_t st) {
  if (cend - c0 > LU_MAXBW || c0 >= cend || m <= c0) return cend <= c0 ? 0 : -3;
  // persistent single-launch path: real precisions, rows fit one per thread in <= #CU workgroups
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_num_cus <= 0) g_num_cus = 1;
  }
  const int rows = m - c0;
  const int gmax = g_num_cus < 256 ? g_num_cus : 256;
  if (pivot && (prec == DPL_D || prec == DPL_S) && rows <= gmax * PLR && cend - c0 <= PBW) {
    int G = (rows + 255) / 256;                 // ~256 rows per workgroup: fewest barrier arrivals
    if (G > gmax) G = gmax;
    if (G < 1) G = 1;
    const int R = (rows + G - 1) / G;
    if (R <= PLR) {
      char* b = (char*)ws;
      double* pval = (double*)b;
      int* pidx = (int*)(b + 8LL * 2 * 256);
      void* cand = (void*)(b + 8LL * 2 * 256 + 4LL * 2 * 256 + 64);
      // exchange counters (9 x 128 B) and group winners behind the candidate rows (real types: 8-B elements)
      char* xb = b + ((8LL * 2 * 256 + 4LL * 2 * 256 + 64 + 3LL * 256 * PBW * 8 + 127) & ~127LL);
      int* ctr = (int*)xb;
      double* gval = (double*)(xb + 9 * 128);
      int* gidx = (int*)(xb + 9 * 128 + 8 * 16);
      if (g_lu_kind == 0) {
        static unsigned epoch = 0;
        epoch = (epoch + 1) & 0x1ffffffu;
        const unsigned tag0 = epoch << 7;
        unsigned long long* rec = (unsigned long long*)(b + LU_TAG_OFF);
        unsigned long long* rws = rec + 2 * 256 * 4;
        unsigned long long* jrw = rws + 2LL * 256 * PBW * 2;
#define LUT_ARGS(T) (T*)A, ld, m, c0, cend, R, ipiv, rec, rws, jrw, tag0, info, info_base
        if (cend - c0 <= 32) {
          if (prec == DPL_D) hipLaunchKernelGGL((k_lu_block_tag<double, 32>), dim3(G), dim3(PLR), 0, st, LUT_ARGS(double));
          else hipLaunchKernelGGL((k_lu_block_tag<float, 32>), dim3(G), dim3(PLR), 0, st, LUT_ARGS(float));
        } else if (prec == DPL_D) {
          hipLaunchKernelGGL((k_lu_block_tag<double, 64>), dim3(G), dim3(PLR), 0, st, LUT_ARGS(double));
        } else {
          hipLaunchKernelGGL((k_lu_block_tag<float, 64>), dim3(G), dim3(PLR), 0, st, LUT_ARGS(float));
        }
#undef LUT_ARGS
        return (int)hipGetLastError();
      }
      const bool flat = g_lu_kind == 2;
      if (flat) ctr = cnt;
      (void)hipMemsetAsync(ctr, 0, flat ? sizeof(int) : 9 * 128, st);
#define LUB_ARGS(T) (T*)A, ld, m, c0, cend, R, ipiv, (T*)cand, pval, pidx, ctr, gval, gidx, info, info_base
      if (g_lu_kind == 1) {
        if (prec == DPL_D)
          hipLaunchKernelGGL((k_lu_block_reg<double>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(double));
        else
          hipLaunchKernelGGL((k_lu_block_reg<float>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(float));
      } else if (cend - c0 <= 32) {
        if (prec == DPL_D) {
          if (flat) hipLaunchKernelGGL((k_lu_block_persist<double, 32, false>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(double));
          else hipLaunchKernelGGL((k_lu_block_persist<double, 32, true>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(double));
        } else {
          if (flat) hipLaunchKernelGGL((k_lu_block_persist<float, 32, false>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(float));
          else hipLaunchKernelGGL((k_lu_block_persist<float, 32, true>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(float));
        }
      } else if (prec == DPL_D) {
        if (flat) hipLaunchKernelGGL((k_lu_block_persist<double, 64, false>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(double));
        else hipLaunchKernelGGL((k_lu_block_persist<double, 64, true>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(double));
      } else {
        if (flat) hipLaunchKernelGGL((k_lu_block_persist<float, 64, false>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(float));
        else hipLaunchKernelGGL((k_lu_block_persist<float, 64, true>), dim3(G), dim3(PLR), 0, st, LUB_ARGS(float));
      }
#undef LUB_ARGS
      return (int)hipGetLastError();
    }
  }
  if (!pivot && cend - c0 <= NPB) {
    const int rows_below = m - c0 - ((cend - c0) < (m - c0) ? (cend - c0) : (m - c0));
    const int G = rows_below > 0 ? (rows_below + 255) / 256 : 1;
    DISPATCH(prec, hipLaunchKernelGGL((k_lu_nopiv_block<T>), dim3(G), dim3(256), 0, st, (T*)A, ld, m, c0, cend, info,
                                      info_base));
    return (int)hipGetLastError();
  }
  const int maxwg = (m + LUR - 1) / LUR;
  for (int j = c0; j <= cend; ++j) {
    const int rows = m - j;
    if (rows <= 0) break;
    const int nwg = (rows + LUR - 1) / LUR;
    DISPATCH(prec, {
      typedef typename ST<T>::real R;
      hipLaunchKernelGGL((k_lu_col<T>), dim3(nwg), dim3(LUR), 0, st, (T*)A, ld, m, c0, cend, j, ipiv, (R*)ws,
                         (int*)((R*)ws + maxwg), cnt, info, info_base, pivot);
    });
  }
  return (int)hipGetLastError();
}

DPL_API int dpl_laswp_panel(int prec, void* A, int ld, int m, int ca, int cb, const int* ipiv, int i0, int i1,
                            int* info, hipStream_t st) {
  if (cb <= ca || i1 <= i0) return 0;
  if (i1 - i0 > 512) {
    DISPATCH(prec, hipLaunchKernelGGL((k_laswp_seq<T>), dim3((cb - ca + 63) / 64), dim3(64), 0, st, (T*)A, ld, m, ca,
                                      cb, ipiv, i0, i1, info));
    return (int)hipGetLastError();
  }
  DISPATCH(prec, hipLaunchKernelGGL((k_laswp_panel<T>), dim3((cb - ca + LSW_COLS - 1) / LSW_COLS), dim3(512), 0, st,
                                    (T*)A, ld, m, ca, cb, ipiv, i0, i1, info));
  return (int)hipGetLastError();
}

DPL_API int dpl_piv_moves(const int* ipiv, int kb, int mrel, int* dst, int* src, int* cnt, int* info, hipStream_t st) {
  if (kb > 1024) return -3;
  hipLaunchKernelGGL(k_piv_moves, dim3(1), dim3(1024), 0, st, ipiv, kb, mrel, dst, src, cnt, info);
  return (int)hipGetLastError();
}

DPL_API int dpl_rows_move(int prec, int gather, void* A, int ld, int mb, int r0, const long long* rowoff, int nrt,
                          const long long* coloff, const int* ncols, int nct, int nb, const int* rows,
                          const int* cnt, int maxcnt, void* buf, int ldb, int* info, hipStream_t st) {
  if (nct <= 0 || maxcnt <= 0) return 0;
  const int W = nct * nb;
  const int gx = (W + 3) / 4 > 2048 ? 2048 : (W + 3) / 4;
  dim3 g(gx, (maxcnt + 63) / 64);
  if (gather) {
    DISPATCH(prec, hipLaunchKernelGGL((k_rows_move<T, true>), g, dim3(256), 0, st, (T*)A, ld, mb, r0, rowoff, nrt,
                                      coloff, ncols, nct, nb, rows, cnt, (T*)buf, ldb, info));
  } else {
    DISPATCH(prec, hipLaunchKernelGGL((k_rows_move<T, false>), g, dim3(256), 0, st, (T*)A, ld, mb, r0, rowoff, nrt,
                                      coloff, ncols, nct, nb, rows, cnt, (T*)buf, ldb, info));
  }
  return (int)hipGetLastError();
}

DPL_API int dpl_rows_permute(int prec, void* A, int ld, int mb, int r0, const long long* rowoff, int nrt,
                             const long long* coloff, const int* ncols, int nct, int nb, const int* dst,
                             const int* src, const int* cnt, int maxcnt, int* info, hipStream_t st) {
  if (nct <= 0 || maxcnt <= 0) return 0;
  if (maxcnt > 1024) return -3;
  const int W = nct * nb;
  const int gx = (W + 3) / 4 > 4096 ? 4096 : (W + 3) / 4;
  DISPATCH(prec, hipLaunchKernelGGL((k_rows_permute<T>), dim3(gx), dim3(256), 0, st, (T*)A, ld, mb, r0, rowoff, nrt,
                                    coloff, ncols, nct, nb, dst, src, cnt, info));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- deferred left interchanges (one process row)
// getrf_1d with DPLASMA_LU_DEFER_LEFT: every step's interchanges touch the trailing columns only, and each factored
// tile column receives, once at the end, the composition of all later steps' interchanges (a permutation of its rows
// [r0, m), host-composed: dplasma_amd.lib._dplasma_rt.piv_compose_left).  GATHER: buf(i, c) = A(src[i], c), the
// reads scattered, the writes coalesced; then A(r0 + i, c) = buf(i, c), coalesced both ways.  Same element moves
// as applying the swaps step by step, each element once (the per-step moves sweep every left column every step).
template <typename T, bool GATHER>
__global__ __launch_bounds__(256) void k_rows_perm_col(T* __restrict__ A, int ld, int mb,
                                                       const long long* __restrict__ rowoff, int nrt, long long coff,
                                                       int ncols, const int* __restrict__ src, int r0, int cnt,
                                                       T* __restrict__ buf, int* __restrict__ info) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cnt) return;
  const int R = GATHER ? src[i] : r0 + i;
  const int rt = R / mb;
  if (R < r0 || rt >= nrt || rowoff[rt] < 0) {   // a row outside [r0, m): a corrupt composition, nothing moves
    if (GATHER) report_bad_pivot(info);
    return;
  }
  const long long base = rowoff[rt] + (R % mb) + coff;
  for (int c = blockIdx.y; c < ncols; c += gridDim.y) {
    if (GATHER) buf[i + (long long)c * cnt] = A[base + (long long)c * ld];
    else A[base + (long long)c * ld] = buf[i + (long long)c * cnt];
  }
}

DPL_API int dpl_rows_perm_col(int prec, void* A, int ld, int mb, const long long* rowoff, int nrt, long long coff,
                              int ncols, const int* src, int r0, int cnt, void* buf, int* info, hipStream_t st) {
  if (cnt <= 0 || ncols <= 0) return 0;
  const dim3 grid((cnt + 255) / 256, ncols < 64 ? ncols : 64);
  DISPATCH(prec, hipLaunchKernelGGL((k_rows_perm_col<T, true>), grid, dim3(256), 0, st, (T*)A, ld, mb, rowoff, nrt,
                                    coff, ncols, src, r0, cnt, (T*)buf, info));
  DISPATCH(prec, hipLaunchKernelGGL((k_rows_perm_col<T, false>), grid, dim3(256), 0, st, (T*)A, ld, mb, rowoff, nrt,
                                    coff, ncols, src, r0, cnt, (T*)buf, info));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- cross-process-row interchanges (P > 1)
// The reference's SWAP_COLLECT / SWAP_SND (src/zgetrf_ptgpanel.jdf:825-984): only the moved rows whose source and
// destination live on DIFFERENT process rows travel, point to point between those two rows of the process column.
// Every rank holds the same net move list (identical pivots), so every rank classifies every move the same way:
//   pack   (s_own == me, d_own == q != me): my staged source row goes into my send buffer for q,
//   unpack (d_own == me, s_own == q != me): q's row arrives in my receive buffer from q,
// at the move's ordinal inside its (source row, destination row) class -- computed identically on both sides, so
// no index travels with the rows.  A class holds at most kb moves (the moves either fill the top block's kb rows or
// empty them), so the buffers are kb rows wide.  xo[t] = (1 << 30 | q << 16 | ord) for pack, (1 << 29 | q << 16 |
// ord) for unpack, -1 for a move that stays on this process row (or is not mine).
__device__ inline int xscan_1024(bool f, int* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long b = __builtin_amdgcn_ballot_w64(f);
  const int in = __builtin_popcountll(b & ((1ULL << lane) - 1ULL));
  if (lane == 0) wsum[w] = __builtin_popcountll(b);
  __syncthreads();
  int off = 0;
  for (int q = 0; q < w; ++q) off += wsum[q];
  __syncthreads();
  return off + in;
}

__global__ __launch_bounds__(1024) void k_rows_xord(const int* __restrict__ dst, const int* __restrict__ src,
                                                    const int* __restrict__ cnt, int r0, int mb,
                                                    const int* __restrict__ prow, int nrt, int me, int P, int ldx,
                                                    int* __restrict__ xo, int* __restrict__ info) {
  __shared__ int wsum[16];
  const int n = cnt[0];
  const int t = threadIdx.x;
  int so = -1, dd = -1;
  if (t < n) {
    const int Rs = r0 + src[t], Rd = r0 + dst[t];
    if (Rs >= 0 && Rd >= 0 && Rs / mb < nrt && Rd / mb < nrt) {
      so = prow[Rs / mb];
      dd = prow[Rd / mb];
    } else {
      report_bad_pivot(info);
    }
  }
  int out = -1;
  for (int q = 0; q < P; ++q) {   // uniform loop: every thread takes part in every scan
    if (q == me) continue;
    const bool fp = so == me && dd == q;
    const int op = xscan_1024(fp, wsum);
    const bool fu = dd == me && so == q;
    const int ou = xscan_1024(fu, wsum);
    if (fp) out = op < ldx ? ((1 << 30) | (q << 16) | op) : -1;
    if (fu) out = ou < ldx ? ((1 << 29) | (q << 16) | ou) : -1;
    if ((fp && op >= ldx) || (fu && ou >= ldx)) report_bad_pivot(info);
  }
  xo[t] = out;
}

// pack: bufs[q][ord + c ldx] = tmp[t + c ldb]; unpack: tmp[t + c ldb] = bufs[q][ord + c ldx] (W columns).  Lanes run
// along the move list, the 4 waves of a workgroup over columns (k_rows_move's shape).
template <typename T, bool PACK>
__global__ __launch_bounds__(256) void k_rows_xcopy(T* __restrict__ tmp, int ldb, int W, const int* __restrict__ xo,
                                                    const int* __restrict__ cnt, T* const* __restrict__ bufs, int ldx) {
  const int n = cnt[0];
  if (blockIdx.y * 64 >= n) return;
  const int t = blockIdx.y * 64 + (threadIdx.x & 63);
  const int x = t < n ? xo[t] : -1;
  const bool act = x >= 0 && ((x >> (PACK ? 30 : 29)) & 1);
  if (__builtin_amdgcn_ballot_w64(act) == 0) return;
  const int q = (x >> 16) & 0x1fff, o = x & 0xffff;
  T* b = act ? bufs[q] : nullptr;
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < W; c += gridDim.x * 4) {
    if (!act) continue;
    if (PACK) b[o + (long long)c * ldx] = tmp[t + (long long)c * ldb];
    else tmp[t + (long long)c * ldb] = b[o + (long long)c * ldx];
  }
}

DPL_API int dpl_rows_xord(const int* dst, const int* src, const int* cnt, int r0, int mb, const int* prow, int nrt,
                          int me, int P, int ldx, int* xo, int* info, hipStream_t st) {
  if (P < 2 || P > 8192 || ldx <= 0 || ldx > 65535) return -3;
  hipLaunchKernelGGL(k_rows_xord, dim3(1), dim3(1024), 0, st, dst, src, cnt, r0, mb, prow, nrt, me, P, ldx, xo, info);
  return (int)hipGetLastError();
}

DPL_API int dpl_rows_xcopy(int prec, int pack, void* tmp, int ldb, int W, const int* xo, const int* cnt, int maxcnt,
                           void* const* bufs, int ldx, hipStream_t st) {
  if (W <= 0 || maxcnt <= 0) return 0;
  if (maxcnt > 1024) return -3;
  const int gx = (W + 3) / 4 > 2048 ? 2048 : (W + 3) / 4;
  dim3 g(gx, (maxcnt + 63) / 64);
  if (pack) {
    DISPATCH(prec, hipLaunchKernelGGL((k_rows_xcopy<T, true>), g, dim3(256), 0, st, (T*)tmp, ldb, W, xo, cnt,
                                      (T* const*)bufs, ldx));
  } else {
    DISPATCH(prec, hipLaunchKernelGGL((k_rows_xcopy<T, false>), g, dim3(256), 0, st, (T*)tmp, ldb, W, xo, cnt,
                                      (T* const*)bufs, ldx));
  }
  return (int)hipGetLastError();
}
