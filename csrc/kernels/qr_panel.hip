// Householder QR of one tall column-major panel in ONE persistent launch (real precisions).
//
// Reference roles: the panel kernels of the tile QR (CORE_zgeqrt / CORE_ztsqrt chains of
// src/zgeqrf.jdf:98-443, core_zgeqrt.c, core_ztsqrt.c) and the compact-WY T construction of
// LAPACK dlarft.  On MI355X the tile chain (one workgroup walks the panel tile by tile, one
// column at a time) is latency bound, so a TS domain of the elimination tree is factored as
// ONE stacked panel here (models/qr_panel.py), spread over up to one workgroup per CU:
//
//  * rows are partitioned once: workgroup w owns rows [w*R, w*R+R) (R <= 256, one row per
//    thread in the column steps) for the whole launch, so every cross-workgroup hand-off is a
//    small reduction (grid_sync.h) and the matrix itself never crosses workgroups;
//  * 32-column blocks live in LDS.  At the start of a block every workgroup forms the block's
//    Gram matrix G = A_b(rows >= b0)^T A_b(rows >= b0) (MFMA partials, ONE grid barrier) and a
//    replica of the block's top 32 rows.  Column j then needs no cross-row reduction at all:
//    G(j, j) = ||A(j:, j)||^2 gives beta / tau, G(j, c) - A(j, j) A(j, c) = x^T A(j+1:, c)
//    gives the reflector's effect on column c, and after the reflector (orthogonal on rows
//    >= j, so the Gram matrix of rows >= j is unchanged) G is downdated by the new row j:
//    G -= r_j^T r_j.  Every workgroup keeps G and the top rows in LDS and updates them
//    redundantly (identical arithmetic -> identical scalars everywhere), so a column costs one
//    workgroup barrier instead of a grid barrier + a 32-value reduction.  When the downdated
//    ||x||^2 falls below 1/8 of the column's block-start norm (cancellation: a nearly
//    dependent column, or the last rows of a square panel) that column takes the exact path:
//    32 partial dot products per workgroup, one grid barrier, redundant reduction (the
//    norm-downdating safeguard of LAPACK dgeqp3, here for the reflector itself);
//  * after a block: Y = V_b^T [V_prev | A_rest] is formed with fp64 MFMA (K = the workgroup's
//    rows), reduced in two barriers (each workgroup sums a slice), then A_rest -= V_b T_b^T Y
//    with MFMA, rows stay resident per workgroup; Y's V_prev part is the T coupling input;
//  * the off-diagonal T blocks T(0:b0, blk) = -T(0:b0,0:b0) (V_prev^T V_b) T_b are formed at
//    the end, each workgroup owning T rows w, w+G, ... (no barrier between blocks).
// Output: P holds R (upper) and V (strictly below the diagonal), V holds V explicitly (unit
// diagonal, zeros above) for the trailing GEMMs, Tm the full upper-triangular kf x kf T
// (its strictly-lower part is left untouched: callers keep it zero).
#include <cstdlib>

#include "common.h"
#include "grid_sync.h"

#define QP_R 256          // rows per workgroup (max)
#define QP_B 32           // block width
#define QP_LD (QP_R + 2)  // LDS column stride (conflict-free MFMA operand reads)
#define QP_WL (QP_B + 2)

template <typename T> struct QPM;
template <> struct QPM<double> {
  typedef d4_t acc_t;
  static __device__ inline acc_t mma(double x, double y, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) + 4 * r; }
  static __device__ inline double rcp(double d) {   // 1/d: hardware estimate + 2 Newton steps
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    return fma(fma(-d, r, 1.0), r, r);
  }
};
template <> struct QPM<float> {
  typedef f4_t acc_t;
  static __device__ inline acc_t mma(float x, float y, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) * 4 + r; }
  static __device__ inline float rcp(float d) { return 1.0f / d; }
};

// mma(x, y, acc): D(p, q) += sum_k x(p, k) y(q, k); input lane l carries p (resp. q) = l & 15,
// k = l >> 4; output acc[r] of lane l is D(drow(l, r), l & 15).
// Workspace layout for a G-workgroup panel (bytes, 256-aligned parts): part1 [2][G][32],
// rowj [2][32] + top rows [32][32] + summed Gram [32][32], part2 [G][32*(nc+32)] (also the Gram partials
// [G][32][32]), Yg [32*(nc+32)], Xc [nblk][32][kf] elements of the precision, then the barrier counter.
__host__ __device__ static inline long long qp_align(long long x) { return (x + 255) & ~255LL; }
__host__ __device__ static inline void qp_layout_g(long long es, int nc, int kf, int G, long long off[6]) {
  const long long nblk = (kf + QP_B - 1) / QP_B;
  off[0] = 0;
  off[1] = off[0] + qp_align(es * 2 * G * QP_B);
  off[2] = off[1] + qp_align(es * (2 * QP_B + 2 * QP_B * QP_B));
  off[3] = off[2] + qp_align(es * (long long)G * QP_B * (nc + QP_B));
  off[4] = off[3] + qp_align(es * QP_B * (nc + QP_B));
  off[5] = off[4] + qp_align(es * nblk * QP_B * kf);
}

template <typename T>
__device__ __forceinline__ void qr_panel_body(T* __restrict__ P0, int ldp, int rbl, long long rstride, int M, int nc,
                                              int kf, int R, T* __restrict__ V, int ldv, T* __restrict__ Tm, int ldt,
                                              T* __restrict__ part1, T* __restrict__ rowj, T* __restrict__ part2,
                                              T* __restrict__ Yg, T* __restrict__ Xc, int* __restrict__ cnt,
                                              int* __restrict__ info, long long* __restrict__ prof, const int G_,
                                              const int w_) {
  typedef QPM<T> MM;
  typedef typename MM::acc_t acc_t;
  __shared__ T Ab[QP_B][QP_LD];     // finished block columns (R / beta / V), later explicit V_b
  __shared__ T Xs[QP_B][QP_LD];     // explicit V_b during the column steps, later streamed chunks
  __shared__ T Ts[QP_B][QP_B + 1];  // T_b, Ts[col][row]
  __shared__ T Ws[QP_B][QP_WL];     // Gram block / Y chunk / T_b^T Y chunk, Ws[col][k]
  __shared__ T red[8][QP_B + 1];
  __shared__ T fin[2 * QP_B];
  __shared__ T ff[QP_B], taus[QP_B];
  const int G = G_, w = w_, tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  __builtin_amdgcn_s_setprio(3);   // critical-path panel: VALU issue priority over co-resident update waves
  const int rbase = w * R;
  const int nr = max(0, min(R, M - rbase));
  const int R16 = (nr + 15) & ~15;
  const int grow = rbase + tid;
  const bool rowok = tid < nr;
  // row grow of the panel starts at P: panel rows come in blocks of rbl rows rstride apart
  // (tile-storage panels are addressed in place; contiguous panels pass rbl >= M)
  T* const P = P0 + (long long)(grow / rbl) * rstride + (grow % rbl) - grow;
  int nsync = 0;
  const int nblk = (kf + QP_B - 1) / QP_B;
  // optional phase timers (workgroup 0, 100 MHz ticks): 0 column-step compute, 1 column barrier,
  // 2 partial reduction, 3 Y partials, 4 Y barriers + reduction + T_b, 5 trailing update, 6 T coupling
  const bool tprof = prof != nullptr && w == 0 && tid == 0;
  unsigned long long tacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // slot 8: column steps up to the reflector effects
  long long nfast = 0, nexact = 0, first_exact = -1;
  double fe_x2 = 0.0, fe_g0 = 0.0;
  unsigned long long tlast = tprof ? __builtin_amdgcn_s_memrealtime() : 0;
#define QP_TICK(slot)                                                \
  if (tprof) {                                                       \
    const unsigned long long tn_ = __builtin_amdgcn_s_memrealtime(); \
    tacc[slot] += tn_ - tlast;                                       \
    tlast = tn_;                                                     \
  }

  // top-rows replica / summed Gram in the workspace (G > 1), Gram partials in part2
  T* const topw = rowj + 2 * QP_B;
  T* const gsum = topw + QP_B * QP_B;
  // LDS replicas of the column steps, aliased on T_b / the Y chunk (both idle during the steps)
  T (*const Gm)[QP_B + 1] = Ts;   // Gram of the block columns over rows >= the active row
  T (*const Tp)[QP_WL] = Ws;      // the block's top 32 rows (Tp[r][c] = A(b0 + r, b0 + c))
  __shared__ T g0[QP_B];          // block-start diagonal of G (cancellation test)

  for (int b = 0; b < nblk; ++b) {
    const int b0 = b * QP_B;
    const int cb = min(QP_B, nc - b0);   // block columns
    const int bw = min(QP_B, kf - b0);   // of which reflectors
    // The thread owning local row tid keeps the row's block in registers, rotated so that the
    // active column is always a[0] (static register indices only).
    T a[QP_B];
#pragma unroll
    for (int c = 0; c < QP_B; ++c) a[c] = (rowok && c < cb) ? P[grow + (long long)(b0 + c) * ldp] : T(0);
    // rows above b0 take no part in the block (zeros of the Gram staging and of V_b): the MFMA K loops
    // start at the first 16-row group that reaches b0
    const int rs16 = max(0, min(R16, b0 - rbase)) & ~15;
    QP_TICK(7);
    // ------------------------------------------------------------ block Gram + top-row replica
    for (int e = tid; e < QP_B * QP_LD; e += 256) {
      (&Xs[0][0])[e] = T(0);
      (&Ab[0][0])[e] = T(0);
    }
    for (int e = tid; e < QP_B * QP_WL; e += 256) (&Tp[0][0])[e] = T(0);
    __syncthreads();
    if (rowok && grow >= b0) {
#pragma unroll
      for (int c = 0; c < QP_B; ++c) Xs[c][tid] = a[c];
    }
    const bool top = rowok && grow >= b0 && grow < b0 + QP_B;
    if (top) {
      if (G == 1) {
#pragma unroll
        for (int c = 0; c < QP_B; ++c) Tp[grow - b0][c] = a[c];
      } else {
#pragma unroll
        for (int c = 0; c < QP_B; ++c) st_sc1(&topw[(grow - b0) * QP_B + c], a[c]);
      }
    }
    __syncthreads();
    {
      const int pt = wv & 1, qt = wv >> 1;
      acc_t a0, a1;
#pragma unroll
      for (int r = 0; r < 4; ++r) a0[r] = a1[r] = T(0);
      for (int r0 = rs16; r0 < R16; r0 += 8) {
        const int rr = r0 + (l >> 4);
        a0 = MM::mma(Xs[pt * 16 + (l & 15)][rr], Xs[qt * 16 + (l & 15)][rr], a0);
        a1 = MM::mma(Xs[pt * 16 + (l & 15)][rr + 4], Xs[qt * 16 + (l & 15)][rr + 4], a1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = pt * 16 + MM::drow(l, r), q = qt * 16 + (l & 15);
        const T y = a0[r] + a1[r];
        if (G == 1) Gm[p][q] = y;
        else st_sc1(&part2[(long long)w * QP_B * QP_B + p * QP_B + q], y);
      }
    }
    if (G > 1) {
      ++nsync;
      grid_sync_counter(cnt, nsync * G, info);
      if (G <= 16) {
        // every workgroup sums the partials itself (same order everywhere: identical G)
        for (int e = tid; e < QP_B * QP_B; e += 256) {
          T t16[16];
#pragma unroll
          for (int bb = 0; bb < 16; ++bb) t16[bb] = bb < G ? ld_sc1(&part2[(long long)bb * QP_B * QP_B + e]) : T(0);
          T s = T(0);
#pragma unroll
          for (int bb = 0; bb < 16; ++bb) s += t16[bb];
          Gm[e >> 5][e & 31] = s;
        }
      } else {
        // workgroup w sums a slice, one more barrier, everyone reads the sum
        const int epw = (QP_B * QP_B + G - 1) / G;
        const int e_beg = w * epw, e_end = min(QP_B * QP_B, e_beg + epw);
        for (int base = e_beg; base < e_end; base += 32) {
          const int e = base + (tid & 31), g = tid >> 5;
          T s = T(0);
          if (e < e_end)
            for (int bb0 = g; bb0 < G; bb0 += 64) {   // 8 partials in flight per thread
              T t8[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int bb = bb0 + 8 * u;
                t8[u] = bb < G ? ld_sc1(&part2[(long long)bb * QP_B * QP_B + e]) : T(0);
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) s += t8[u];
            }
          red[g][tid & 31] = s;
          __syncthreads();
          if (tid < 32 && e < e_end) {
            T y = T(0);
#pragma unroll
            for (int gg = 0; gg < 8; ++gg) y += red[gg][tid];
            st_sc1(&gsum[e], y);
          }
          __syncthreads();
        }
        ++nsync;
        grid_sync_counter(cnt, nsync * G, info);
        for (int e = tid; e < QP_B * QP_B; e += 256) Gm[e >> 5][e & 31] = ld_sc1(&gsum[e]);
      }
      for (int e = tid; e < QP_B * QP_B; e += 256) {
        const int r = e >> 5, c = e & 31;
        Tp[r][c] = b0 + r < M ? ld_sc1(&topw[e]) : T(0);
      }
    }
    __syncthreads();
    if (tid < QP_B) g0[tid] = Gm[tid][tid];
    for (int e = tid; e < QP_B * QP_LD; e += 256) (&Xs[0][0])[e] = T(0);
    __syncthreads();
    QP_TICK(0);
    // ------------------------------------------------------------ column steps
    for (int jj = 0; jj < bw; ++jj) {
      const int j = b0 + jj;
      const int sh = QP_B - jj;  // live slots: slot s is column jj + s
      // this thread's replica operands (entries (r0 + 8u, c) below): they do not depend on the column's
      // reflector, so their LDS loads are issued first and overlap its computation
      const int rc_c = tid & 31, rc_r0 = tid >> 5;
      T p_trj[4], p_tjr[4], p_tpv[4], p_gmv[4];
      const T p_tjc = Tp[jj][rc_c];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rc_r0 + 8 * u;
        p_trj[u] = Tp[r][jj];
        p_tjr[u] = Tp[jj][r];
        p_tpv[u] = Tp[r][rc_c];
        p_gmv[u] = Gm[r][rc_c];
      }
      const T alpha = Tp[jj][jj], gjj = Gm[jj][jj];
      const T x2f = gjj - alpha * alpha;
      // uniform over the whole grid: every workgroup holds the same replicas
      const bool fast = x2f > T(0.125) * g0[jj];
      if (tprof) {
        if (fast) ++nfast;
        else {
          if (nexact++ == 0) { first_exact = j; fe_x2 = (double)x2f; fe_g0 = (double)g0[jj]; }
        }
      }
      T beta, tau, scale;
      const T* fw;   // slot-indexed reflector effects ff(s) = tau (A(j, jj+s) + scale x^T A(j+1:, jj+s))
      if (fast) {
        const T nrm = sqrt(gjj);
        beta = alpha >= T(0) ? -nrm : nrm;
        // reciprocals by the hardware estimate + Newton steps (full precision) instead of two IEEE divisions on
        // the column's dependent chain
        tau = (beta - alpha) * MM::rcp(beta);
        scale = MM::rcp(alpha - beta);
        // each wave derives the 32 effects itself (no workgroup barrier): lane s -> column jj + s
        if (l < QP_B) {
          const int c = jj + l;
          T f = T(0);
          if (l >= 1 && c < cb) {
            const T tj = Tp[jj][c];
            f = tau * (tj + scale * (Gm[jj][c] - alpha * tj));
          }
          red[wv][l] = f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        fw = red[wv];
        QP_TICK(8);
      } else {
      const int par = nsync & 1;
      {
        // x = A(r > j, j) against every live column, then a wave transpose-reduction:
        // lane l ends with the wave's sum for slot l >> 1
        const T x = (rowok && grow > j) ? a[0] : T(0);
        T v[QP_B];
#pragma unroll
        for (int s = 0; s < QP_B; ++s) v[s] = s < sh ? x * a[s] : T(0);
#pragma unroll
        for (int wdt = QP_B / 2, m = 32; wdt >= 1; wdt >>= 1, m >>= 1) {
          const bool hi = (l & m) != 0;
#pragma unroll
          for (int i = 0; i < wdt; ++i) {
            const T send = hi ? v[i] : v[wdt + i];
            const T keep = hi ? v[wdt + i] : v[i];
            v[i] = keep + __shfl_xor(send, m, 64);
          }
        }
        v[0] += __shfl_xor(v[0], 1, 64);
        if ((l & 1) == 0) red[wv][l >> 1] = v[0];
        if (rowok && grow == j) {
          if (G == 1) {   // one workgroup: row j's snapshot through LDS
#pragma unroll
            for (int s = 0; s < QP_B; ++s) fin[QP_B + s] = s < sh ? a[s] : T(0);
          } else {
            T* rj = rowj + par * QP_B;
#pragma unroll
            for (int s = 0; s < QP_B; ++s)
              if (s < sh) st_sc1(&rj[s], a[s]);
          }
        }
      }
      __syncthreads();
      if (G == 1) {
        // one workgroup: the four waves' partials are the whole sum -- no global round trip
        if (tid < QP_B) fin[tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        __syncthreads();
      } else {
      if (tid < QP_B) {
        const T d = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        st_sc1(&part1[((long long)par * G + w) * QP_B + tid], d);
      }
      ++nsync;
      grid_sync_counter(cnt, nsync * G, info);
      {
        // thread (slot s, group q) sums partials q, q+8, ... (up to 16 loads in flight)
        const int s = tid & 31, q = tid >> 5;
        T acc = T(0);
        if (s < sh) {
          const T* src = part1 + (long long)par * G * QP_B + s;
          for (int base = q; base < G; base += 8 * 16) {
            T t[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int bb = base + 8 * u;
              t[u] = bb < G ? ld_sc1(&src[(long long)bb * QP_B]) : T(0);
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) acc += t[u];
          }
        }
        red[q][s] = acc;
        if (tid < QP_B) fin[QP_B + tid] = tid < sh ? ld_sc1(&rowj[par * QP_B + tid]) : T(0);
      }
      __syncthreads();
      if (tid < QP_B) {
        T d = T(0);
#pragma unroll
        for (int q = 0; q < 8; ++q) d += red[q][tid];
        fin[tid] = d;
      }
      __syncthreads();
      }
      // dlarfg (every thread derives the same scalars); slot 0 is column jj
      const T ea = fin[QP_B], x2 = fin[0];
      if (x2 == T(0)) {
        beta = ea;
        tau = T(0);
        scale = T(0);
      } else {
        const T nrm = sqrt(ea * ea + x2);
        beta = ea >= T(0) ? -nrm : nrm;
        tau = (beta - ea) / beta;
        scale = T(1) / (ea - beta);
      }
      if (tid < QP_B)
        ff[tid] = (tid >= 1 && tid < sh && jj + tid < cb) ? tau * (fin[QP_B + tid] + scale * fin[tid]) : T(0);
      __syncthreads();
      fw = ff;
      QP_TICK(2);
      }
      if (tid == 0) taus[jj] = tau;
      if (rowok) {
        const T x = a[0];
        const T vr = grow > j ? scale * x : (grow == j ? T(1) : T(0));
#pragma unroll
        for (int s = 1; s < QP_B; ++s) a[s] -= vr * fw[s];
        Ab[jj][tid] = grow < j ? x : (grow == j ? beta : vr);
        Xs[jj][tid] = vr;
      }
      // replicas: rows r > jj of the top block take the reflector like any row; the Gram matrix
      // of rows > j is the (unchanged) one of rows >= j minus the new row j's outer product
      {
        // thread (c, r0) owns entries (r0 + 8u, c), u < 4: every operand was loaded at the top of the step
        const int c = rc_c, r0 = rc_r0;
        if (c > jj) {
          const T fc = fw[c - jj];
          const T njc = p_tjc - fc;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = r0 + 8 * u;
            if (r > jj) {
              const T nrj = p_tjr[u] - fw[r - jj];
              Tp[r][c] = p_tpv[u] - (scale * p_trj[u]) * fc;
              Gm[r][c] = p_gmv[u] - nrj * njc;
            }
          }
        }
      }
#pragma unroll
      for (int s = 0; s < QP_B - 1; ++s) a[s] = a[s + 1];
      a[QP_B - 1] = T(0);
      __syncthreads();
      QP_TICK(1);
    }
    for (int e = tid; e < QP_B * (QP_B + 1); e += 256) (&Ts[0][0])[e] = T(0);
    // non-reflector block columns (kf < nc): still in registers, rotated by bw
    if (rowok)
#pragma unroll
      for (int s = 0; s < QP_B; ++s)
        if (s < cb - bw) Ab[(bw + s) & (QP_B - 1)][tid] = a[s];
    __syncthreads();
    // ------------------------------------------------------------ block results (row per thread)
    if (rowok) {
#pragma unroll
      for (int c = 0; c < QP_B; ++c) {
        if (c < cb) P[grow + (long long)(b0 + c) * ldp] = Ab[c][tid];
        if (c < bw) V[grow + (long long)(b0 + c) * ldv] = Xs[c][tid];
      }
    }
    if (tid < R16)
      for (int c = 0; c < QP_B; ++c) Ab[c][tid] = c < bw ? Xs[c][tid] : T(0);
    __syncthreads();
    // ------------------------------------------------------------ Y partials: V_b^T [V_b | V_prev | A_rest]
    const int nA = nc - b0 - cb;
    const int nX = QP_B + b0 + nA;
    const bool act = rbase + nr > b0;
    const long long E = (long long)QP_B * nX;
    // the next global chunk's loads are issued before the current chunk's MFMA (in flight during it)
    T t[QP_B];
    auto fetch_y = [&](int x0) {
      const int cw = min(QP_B, nX - x0);
      const bool live = act && tid < R16 && rowok && grow >= b0;
      // chunks never straddle the V_b | V_prev | A_rest boundaries (b0 is a multiple of 32)
      const T* src = x0 < QP_B + b0 ? V + grow + (long long)(x0 - QP_B) * ldv
                                    : P + grow + (long long)(cb + x0 - QP_B) * ldp;
      const long long ld = x0 < QP_B + b0 ? ldv : ldp;
#pragma unroll
      for (int c = 0; c < QP_B; ++c) t[c] = (live && c < cw) ? src[c * ld] : T(0);
    };
    if (nX > QP_B) fetch_y(QP_B);
    for (int x0 = 0; x0 < nX; x0 += QP_B) {
      const int cw = min(QP_B, nX - x0);
      T* pw = G == 1 ? Yg : part2 + (long long)w * E;   // one workgroup: its partial IS Y
      if (act) {
        if (tid < R16) {
          if (x0 < QP_B) {
            for (int c = 0; c < QP_B; ++c) Xs[c][tid] = Ab[c][tid];
          } else {
#pragma unroll
            for (int c = 0; c < QP_B; ++c) Xs[c][tid] = t[c];
          }
        }
        __syncthreads();
        if (x0 >= QP_B && x0 + QP_B < nX) fetch_y(x0 + QP_B);
        const int pt = wv & 1, qt = wv >> 1;
        acc_t a0, a1, a2, a3;
#pragma unroll
        for (int r = 0; r < 4; ++r) a0[r] = a1[r] = a2[r] = a3[r] = T(0);
        for (int r0 = rs16; r0 < R16; r0 += 16) {
          const int rr = r0 + (l >> 4);
          a0 = MM::mma(Ab[pt * 16 + (l & 15)][rr], Xs[qt * 16 + (l & 15)][rr], a0);
          a1 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 4], Xs[qt * 16 + (l & 15)][rr + 4], a1);
          a2 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 8], Xs[qt * 16 + (l & 15)][rr + 8], a2);
          a3 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 12], Xs[qt * 16 + (l & 15)][rr + 12], a3);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = pt * 16 + MM::drow(l, r), q = qt * 16 + (l & 15);
          if (q < cw) {
            const T y = (a0[r] + a1[r]) + (a2[r] + a3[r]);
            st_sc1(&pw[(long long)p * nX + x0 + q], y);
            const int xc = x0 + q;
            if (G == 1 && xc >= QP_B && xc < QP_B + b0) st_sc1(&Xc[((long long)b * QP_B + p) * kf + xc - QP_B], y);
          }
        }
        __syncthreads();
      } else {
        for (int p = wv; p < QP_B; p += 4)
          if (l < cw) st_sc1(&pw[(long long)p * nX + x0 + l], T(0));
      }
    }
    QP_TICK(3);
    if (G == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    // ------------------------------------------------------------ Y = sum of partials
    if (G <= 8) {
      // few partials: thread per entry, no LDS round
      const long long epw = (E + G - 1) / G;
      const long long e_beg = (long long)w * epw, e_end = min(E, e_beg + epw);
      for (long long e = e_beg + tid; e < e_end; e += 256) {
        T t8[8];
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) t8[bb] = bb < G ? ld_sc1(&part2[(long long)bb * E + e]) : T(0);
        T y = T(0);
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) y += t8[bb];
        st_sc1(&Yg[e], y);
        const int p = (int)(e / nX), xc = (int)(e - (long long)p * nX);
        if (xc >= QP_B && xc < QP_B + b0) st_sc1(&Xc[((long long)b * QP_B + p) * kf + xc - QP_B], y);
      }
    } else {
      const long long epw = (E + G - 1) / G;
      const long long e_beg = (long long)w * epw, e_end = min(E, e_beg + epw);
      for (long long base = e_beg; base < e_end; base += 32) {
        const long long e = base + (tid & 31);
        const int g = tid >> 5;
        T s = T(0);
        if (e < e_end)
          for (int bb0 = g; bb0 < G; bb0 += 64) {   // 8 partials in flight per thread
            T t8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int bb = bb0 + 8 * u;
              t8[u] = bb < G ? ld_sc1(&part2[(long long)bb * E + e]) : T(0);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s += t8[u];
          }
        red[g][tid & 31] = s;
        __syncthreads();
        if (tid < 32 && e < e_end) {
          T y = T(0);
#pragma unroll
          for (int gg = 0; gg < 8; ++gg) y += red[gg][tid];
          st_sc1(&Yg[e], y);
          const int p = (int)(e / nX), xc = (int)(e - (long long)p * nX);
          if (xc >= QP_B && xc < QP_B + b0) st_sc1(&Xc[((long long)b * QP_B + p) * kf + xc - QP_B], y);
        }
        __syncthreads();
      }
    }
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    }
    // ------------------------------------------------------------ T_b from taus and the Gram block
    for (int e = tid; e < QP_B * QP_B; e += 256) {
      const int c = e >> 5, k = e & 31;
      Ws[c][k] = ld_sc1(&Yg[(long long)k * nX + c]);   // G_b(k, c) = v_k^T v_c
    }
    __syncthreads();
    if (tid < bw) {
      // T_b in two 16-reflector halves: lane i builds row i of T11 (i < 16) or of T22 (the compact-WY factor of
      // reflectors 16..31 alone) by the dlarft recurrence T(i, j) = -tau_j sum_{k=i}^{j-1} T(i, k) G(k, j) --
      // a quarter of the 32-long recurrence's sequential work (~20 us of LDS round trips per block before)
      const int i = tid, h1 = min(bw, (i < 16 ? 0 : 16) + 16);
      Ts[i][i] = taus[i];
      for (int jc = i + 1; jc < h1; ++jc) {
        T z = T(0);
        for (int k = i; k < jc; ++k) z += Ts[k][i] * Ws[jc][k];
        Ts[jc][i] = -taus[jc] * z;
      }
    }
    __syncthreads();
    if (bw > 16) {
      // T12 = -T11 (V1^T V2) T22: X = G12 T22 then T11 X, a thread per entry (16 x 16 = 256 threads); Xs is idle
      // between the column steps and the trailing update
      const int i = tid & 15, j = 16 + (tid >> 4);
      T x = T(0);
      if (j < bw)
        for (int k = 16; k <= j; ++k) x += Ws[k][i] * Ts[j][k];   // G(i, k) T22(k, j)
      Xs[j - 16][i] = x;
      __syncthreads();
      if (j < bw) {
        T y = T(0);
        for (int k = i; k < 16; ++k) y += Ts[k][i] * Xs[j - 16][k];
        Ts[j][i] = -y;
      }
      __syncthreads();
    }
    if (w == 0)
      for (int e = tid; e < bw * bw; e += 256) {
        const int c = e / bw, i = e - c * bw;
        st_sc1(&Tm[(b0 + i) + (long long)(b0 + c) * ldt], i <= c ? Ts[c][i] : T(0));
      }
    QP_TICK(4);
    // ------------------------------------------------------------ A_rest -= V_b (T_b^T Y)
    if (nA > 0 && act) {
      const int ycol0 = QP_B + b0;
      const bool live = tid < R16 && rowok && grow >= b0;
      auto fetch_a = [&](int a0) {
        const int cw = min(QP_B, nA - a0);
        const T* src = P + grow + (long long)(b0 + cb + a0) * ldp;
#pragma unroll
        for (int c = 0; c < QP_B; ++c) t[c] = (live && c < cw) ? src[(long long)c * ldp] : T(0);
      };
      fetch_a(0);
      for (int a0 = 0; a0 < nA; a0 += QP_B) {
        const int cw = min(QP_B, nA - a0);
        for (int e = tid; e < QP_B * QP_B; e += 256) {
          const int q = e >> 5, i = e & 31;
          Ws[q][i] = q < cw ? ld_sc1(&Yg[(long long)i * nX + ycol0 + a0 + q]) : T(0);
        }
        if (tid < R16) {
#pragma unroll
          for (int c = 0; c < QP_B; ++c) Xs[c][tid] = t[c];
        }
        __syncthreads();
        if (a0 + QP_B < nA) fetch_a(a0 + QP_B);   // next chunk in flight during this one
        {
          // W' = T_b^T Y_chunk on MFMA: wave (pt, qt) forms the 16 x 16 tile W'(pt, qt), K = 32
          const int pt = wv & 1, qt = wv >> 1;
          acc_t acc;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = T(0);
#pragma unroll
          for (int i0 = 0; i0 < QP_B; i0 += 4) {
            const int i = i0 + (l >> 4);
            acc = MM::mma(Ts[pt * 16 + (l & 15)][i], Ws[qt * 16 + (l & 15)][i], acc);
          }
          __syncthreads();
#pragma unroll
          for (int r = 0; r < 4; ++r) Ws[qt * 16 + (l & 15)][pt * 16 + MM::drow(l, r)] = acc[r];
        }
        __syncthreads();
        const int RT = R16 / 16;
        for (int tt = rs16 / 16 * 2 + wv; tt < RT * 2; tt += 4) {
          const int rt = tt >> 1, qt = tt & 1;
          acc_t acc;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = Xs[qt * 16 + (l & 15)][rt * 16 + MM::drow(l, r)];
#pragma unroll
          for (int k0 = 0; k0 < QP_B; k0 += 4) {
            const int k = k0 + (l >> 4);
            acc = MM::mma(-Ab[k][rt * 16 + (l & 15)], Ws[qt * 16 + (l & 15)][k], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) Xs[qt * 16 + (l & 15)][rt * 16 + MM::drow(l, r)] = acc[r];
        }
        __syncthreads();
        if (rowok && grow >= b0) {
          T* dst = P + grow + (long long)(b0 + cb + a0) * ldp;
#pragma unroll
          for (int c = 0; c < QP_B; ++c)
            if (c < cw) dst[(long long)c * ldp] = Xs[c][tid];
        }
        __syncthreads();
      }
    }
    QP_TICK(5);
  }
  // ------------------------------------------------------------ off-diagonal T blocks
  // T(0:b0, blk) = -T(0:b0, 0:b0) Z, Z = X_b T_b, X_b = V_prev^T V_b.  Workgroup w owns the 16-row tiles
  // w, w+G, ... of T for every block, so besides the diagonal blocks (final before the barrier) it reads
  // only T rows it wrote itself.  Two row tiles at a time are staged in LDS and multiplied by Z with
  // MFMA (the k-range of a row tile starts at its diagonal: T is upper triangular) -- was a scalar
  // row-by-row loop whose global round trips cost ~0.7 ms per 256-column panel on one workgroup.
  if (nblk > 1) {
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    for (int b = 1; b < nblk; ++b) {
      const int b0 = b * QP_B, bw = min(QP_B, kf - b0);
      const int nrt = b0 / 16;
      if (w >= nrt) continue;
      for (int e = tid; e < QP_B * QP_B; e += 256) {
        const int c = e >> 5, k = e & 31;
        Ts[c][k] = (k <= c && c < bw) ? ld_sc1(&Tm[(b0 + k) + (long long)(b0 + c) * ldt]) : T(0);
      }
      if (tid < b0)
        for (int k = 0; k < QP_B; ++k) Ab[k][tid] = k < bw ? ld_sc1(&Xc[((long long)b * QP_B + k) * kf + tid]) : T(0);
      __syncthreads();
      // Z = X_b T_b on MFMA (b0 x 32 times 32 x 32, T_b upper triangular with zeros below): wave wv forms the
      // 16 x 16 tiles wv, wv + 4, ... of Z -- was a scalar 32 x 32 loop per row (~0.2 ms per panel on G = 1)
      for (int zt = wv; zt < (b0 / 16) * 2; zt += 4) {
        const int pt = zt >> 1, qt = zt & 1;
        acc_t acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = T(0);
#pragma unroll
        for (int k0 = 0; k0 < QP_B; k0 += 4) {
          const int k = k0 + (l >> 4);
          acc = MM::mma(Ab[k][pt * 16 + (l & 15)], Ts[qt * 16 + (l & 15)][k], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Xs[qt * 16 + (l & 15)][pt * 16 + MM::drow(l, r)] = acc[r];   // Z(j, c)
      }
      __syncthreads();
      T* trow = &Ab[0][0];   // [32][b0]: the staged T rows of two own row tiles
      const int own_rt = (nrt - w + G - 1) / G;
      for (int o0 = 0; o0 < own_rt; o0 += 2) {
        for (int e = tid; e < 32 * b0; e += 256) {
          const int rl = e / b0, k = e - rl * b0;
          const int ot = o0 + (rl >> 4);
          const int i = (w + ot * G) * 16 + (rl & 15);
          trow[e] = (ot < own_rt && k >= i) ? ld_sc1(&Tm[i + (long long)k * ldt]) : T(0);
        }
        __syncthreads();
        const int ot = o0 + (wv >> 1), ch = wv & 1;
        if (ot < own_rt) {
          const int rt = w + ot * G, rl0 = (wv >> 1) * 16;
          acc_t acc;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = T(0);
          for (int k0 = rt * 16; k0 < b0; k0 += 4) {
            const int k = k0 + (l >> 4);
            acc = MM::mma(trow[(rl0 + (l & 15)) * b0 + k], Xs[ch * 16 + (l & 15)][k], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = ch * 16 + (l & 15);
            if (c < bw) st_sc1(&Tm[(rt * 16 + MM::drow(l, r)) + (long long)(b0 + c) * ldt], -acc[r]);
          }
        }
        __syncthreads();
      }
    }
  }
  QP_TICK(6);
  if (tprof)
    for (int i = 0; i < 8; ++i) prof[i] += (long long)tacc[i];
  if (tprof) prof[13] += (long long)tacc[8];
  if (tprof) {   // column-path counters (the prof buffer holds 16 slots)
    prof[8] += nfast;
    prof[9] += nexact;
    prof[10] = first_exact;
    prof[11] = __double_as_longlong(fe_x2);
    prof[12] = __double_as_longlong(fe_g0);
  }
#undef QP_TICK
}

template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_panel_persist(T* __restrict__ P0, int ldp, int rbl, long long rstride,
                                                             int M, int nc, int kf, int R,
                                                             T* __restrict__ V, int ldv, T* __restrict__ Tm, int ldt,
                                                             T* __restrict__ part1, T* __restrict__ rowj,
                                                             T* __restrict__ part2, T* __restrict__ Yg,
                                                             T* __restrict__ Xc, int* __restrict__ cnt,
                                                             int* __restrict__ info, long long* __restrict__ prof,
                                                             const int* __restrict__ pred) {
  // predicated issue (a device-decided branch, dpl_qr_panel_set_pred): every workgroup reads the same flag before
  // any hand-off, so a skipped launch exits whole
  if (pred && __builtin_amdgcn_readfirstlane(*pred) == 0) return;
  qr_panel_body<T>(P0, ldp, rbl, rstride, M, nc, kf, R, V, ldv, Tm, ldt, part1, rowj, part2, Yg, Xc, cnt, info, prof,
                   gridDim.x, blockIdx.x);
}

// Several independent panels in ONE launch (the TS domains of one panel step of a hierarchical tree,
// or the TT stacks of one tree round): panel e owns workgroups [wbase, wbase + G) and its own
// workspace / barrier counter; every panel's workgroups are co-resident (sum of G <= CUs).
struct QpItem {
  void* P0;
  long long rstride;
  void* V;
  void* Tm;
  char* ws;   // qp_layout_g parts 0..4
  int* cnt;   // barrier counter (zeroed before every launch)
  int ldp, rbl, M, nc, kf, R, ldv, ldt, G, wbase;
};

template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_panel_multi(const QpItem* __restrict__ items, int nitems,
                                                           int* __restrict__ info, const int* __restrict__ pred) {
  if (pred && __builtin_amdgcn_readfirstlane(*pred) == 0) return;
  int e = 0;
  while (e + 1 < nitems && items[e + 1].wbase <= (int)blockIdx.x) ++e;
  const QpItem it = items[e];
  long long off[6];
  qp_layout_g(sizeof(T), it.nc, it.kf, it.G, off);
  char* b = it.ws;
  qr_panel_body<T>((T*)it.P0, it.ldp, it.rbl, it.rstride, it.M, it.nc, it.kf, it.R, (T*)it.V, it.ldv, (T*)it.Tm,
                   it.ldt, (T*)(b + off[0]), (T*)(b + off[1]), (T*)(b + off[2]), (T*)(b + off[3]), (T*)(b + off[4]),
                   it.cnt, info, nullptr, it.G, (int)blockIdx.x - it.wbase);
}

static int g_qp_cus = 0;
static int qp_cus() {
  if (g_qp_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_qp_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_qp_cus <= 0) g_qp_cus = 1;
    if (g_qp_cus > 256) g_qp_cus = 256;
  }
  return g_qp_cus;
}

static long long* g_qp_prof = nullptr;
// Predicate of the next launches (device int32, 0 = skip; nullptr: none): models/lu_qr.py's device-decided steps
// issue the QR branch under the decision flag (ops/batch.py predicated), and the real-precision panel kernels honour
// it like the batched launches (complex panels run and their results are discarded by the predicated write-back)
static const int* g_qp_pred = nullptr;
DPL_API int dpl_qr_panel_set_pred(const void* dev_ptr) {
  g_qp_pred = (const int*)dev_ptr;
  return 0;
}
// Debug: accumulate workgroup 0's phase timers (8 x int64, 100 MHz ticks) into dev_ptr (nullptr: off).
DPL_API int dpl_qr_panel_set_prof(void* dev_ptr) {
  g_qp_prof = (long long*)dev_ptr;
  return 0;
}

// single-panel layout: sized for the largest grid (one workgroup per CU, <= 256)
static inline void qp_layout(long long es, int nc, int kf, long long off[6]) { qp_layout_g(es, nc, kf, 256, off); }

// complex precisions: qr_panel_z.hip (16-column blocks, VALU block products)
DPL_API long long dpl_qr_panel_z_ws_bytes(int prec, int nc, int kf);
DPL_API int dpl_qr_panel_z(int prec, void* P, int ldp, int rbl, long long rstride, int M, int nc, int kf, void* V,
                           int ldv, void* Tm, int ldt, void* ws, int* info, hipStream_t st);

DPL_API long long dpl_qr_panel_ws_bytes(int prec, int nc, int kf) {
  if (prec == DPL_Z || prec == DPL_C) return dpl_qr_panel_z_ws_bytes(prec, nc, kf);
  long long off[6];
  qp_layout(prec == DPL_D ? 8 : 4, nc, kf, off);
  return off[5] + 256;
}

// Largest panel height the single-launch kernel takes (one workgroup per CU, <= 256 rows each).
DPL_API int dpl_qr_panel_max_rows() { return qp_cus() * QP_R; }

// P: column-major panel (ld ldp); rbl > 0 && rbl < M: rows come in blocks of rbl rows that are
// rstride elements apart (tile storage: rbl = mb, rstride = mb * nb, ldp = mb).
DPL_API int dpl_qr_panel(int prec, void* P, int ldp, int rbl, long long rstride, int M, int nc, int kf, void* V,
                         int ldv, void* Tm, int ldt, void* ws, int* info, hipStream_t st) {
  if (kf <= 0) return 0;
  if (prec == DPL_Z || prec == DPL_C) return dpl_qr_panel_z(prec, P, ldp, rbl, rstride, M, nc, kf, V, ldv, Tm, ldt, ws, info, st);
  if (prec != DPL_D && prec != DPL_S) return -2;
  if (rbl <= 0 || rbl >= M) {
    rbl = 1 << 30;
    rstride = 0;
    if (ldp < M) return -3;
  } else if (ldp < rbl) {
    return -3;
  }
  if (kf > M || kf > nc || kf > QP_R || ldv < M || ldt < kf) return -3;
  const int cus = qp_cus();
  int G = (M + QP_R - 1) / QP_R;
  if (G > cus) return -4;
  if (G < 1) G = 1;
  {  // DPLASMA_QP_GMIN=g (measurement knob): at least g workgroups -- short panels (TT kills: 2 x nb rows) get more
     // hands for their Y partials and T coupling, at the price of wider per-column reductions
    static int gmin = -1, rmax = -1;
    if (gmin < 0) {
      const char* e = getenv("DPLASMA_QP_GMIN");
      gmin = e ? atoi(e) : 0;
      const char* r = getenv("DPLASMA_QP_RMAX");   // at most this many rows per workgroup (measurement knob)
      rmax = r ? atoi(r) : 0;
    }
    int want = gmin;
    if (rmax > 0 && (M + rmax - 1) / rmax > want) want = (M + rmax - 1) / rmax;
    if (want > G) G = want < cus ? (want < M ? want : M) : cus;
  }
  const int R = (M + G - 1) / G;
  long long off[6];
  qp_layout(prec == DPL_D ? 8 : 4, nc, kf, off);
  char* b = (char*)ws;
  void *part1 = b + off[0], *rowj = b + off[1], *part2 = b + off[2], *Yg = b + off[3], *Xc = b + off[4];
  int* cnt = (int*)(b + off[5]);
  hipMemsetAsync(cnt, 0, sizeof(int), st);
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_qr_panel_persist<double>), dim3(G), dim3(256), 0, st, (double*)P, ldp, rbl, rstride, M, nc, kf, R,
                       (double*)V, ldv, (double*)Tm, ldt, (double*)part1, (double*)rowj, (double*)part2, (double*)Yg, (double*)Xc,
                       cnt, info, g_qp_prof, g_qp_pred);
  else
    hipLaunchKernelGGL((k_qr_panel_persist<float>), dim3(G), dim3(256), 0, st, (float*)P, ldp, rbl, rstride, M, nc, kf, R,
                       (float*)V, ldv, (float*)Tm, ldt, (float*)part1, (float*)rowj, (float*)part2, (float*)Yg, (float*)Xc, cnt,
                       info, g_qp_prof, g_qp_pred);
  return (int)hipGetLastError();
}

// dst[i] = sum_s src[s * stride + i], i < L: the split-K partials of the QR trailing GEMMs
// (wide grid, 2 elements per thread, S loads in flight per thread).
template <typename T>
__global__ __launch_bounds__(256) void k_sum_partials(const T* __restrict__ src, long long stride, int S, long long L,
                                                     T* __restrict__ dst) {
  const long long i = 2 * ((long long)blockIdx.x * 256 + threadIdx.x);
  if (i >= L) return;
  const bool two = i + 1 < L;
  T a0 = T(0), a1 = T(0), b0 = T(0), b1 = T(0);
  int s = 0;
  for (; s + 1 < S; s += 2) {
    const T* p = src + (long long)s * stride + i;
    a0 += p[0];
    b0 += p[stride];
    if (two) {
      a1 += p[1];
      b1 += p[stride + 1];
    }
  }
  if (s < S) {
    const T* p = src + (long long)s * stride + i;
    a0 += p[0];
    if (two) a1 += p[1];
  }
  dst[i] = a0 + b0;
  if (two) dst[i + 1] = a1 + b1;
}

DPL_API int dpl_sum_partials(int prec, const void* src, long long stride, int S, long long L, void* dst,
                             hipStream_t st) {
  if (L <= 0 || S <= 0) return 0;
  if (prec == DPL_Z || prec == DPL_C) {   // complex sums are sums of (re, im) pairs
    prec = prec == DPL_Z ? DPL_D : DPL_S;
    stride *= 2;
    L *= 2;
  }
  const unsigned nblk = (unsigned)((L + 511) / 512);
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_sum_partials<double>), dim3(nblk), dim3(256), 0, st, (const double*)src, stride, S, L,
                       (double*)dst);
  else if (prec == DPL_S)
    hipLaunchKernelGGL((k_sum_partials<float>), dim3(nblk), dim3(256), 0, st, (const float*)src, stride, S, L,
                       (float*)dst);
  else
    return -2;
  return (int)hipGetLastError();
}

// Workspace bytes of one panel of a multi launch (G workgroups).
DPL_API long long dpl_qr_panel_multi_ws_bytes(int prec, int nc, int kf, int G) {
  long long off[6];
  qp_layout_g(prec == DPL_D ? 8 : 4, nc, kf, G, off);
  return off[5] + 256;
}

// items: device array of n panels (QpItem, validated by the caller: rbl in (0, M) or 1 << 30, G = ceil(M / 256),
// R = ceil(M / G), wbase = prefix sum of G, sum of G = total <= CUs); the n barrier counters are the
// ints cnt0[0..n) (each item's cnt points there), zeroed here.  Real precisions only.
DPL_API int dpl_qr_panel_multi(int prec, int n, int total, const void* items, int* cnt0, int* info, hipStream_t st) {
  if (n <= 0) return 0;
  if (prec != DPL_D && prec != DPL_S) return -2;
  if (total <= 0 || total > qp_cus()) return -4;
  HIP_CHECK_RET(hipMemsetAsync(cnt0, 0, sizeof(int) * n, st));
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_qr_panel_multi<double>), dim3(total), dim3(256), 0, st, (const QpItem*)items, n, info, g_qp_pred);
  else
    hipLaunchKernelGGL((k_qr_panel_multi<float>), dim3(total), dim3(256), 0, st, (const QpItem*)items, n, info, g_qp_pred);
  return (int)hipGetLastError();
}

DPL_API int dpl_qr_panel_item_bytes() { return (int)sizeof(QpItem); }
