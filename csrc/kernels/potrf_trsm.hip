// Triangular tile kernels: POTRF of one diagonal tile and batched TRSM strips.
//
// Reference roles:
//   * POTRF tile  — cusolverDnZpotrf in src/zpotrf_L.jdf:118-146 (CUDA body) and
//                   CORE_zpotrf -> LAPACKE_zpotrf_work (src/cores/core_zpotrf.c:68-74);
//                   info convention *INFO = k*mb + iinfo (src/zpotrf_L.jdf:180-182).
//   * TRSM tile   — cublasZtrsm_v2 in src/zpotrf_L.jdf:221-243 and CORE_ztrsm
//                   (src/cores/core_ztrsm.c:80); all 8 side/uplo/trans variants.
//
// Design (CDNA4): the POTRF tile is latency-critical (it sits on the lookahead
// critical path) but tiny (n^3/3 flops), so it runs as ONE 512-thread
// workgroup: a right-looking blocked factorization with b=16 column panels kept
// in LDS; the diagonal 16x16 block is factored and inverted by one wave, the
// panel below is multiplied by inv(D)^H by all waves, and the trailing update
// is register-blocked 4x4 per thread from the LDS panel.
// TRSM is batched: one 256-thread workgroup per (tile, strip of VS independent
// vectors); the strip of X lives in LDS for the whole solve (left-looking),
// the triangular factor is streamed through LDS in 16x64 chunks, and each
// 16x16 diagonal block is solved by one wave.  Every side/uplo/trans/diag
// variant reduces to "lower-triangular M, forward order" through strides and an
// index reversal, so one kernel template serves all eight.
#include "common.h"

// ------------------------------------------------------------------ POTRF
// Access L(i,j) = conj?(A[i*si + j*sj]) : lower storage si=1,sj=lda; upper
// storage (factor U = L^H) si=lda, sj=1, conj for complex.
template <typename T>
__device__ inline T ldL(const T* A, int i, int j, int si, int sj, bool cj) {
  T v = A[(long long)i * si + (long long)j * sj];
  return cj ? conj_(v) : v;
}
template <typename T>
__device__ inline void stL(T* A, int i, int j, int si, int sj, bool cj, T v) {
  A[(long long)i * si + (long long)j * sj] = cj ? conj_(v) : v;
}

#define PB 16
// intra-wave LDS hand-off: order this wave's LDS traffic and stop the compiler
// from moving LDS accesses across the point
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
template <typename T>
__global__ __launch_bounds__(512) void k_potrf_tile(T* __restrict__ A, int n, int si, int sj, int cj,
                                                     int* __restrict__ info, int info_base) {
  extern __shared__ unsigned char smem_raw[];
  T* Ps = (T*)smem_raw;                 // n x PB panel, row-major [r][c] with stride PB+1
  __shared__ T Ds[PB][PB + 1];          // diagonal block (factored)
  __shared__ T Di[PB][PB + 1];          // inverse of diagonal block
  __shared__ int s_fail;
  const int tid = threadIdx.x;
  const bool conjf = cj != 0;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  for (int j0 = 0; j0 < n; j0 += PB) {
    const int jb = min(PB, n - j0);
    // (1) diagonal block: wave 0
    if (tid < 64) {
      const int l = tid;
      for (int e = l; e < PB * PB; e += 64) {
        const int r = e % PB, c = e / PB;
        T v = ST<T>::zero();
        if (r < jb && c < jb && r >= c) v = ldL(A, j0 + r, j0 + c, si, sj, conjf);
        Ds[r][c] = v;
      }
      // unblocked Cholesky: lane r owns row r
      for (int c = 0; c < jb; ++c) {
        wave_sync();
        typename ST<T>::real d = realv(Ds[c][c]);
        bool bad = !(d > 0);  // catches NaN
        if (bad && l == 0 && s_fail == 0) {
          s_fail = 1;
          if (info && *info == 0) *info = info_base + j0 + c + 1;
        }
        typename ST<T>::real sd = sqrt(d);
        wave_sync();
        if (l == c) Ds[c][c] = from_real<T>(sd);
        if (l > c && l < jb) Ds[l][c] = divv(Ds[l][c], from_real<T>(sd));
        wave_sync();
        if (l > c && l < jb) {
          const T lc = Ds[l][c];
          for (int k = c + 1; k <= l; ++k) Ds[l][k] = sub(Ds[l][k], mul(lc, conj_(Ds[k][c])));
        }
      }
      wave_sync();
      // inverse of the lower triangular block: lane c computes column c in LDS
      if (l < PB) {
        const int c = l;
        for (int r = 0; r < PB; ++r) {
          T s = ST<T>::zero();
          if (c < jb && r >= c && r < jb) {
            s = (r == c) ? ST<T>::one() : ST<T>::zero();
            for (int k = c; k < r; ++k) s = sub(s, mul(Ds[r][k], Di[k][c]));
            s = divv(s, Ds[r][r]);
          }
          Di[r][c] = s;
        }
      }
      wave_sync();
      for (int e = l; e < PB * PB; e += 64) {
        const int r = e % PB, c = e / PB;
        if (r < jb && c < jb && r >= c) stL(A, j0 + r, j0 + c, si, sj, conjf, Ds[r][c]);
      }
    }
    __syncthreads();
    // (2) panel: P = A[j0+jb:, j0:j0+jb] * inv(D)^H
    const int r0 = j0 + jb;
    const int np = n - r0;
    for (int r = tid; r < np; r += blockDim.x) {
      T* pr = Ps + r * (PB + 1);
      for (int c = 0; c < PB; ++c) pr[c] = (c < jb) ? ldL(A, r0 + r, j0 + c, si, sj, conjf) : ST<T>::zero();
      // in place, highest column first: P[r][c] = sum_{k<=c} a[k] conj(Di[c][k])
      for (int c = jb - 1; c >= 0; --c) {
        T s = ST<T>::zero();
        for (int k = 0; k <= c; ++k) s = fma_(pr[k], conj_(Di[c][k]), s);
        pr[c] = s;
        stL(A, r0 + r, j0 + c, si, sj, conjf, s);
      }
    }
    __syncthreads();
    // (3) trailing update (lower): A[r][s] -= sum_c P[r][c] conj(P[s][c]), r >= s
    // 4x4 register blocks; block (R, S) covers rows 4R.., cols 4S..
    const int nb4 = (np + 3) / 4;
    const long long nblk = (long long)nb4 * (nb4 + 1) / 2;
    for (long long bidx = tid; bidx < nblk; bidx += blockDim.x) {
      // invert triangular numbering: R >= S
      int R = (int)((sqrt(8.0 * (double)bidx + 1.0) - 1.0) * 0.5);
      while ((long long)R * (R + 1) / 2 > bidx) --R;
      while ((long long)(R + 1) * (R + 2) / 2 <= bidx) ++R;
      const int S = (int)(bidx - (long long)R * (R + 1) / 2);
      T acc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[i][k] = ST<T>::zero();
      for (int c = 0; c < jb; ++c) {
        T pr[4], ps[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = min(4 * R + i, np - 1), ss = min(4 * S + i, np - 1);
          pr[i] = Ps[rr * (PB + 1) + c];
          ps[i] = conj_(Ps[ss * (PB + 1) + c]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[i][k] = fma_(pr[i], ps[k], acc[i][k]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int rr = 4 * R + i, ss = 4 * S + k;
          if (rr < np && ss < np && rr >= ss) {
            T v = ldL(A, r0 + rr, r0 + ss, si, sj, conjf);
            stL(A, r0 + rr, r0 + ss, si, sj, conjf, sub(v, acc[i][k]));
          }
        }
    }
    __syncthreads();
  }
}

template <typename T>
static int potrf_launch(int uplo, int n, T* A, int lda, int* info, int info_base, hipStream_t st) {
  if (n <= 0) return 0;
  const size_t lds = (size_t)n * (PB + 1) * sizeof(T);
  if (lds > 150 * 1024) return -3;  // tile too large for the single-workgroup panel kernel
  int si, sj, cj;
  if (uplo == DPL_LOWER) { si = 1; sj = lda; cj = 0; }
  else { si = lda; sj = 1; cj = 1; }
  hipLaunchKernelGGL((k_potrf_tile<T>), dim3(1), dim3(512), lds, st, A, n, si, sj, cj, info, info_base);
  return (int)hipGetLastError();
}

DPL_API int dpl_potrf_tile(int prec, int uplo, int n, void* A, long long a_off, int lda, int* info, int info_base,
                           hipStream_t st) {
  switch (prec) {
    case DPL_S: return potrf_launch<float>(uplo, n, (float*)A + a_off, lda, info, info_base, st);
    case DPL_D: return potrf_launch<double>(uplo, n, (double*)A + a_off, lda, info, info_base, st);
    case DPL_C: return potrf_launch<hipFloatComplex>(uplo, n, (hipFloatComplex*)A + a_off, lda, info, info_base, st);
    case DPL_Z: return potrf_launch<hipDoubleComplex>(uplo, n, (hipDoubleComplex*)A + a_off, lda, info, info_base, st);
  }
  return -2;
}

// ------------------------------------------------------------------ TRSM
// Solve for a strip of VS vectors: sum_p M(q,p) X(v,p) = alpha B(v,q), M lower
// (after reversal), with
//   M(q,p)  = conj?( A[ qq*sq + pp*sp ] ),   qq = rev ? n-1-q : q (same for p)
//   B(v,q)  = B[ v*sbv + qq*sbp ]
// Items: TileItem{a_off (triangle), b_off (B tile), m, n (B extent)}.
struct TrsmParams {
  int side_left;      // vectors are columns of B (left) or rows (right)
  int sq, sp;         // M strides in A (derived from side/trans, A's lda)
  int sbv_ld;         // 1 => B strides (ldb, 1) else (1, ldb) -- see host
  int rev;            // M upper => process positions in reverse
  int cj;             // conjugate M
  int unit;           // unit diagonal
};

#define TQ 16
#define TP 64
template <typename T, int VS>
__global__ __launch_bounds__(256) void k_trsm_strip(const TileItem* __restrict__ items, int nstrips_max,
                                                    const T* __restrict__ A, int lda, T* __restrict__ B, int ldb,
                                                    T alpha, TrsmParams pr) {
  extern __shared__ unsigned char smem_raw[];
  T* Xs = (T*)smem_raw;                  // [npos][VS]
  __shared__ T Ms[TQ][TP + 1];           // chunk of M rows q-block x p-chunk
  __shared__ T Md[TQ][TQ + 1];           // diagonal block
  __shared__ T Sacc[TQ][VS + 1];         // accumulated rhs for the block, [q][v]

  const int item = blockIdx.x / nstrips_max, strip = blockIdx.x % nstrips_max;
  const TileItem it = items[item];
  const int nvec = pr.side_left ? it.n : it.m;
  const int npos = pr.side_left ? it.m : it.n;
  const int v0 = strip * VS;
  if (v0 >= nvec) return;
  const int nv = min(VS, nvec - v0);
  const T* Ab = A + it.a_off;
  T* Bb = B + it.b_off;
  // B(v, pos) address
  const long long sbv = pr.side_left ? ldb : 1, sbp = pr.side_left ? 1 : ldb;
  const bool cj = pr.cj != 0;
  const int tid = threadIdx.x;
  auto Midx = [&](int q, int p) -> T {
    const int qq = pr.rev ? npos - 1 - q : q, pp = pr.rev ? npos - 1 - p : p;
    T v = Ab[(long long)qq * pr.sq + (long long)pp * pr.sp];
    return cj ? conj_(v) : v;
  };
  auto Bptr = [&](int v, int q) -> T* {
    const int qq = pr.rev ? npos - 1 - q : q;
    return Bb + (long long)(v0 + v) * sbv + (long long)qq * sbp;
  };

  for (int q0 = 0; q0 < npos; q0 += TQ) {
    const int qb = min(TQ, npos - q0);
    // init accumulator: thread -> (v, q)
    T acc = ST<T>::zero();
    const int av = tid % VS, aq = tid / VS;  // aq in [0, 256/VS)
    const bool act = aq < TQ && av < nv && aq < qb;
    if (act) acc = mul(alpha, *Bptr(av, q0 + aq));
    // left-looking: subtract sum_{p<q0} M(q,p) X(v,p)
    for (int p0 = 0; p0 < q0; p0 += TP) {
      const int pc = min(TP, q0 - p0);
      for (int e = tid; e < TQ * TP; e += 256) {
        const int q = e % TQ, p = e / TQ;
        Ms[q][p] = (q < qb && p < pc) ? Midx(q0 + q, p0 + p) : ST<T>::zero();
      }
      __syncthreads();
      if (act) {
        for (int p = 0; p < pc; ++p) acc = sub(acc, mul(Ms[aq][p], Xs[(p0 + p) * VS + av]));
      }
      __syncthreads();
    }
    // diagonal block
    for (int e = tid; e < TQ * TQ; e += 256) {
      const int q = e % TQ, p = e / TQ;
      Md[q][p] = (q < qb && p < qb && p <= q) ? Midx(q0 + q, q0 + p) : ST<T>::zero();
    }
    if (act) Sacc[aq][av] = acc;
    __syncthreads();
    if (tid < VS && tid < nv) {
      const int v = tid;
      for (int q = 0; q < qb; ++q) {
        T s = Sacc[q][v];
        for (int p = 0; p < q; ++p) s = sub(s, mul(Md[q][p], Xs[(q0 + p) * VS + v]));
        if (!pr.unit) s = divv(s, Md[q][q]);
        Xs[(q0 + q) * VS + v] = s;
      }
    }
    __syncthreads();
  }
  // write back X
  for (int e = tid; e < npos * VS; e += 256) {
    const int v = e % VS, q = e / VS;
    if (v < nv) *Bptr(v, q) = Xs[q * VS + v];
  }
}

template <typename T>
static int trsm_launch(int side, int uplo, int trans, int diag, int nitems, const TileItem* items, int max_vec,
                       int max_pos, T alpha, const T* A, int lda, T* B, int ldb, hipStream_t st) {
  if (nitems <= 0) return 0;
  TrsmParams pr;
  pr.side_left = side == DPL_LEFT;
  const bool tr = trans != DPL_NOTRANS;
  pr.cj = trans == DPL_CONJTRANS;
  pr.unit = diag == DPL_UNIT;
  // M(q,p) = op(A)(q,p) for left, op(A)(p,q) for right
  bool m_is_opA_T;  // M(q,p) = A[p + q*lda] ?
  if (pr.side_left) m_is_opA_T = tr;   // N: A[q + p lda]; T: A[p + q lda]
  else m_is_opA_T = !tr;               // N: A[p + q lda]; T: A[q + p lda]
  if (m_is_opA_T) { pr.sq = lda; pr.sp = 1; } else { pr.sq = 1; pr.sp = lda; }
  // M lower?  M = A (if !m_is_opA_T) keeps A's uplo; transposed flips it
  const bool a_lower = uplo == DPL_LOWER;
  const bool m_lower = m_is_opA_T ? !a_lower : a_lower;
  pr.rev = m_lower ? 0 : 1;
  pr.sbv_ld = pr.side_left;
  // pick strip width so the X strip fits in 64 KB of LDS
  int vs = 16;
  while (vs > 1 && (size_t)vs * max_pos * sizeof(T) > 64 * 1024) vs >>= 1;
  if ((size_t)vs * max_pos * sizeof(T) > 64 * 1024) return -3;
  const size_t lds = (size_t)vs * max_pos * sizeof(T);
  const int ns = cdiv(max_vec, vs);
  dim3 g(nitems * ns), b(256);
  switch (vs) {
    case 16: hipLaunchKernelGGL((k_trsm_strip<T, 16>), g, b, lds, st, items, ns, A, lda, B, ldb, alpha, pr); break;
    case 8: hipLaunchKernelGGL((k_trsm_strip<T, 8>), g, b, lds, st, items, ns, A, lda, B, ldb, alpha, pr); break;
    case 4: hipLaunchKernelGGL((k_trsm_strip<T, 4>), g, b, lds, st, items, ns, A, lda, B, ldb, alpha, pr); break;
    case 2: hipLaunchKernelGGL((k_trsm_strip<T, 2>), g, b, lds, st, items, ns, A, lda, B, ldb, alpha, pr); break;
    default: hipLaunchKernelGGL((k_trsm_strip<T, 1>), g, b, lds, st, items, ns, A, lda, B, ldb, alpha, pr); break;
  }
  return (int)hipGetLastError();
}

// items: device TileItem array; max_m/max_n: largest B tile extent in the batch
DPL_API int dpl_trsm_batched(int prec, int side, int uplo, int trans, int diag, int nitems, const void* items,
                             int max_m, int max_n, const void* alpha, const void* A, int lda, void* B, int ldb,
                             hipStream_t st) {
  const int max_vec = side == DPL_LEFT ? max_n : max_m;
  const int max_pos = side == DPL_LEFT ? max_m : max_n;
  const TileItem* it = (const TileItem*)items;
  switch (prec) {
    case DPL_S: return trsm_launch<float>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const float*)alpha, (const float*)A, lda, (float*)B, ldb, st);
    case DPL_D: return trsm_launch<double>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const double*)alpha, (const double*)A, lda, (double*)B, ldb, st);
    case DPL_C: return trsm_launch<hipFloatComplex>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const hipFloatComplex*)alpha, (const hipFloatComplex*)A, lda, (hipFloatComplex*)B, ldb, st);
    case DPL_Z: return trsm_launch<hipDoubleComplex>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const hipDoubleComplex*)alpha, (const hipDoubleComplex*)A, lda, (hipDoubleComplex*)B, ldb, st);
  }
  return -2;
}
