// Triangular tile kernels: POTRF of one diagonal tile and batched TRSM strips.
//
// Reference roles:
//   * POTRF tile  — cusolverDnZpotrf in src/zpotrf_L.jdf:118-146 (CUDA body) and
//                   CORE_zpotrf -> LAPACKE_zpotrf_work (src/cores/core_zpotrf.c:68-74);
//                   info convention *INFO = k*mb + iinfo (src/zpotrf_L.jdf:180-182).
//   * TRSM tile   — cublasZtrsm_v2 in src/zpotrf_L.jdf:221-243 and CORE_ztrsm
//                   (src/cores/core_ztrsm.c:80); all 8 side/uplo/trans variants.
//
// Design (CDNA4).  Both kernels are LEFT-LOOKING over 16-wide column blocks so
// the only global traffic is streaming reads of already-final data (no
// read-modify-write of a trailing matrix), and both are built on one primitive,
// a 16x16 block product  acc(i,j) += sum_p X(i,p) * Y(j,p)  which for fp64 is a
// chain of v_mfma_f64_16x16x4_f64 (two accumulators to cover the dependent
// MFMA latency) and for other precisions a register-blocked VALU loop.
//
//   POTRF (one 256-thread workgroup per tile: a latency-critical panel task):
//   for each 16-column block J the 4 waves compute the updated block column
//   P = A(J:, J) - L(J:, 0:J) L(J, 0:J)^H (the L(J, 0:J) row strip is staged in
//   LDS once per J, the L(J:, 0:J) operand streams from L2), wave 0 factors the
//   16x16 diagonal block and inverts it in LDS, all waves apply inv(D)^H to the
//   rest of the block column, and the block column is written back once.
//   TRSM (one workgroup per (tile, strip of 16 independent vectors)): the strip
//   of X stays in LDS for the whole solve; for each 16-position block the 4
//   waves split the left-looking contraction over p and reduce through LDS; the
//   16x16 diagonal solve is a parallel product with the PRECOMPUTED inverse of
//   that diagonal block (k_diag_inv16, one small launch per batch), so no lane
//   ever runs a sequential substitution.  Every side/uplo/trans/diag variant
//   reduces to "lower-triangular M, forward order" through strides and an index
//   reversal, so one kernel template serves all eight.
#include "common.h"

__device__ inline float shfl_t(float v, int src) { return __shfl(v, src, 64); }
__device__ inline double shfl_t(double v, int src) { return __shfl(v, src, 64); }
__device__ inline hipFloatComplex shfl_t(hipFloatComplex v, int src) {
  return make_hipFloatComplex(__shfl(v.x, src, 64), __shfl(v.y, src, 64));
}
__device__ inline hipDoubleComplex shfl_t(hipDoubleComplex v, int src) {
  return make_hipDoubleComplex(__shfl(v.x, src, 64), __shfl(v.y, src, 64));
}

// ------------------------------------------------------------------ 16x16 block-product engine
// acc(i,j) += sum_{p0<=p<p1} X(i,p) * Y(j,p); X/Y are functors returning T.
// Lane l owns 4 results: (brow(l, r), bcol(l, r)), r = 0..3.
template <typename T> struct Blk16 {
  T v[4];
  __device__ inline void zero() {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ST<T>::zero();
  }
  static __device__ inline int brow(int l, int r) { return (l & 15); }
  static __device__ inline int bcol(int l, int r) { return (l >> 4) * 4 + r; }
  template <class FX, class FY>
  __device__ inline void add(const FX& X, const FY& Y, int p0, int p1) {
    const int l = lane_id();
    const int i = l & 15, jb = (l >> 4) * 4;
    for (int p = p0; p < p1; ++p) {
      const T x = X(i, p);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fma_(x, Y(jb + r, p), v[r]);
    }
  }
  __device__ inline T get(int r) const { return v[r]; }
  __device__ inline void set(int r, T x) { v[r] = x; }
  // this = P * D^H where P is held in `src` (this layout) and D in LDS (16x17)
  __device__ inline void mul_regs(const Blk16<T>& src, const T (*D)[17], int jb) {
    // generic path: go through LDS-free shuffles of the row: each lane needs P[i][k] for
    // all k; lanes with the same i hold k = (l>>4)*4 + r.  Use __shfl over the 4 lane groups.
    const int l = lane_id();
    const int i = l & 15, cb = (l >> 4) * 4;
    T pr[16];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) pr[g * 4 + r] = shfl_t(src.v[r], i + 16 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = cb + r;
      T s = ST<T>::zero();
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k <= c) s = fma_(pr[k], conj_(D[c][k]), s);
      v[r] = s;
    }
  }
};
template <> struct Blk16<double> {
  d4_t a0, a1;
  __device__ inline void zero() {
    a0 = d4_t{0, 0, 0, 0};
    a1 = d4_t{0, 0, 0, 0};
  }
  // v_mfma_f64_16x16x4_f64 D layout: col = l&15, row = (l>>4) + 4r.  X goes in
  // the B operand and Y in the A operand, so lane l holds i = l&15, j = (l>>4)+4r.
  static __device__ inline int brow(int l, int r) { return (l & 15); }
  static __device__ inline int bcol(int l, int r) { return (l >> 4) + 4 * r; }
  template <class FX, class FY>
  __device__ inline void add(const FX& X, const FY& Y, int p0, int p1) {
    const int l = lane_id();
    const int li = l & 15, lk = l >> 4;
    int p = p0;
    for (; p + 16 <= p1; p += 16) {  // 8 loads in flight, two accumulation chains
      double x[4], y[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x[u] = X(li, p + 4 * u + lk);
        y[u] = Y(li, p + 4 * u + lk);
      }
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[0], x[0], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[1], x[1], a1, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[2], x[2], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[3], x[3], a1, 0, 0, 0);
    }
    for (; p < p1; p += 4) {
      const bool ok = p + lk < p1;
      const double x0 = ok ? X(li, p + lk) : 0.0, y0 = ok ? Y(li, p + lk) : 0.0;
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y0, x0, a0, 0, 0, 0);
    }
  }
  __device__ inline double get(int r) const { return a0[r] + a1[r]; }
  __device__ inline void set(int r, double x) {
    a0[r] = x;
    a1[r] = 0.0;
  }
  // this = P * D^H with P in `src`: the D layout of src (lane i = l&15 holds
  // P[i][(l>>4) + 4r]) is exactly the B-operand layout of k-step r, so 4 MFMAs.
  __device__ inline void mul_regs(const Blk16<double>& src, const double (*D)[17], int jb) {
    const int l = lane_id(), li = l & 15, lk = l >> 4;
    zero();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double y = D[li][4 * r + lk];  // Y(c = li, p = 4r + lk) = conj(Dinv[c][p]) (real)
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, src.get(r), a0, 0, 0, 0);
    }
  }
};

// intra-wave LDS hand-off: a wave's LDS operations retire in order, so waiting
// for its own LDS counter plus a compiler memory barrier is enough (a
// seq_cst workgroup fence here measured ~1500 cycles per call on gfx950).
__device__ inline void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// One wave: Cholesky of the 16x16 Hermitian block whose lower part is in
// Ds[r][c] (LDS), factor L back into Ds, inverse of L into Di.  All 64 lanes
// work: lane owns 4 elements (row l&15, cols (l>>4)*4 .. +3) of the trailing
// update at every step, so each of the 16 steps is a handful of broadcast LDS
// reads + 4 FMAs.  Returns the first failing column + 1 (0 = success).
template <typename T>
__device__ int chol16_inv(T (*Ds)[17], T (*Di)[17], int jb) {
  const int l = lane_id();
  // column-per-lane right-looking Cholesky: lane j (< 16) holds column j in registers
  __shared__ T Lc[16];
  T col[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) col[k] = (l < jb && k >= l && k < jb) ? Ds[k][l] : ST<T>::zero();
  bool bad = false;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c < jb) {
      if (l == c) {  // finalize column c from this lane's registers
        const typename ST<T>::real d = realv(col[c]);
        bad = !(d > 0);
        const typename ST<T>::real sd = sqrt(d);
        const T inv = from_real<T>(1 / sd);
        col[c] = from_real<T>(sd);
#pragma unroll
        for (int k = c + 1; k < 16; ++k) col[k] = mul(col[k], inv);
#pragma unroll
        for (int k = c; k < 16; ++k) Lc[k] = col[k];
      }
      wave_sync();
      if (l > c && l < jb) {  // update column l with column c
        const T ljc = conj_(Lc[l]);
#pragma unroll
        for (int k = c + 1; k < 16; ++k)
          if (k >= l) col[k] = sub(col[k], mul(Lc[k], ljc));
      }
      wave_sync();
    }
  }
  if (l < 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) Ds[k][l] = (l < jb && k >= l && k < jb) ? col[k] : ST<T>::zero();
  }
  const unsigned long long bm = __ballot(bad ? 1 : 0);
  const int bad_col = bm ? (__ffsll((long long)bm)) : 0;  // first failing column + 1
  wave_sync();
  // inverse: lane j (< 16) computes column j of inv(L) by forward substitution,
  // fully unrolled (static register indices); the L values are wave-uniform
  // broadcast LDS reads that do not depend on x, so they are all in flight.
  if (l < 16) {
    T x[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      T s = (rr == l) ? ST<T>::one() : ST<T>::zero();
#pragma unroll
      for (int k = 0; k < rr; ++k) s = sub(s, mul(Ds[rr][k], x[k]));
      x[rr] = (rr < jb) ? divv(s, Ds[rr][rr]) : ST<T>::zero();
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) Di[rr][l] = (l < jb) ? x[rr] : ST<T>::zero();
  }
  wave_sync();
  return bad_col;
}

// ------------------------------------------------------------------ POTRF
#define PT 512         // threads (8 waves)
#define PRB 5          // max row blocks per worker wave (1 + 7*PRB >= 32 for n <= 512)
static int g_phase_mask = 0xff;  // debug/tuning: skip phases of the panel kernel
DPL_API void dpl_debug_set_phase_mask(int m) { g_phase_mask = m; }

// acc[b] += sum_p X(b, i, p) * Y(j, p) for the wave's row blocks b < nb (shared Y):
// for fp64 all row blocks advance together so 4 + 4*nb loads are in flight per 16 k.
template <typename T, class FX, class FY>
__device__ inline void add_rows(Blk16<T>* acc, int nb, const FX& X, const FY& Y, int p0, int p1) {
#pragma unroll
  for (int b = 0; b < PRB; ++b)
    if (b < nb) {
      auto Xb = [&](int i, int p) -> T { return X(b, i, p); };
      acc[b].add(Xb, Y, p0, p1);
    }
}
template <class FX, class FY>
__device__ inline void add_rows(Blk16<double>* acc, int nb, const FX& X, const FY& Y, int p0, int p1) {
  const int l = lane_id(), li = l & 15, lk = l >> 4;
  int p = p0;
  for (; p + 16 <= p1; p += 16) {
    double y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) y[u] = Y(li, p + 4 * u + lk);
    double x[PRB][4];
#pragma unroll
    for (int b = 0; b < PRB; ++b)
#pragma unroll
      for (int u = 0; u < 4; ++u) x[b][u] = (b < nb) ? X(b, li, p + 4 * u + lk) : 0.0;
#pragma unroll
    for (int b = 0; b < PRB; ++b)
      if (b < nb) {
        acc[b].a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[0], x[b][0], acc[b].a0, 0, 0, 0);
        acc[b].a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[1], x[b][1], acc[b].a1, 0, 0, 0);
        acc[b].a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[2], x[b][2], acc[b].a0, 0, 0, 0);
        acc[b].a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y[3], x[b][3], acc[b].a1, 0, 0, 0);
      }
  }
  for (; p < p1; p += 4) {
    const bool ok = p + lk < p1;
    const double y0 = ok ? Y(li, p + lk) : 0.0;
#pragma unroll
    for (int b = 0; b < PRB; ++b)
      if (b < nb) {
        const double x0 = ok ? X(b, li, p + lk) : 0.0;
        acc[b].a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(y0, x0, acc[b].a0, 0, 0, 0);
      }
  }
}

// Left-looking blocked Cholesky of one n x n tile (n <= 512), one workgroup.
// Per 16-column block J (3 barriers):
//   A. wave 0: P0 = A(J,J) - L(J,0:J) L(J,0:J)^H, then factor + invert it (LDS);
//      waves 1..7: P_b = A(Ib,J) - L(Ib,0:J) L(J,0:J)^H for their row blocks Ib
//      (accumulators stay in registers);
//   C. every worker multiplies its P_b by inv(D)^H straight from the accumulator
//      registers (the f64 MFMA D layout is the B-operand layout of the next
//      product) and stores the final L block rows to global; wave 0 stores L(J,J);
//   S. stage conj(L(J+1, 0:J+1)) (the shared Y operand of the next step) in LDS.
template <typename T, bool STAGE_Y>
__global__ __launch_bounds__(PT) void k_potrf_ll(T* __restrict__ A, int n, int si, int sj, int cj,
                                                 int* __restrict__ info, int info_base, int pmask) {
  extern __shared__ unsigned char smem_raw[];
  T* Ys = (T*)smem_raw;  // [n][16]: conj(L(j0 + c, p)) at p*16 + c
  __shared__ T Ds[16][17];
  __shared__ T Di[16][17];
  __shared__ int s_fail;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const bool conjf = cj != 0;
  auto LD = [&](int i, int j) -> T {
    T v = A[(long long)i * si + (long long)j * sj];
    return conjf ? conj_(v) : v;
  };
  auto STO = [&](int i, int j, T v) { A[(long long)i * si + (long long)j * sj] = conjf ? conj_(v) : v; };
  if (tid == 0) s_fail = 0;
  __syncthreads();
  for (int j0 = 0; j0 < n; j0 += 16) {
    const int jb = min(16, n - j0), np = n - j0, nrb = (np + 15) / 16;
    auto Ystage = [&](int c, int p) -> T { return Ys[p * 16 + c]; };
    auto Yglob = [&](int c, int p) -> T { return (c < jb) ? conj_(LD(j0 + c, p)) : ST<T>::zero(); };
    // ---------------- A
    Blk16<T> acc[PRB];
    int nmy = 0;  // number of row blocks of this wave (workers)
    if (w == 0) {
      Blk16<T> a0;
      a0.zero();
      if (j0 > 0 && (pmask & 2)) {
        // rows past the last (partial) column block are outside the tile: never read them
        auto X = [&](int b, int i, int p) -> T { return (i < jb) ? LD(j0 + i, p) : ST<T>::zero(); };
        if (STAGE_Y) add_rows<T>(&a0, 1, X, Ystage, 0, j0);
        else add_rows<T>(&a0, 1, X, Yglob, 0, j0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = Blk16<T>::brow(l, r), c = Blk16<T>::bcol(l, r);
        Ds[i][c] = (i < jb && c < jb && i >= c) ? sub(LD(j0 + i, j0 + c), a0.get(r)) : ST<T>::zero();
      }
      if (pmask & 4) {
        const int bad = chol16_inv<T>(Ds, Di, jb);
        if (l == 0 && bad && s_fail == 0) {
          s_fail = 1;
          if (info && *info == 0) *info = info_base + j0 + bad;
        }
      }
      // store L(J, J) (lower part)
      for (int e = l; e < 256; e += 64) {
        const int c = e >> 4, i = e & 15;
        if (i < jb && c < jb && i >= c) STO(j0 + i, j0 + c, Ds[i][c]);
      }
    } else {
#pragma unroll
      for (int b = 0; b < PRB; ++b) {
        acc[b].zero();
        if (1 + (w - 1) + 7 * b < nrb) nmy = b + 1;
      }
      if (j0 > 0 && (pmask & 2) && nmy > 0) {
        auto X = [&](int b, int i, int p) -> T {
          const int row = j0 + 16 * (1 + (w - 1) + 7 * b) + i;
          return (row < n) ? LD(row, p) : ST<T>::zero();
        };
        if (STAGE_Y) add_rows<T>(acc, nmy, X, Ystage, 0, j0);
        else add_rows<T>(acc, nmy, X, Yglob, 0, j0);
      }
      // P_b = A(Ib, J) - acc  (in registers, MFMA layout)
#pragma unroll
      for (int b = 0; b < PRB; ++b)
        if (b < nmy) {
          const int r0 = j0 + 16 * (1 + (w - 1) + 7 * b);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = Blk16<T>::brow(l, r), c = Blk16<T>::bcol(l, r);
            const T a = (r0 + i < n && c < jb) ? LD(r0 + i, j0 + c) : ST<T>::zero();
            acc[b].set(r, sub(a, acc[b].get(r)));
          }
        }
    }
    __syncthreads();
    // ---------------- C: L(Ib, J) = P_b inv(D)^H
    if (w > 0 && (pmask & 8)) {
#pragma unroll
      for (int b = 0; b < PRB; ++b)
        if (b < nmy) {
          const int r0 = j0 + 16 * (1 + (w - 1) + 7 * b);
          Blk16<T> out;
          out.mul_regs(acc[b], Di, jb);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = Blk16<T>::brow(l, r), c = Blk16<T>::bcol(l, r);
            if (r0 + i < n && c < jb) STO(r0 + i, j0 + c, out.get(r));
          }
        }
    }
    __syncthreads();
    // ---------------- S: stage the next Y operand
    const int j1 = j0 + 16;
    if (STAGE_Y && j1 < n && (pmask & 1)) {
      const int jb1 = min(16, n - j1);
      for (int e = tid; e < j1 * 16; e += PT) {
        const int c = e & 15, p = e >> 4;
        Ys[e] = (c < jb1) ? conj_(LD(j1 + c, p)) : ST<T>::zero();
      }
    }
    __syncthreads();
  }
}

template <typename T>
static int potrf_launch(int uplo, int n, T* A, int lda, int* info, int info_base, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > 16 * (1 + 7 * PRB)) return -3;  // at most PRB row blocks per worker wave
  const bool stage = true;
  const size_t lds = (size_t)n * 16 * sizeof(T);
  if (lds > 150 * 1024) return -3;  // tile too large for the single-workgroup panel kernel
  int si, sj, cj;
  if (uplo == DPL_LOWER) { si = 1; sj = lda; cj = 0; }
  else { si = lda; sj = 1; cj = 1; }
  if (stage)
    hipLaunchKernelGGL((k_potrf_ll<T, true>), dim3(1), dim3(PT), lds, st, A, n, si, sj, cj, info, info_base,
                       g_phase_mask);
  else
    hipLaunchKernelGGL((k_potrf_ll<T, false>), dim3(1), dim3(PT), lds, st, A, n, si, sj, cj, info, info_base,
                       g_phase_mask);
  return (int)hipGetLastError();
}

// fp64 tiles with n <= 512 go to the multi-workgroup dataflow kernel (potrf_rb.hip) unless
// dpl_potrf_tile_set_kind(1) selects the single-workgroup kernel (ablation / comparison).
DPL_API int dpl_potrf_tile_rb(int uplo, int n, double* A, int lda, int* info, int info_base, hipStream_t st);
static int g_potrf_kind = 0;
DPL_API int dpl_potrf_tile_set_kind(int kind) {
  const int old = g_potrf_kind;
  g_potrf_kind = kind;
  return old;
}

DPL_API int dpl_potrf_tile(int prec, int uplo, int n, void* A, long long a_off, int lda, int* info, int info_base,
                           hipStream_t st) {
  switch (prec) {
    case DPL_S: return potrf_launch<float>(uplo, n, (float*)A + a_off, lda, info, info_base, st);
    case DPL_D:
      if (g_potrf_kind == 0 && n <= 512)
        return dpl_potrf_tile_rb(uplo, n, (double*)A + a_off, lda, info, info_base, st);
      return potrf_launch<double>(uplo, n, (double*)A + a_off, lda, info, info_base, st);
    case DPL_C: return potrf_launch<hipFloatComplex>(uplo, n, (hipFloatComplex*)A + a_off, lda, info, info_base, st);
    case DPL_Z: return potrf_launch<hipDoubleComplex>(uplo, n, (hipDoubleComplex*)A + a_off, lda, info, info_base, st);
  }
  return -2;
}

// ------------------------------------------------------------------ TRSM
// Solve for a strip of 16 vectors: sum_p M(q,p) X(v,p) = alpha B(v,q), M lower
// (after reversal), with
//   M(q,p)  = conj?( A[ qq*sq + pp*sp ] ),   qq = rev ? n-1-q : q (same for p)
//   B(v,q)  = B[ v*sbv + qq*sbp ]
struct TrsmParams {
  int side_left;  // vectors are columns of B (left) or rows (right)
  int sq, sp;     // M strides in A
  int rev;        // M upper => process positions in reverse
  int cj;         // conjugate M
  int unit;       // unit diagonal
};

// invd[t][J][q][q'] = inverse of M's 16x16 diagonal block J of triangle t (row-major)
template <typename T>
__global__ __launch_bounds__(64) void k_diag_inv16(const long long* __restrict__ tri_off, int npos, int nJ,
                                                   const T* __restrict__ A, TrsmParams pr, T* __restrict__ invd) {
  __shared__ T Mb[16][17];
  __shared__ T Xi[16][17];
  const int t = blockIdx.x / nJ, J = blockIdx.x % nJ;
  const T* Ab = A + tri_off[t];
  const int l = threadIdx.x;
  const int q0 = J * 16, qb = min(16, npos - q0);
  for (int e = l; e < 256; e += 64) {
    const int q = e >> 4, p = e & 15;
    T v = ST<T>::zero();
    if (q < qb && p <= q) {
      const int qq = pr.rev ? npos - 1 - (q0 + q) : q0 + q, pp = pr.rev ? npos - 1 - (q0 + p) : q0 + p;
      v = Ab[(long long)qq * pr.sq + (long long)pp * pr.sp];
      if (pr.cj) v = conj_(v);
      if (pr.unit && p == q) v = ST<T>::one();
    }
    Mb[q][p] = v;
  }
  wave_sync();
  if (l < 16) {
    const int c = l;  // column of the inverse, fully unrolled forward substitution
    T x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      T acc = (r == c) ? ST<T>::one() : ST<T>::zero();
#pragma unroll
      for (int k = 0; k < r; ++k) acc = sub(acc, mul(Mb[r][k], x[k]));
      x[r] = (r < qb) ? divv(acc, Mb[r][r]) : ST<T>::zero();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) Xi[r][c] = (c < qb) ? x[r] : ST<T>::zero();
  }
  wave_sync();
  T* out = invd + ((size_t)t * nJ + J) * 256;
  for (int e = l; e < 256; e += 64) out[e] = Xi[e >> 4][e & 15];
}

template <typename T, bool STAGE_M>
__global__ __launch_bounds__(256) void k_trsm_strip(const TileItem* __restrict__ items, int nstrips_max,
                                                    const T* __restrict__ A, int lda, T* __restrict__ B, int ldb,
                                                    T alpha, TrsmParams pr, const T* __restrict__ invd, int nJ,
                                                    int npos_max) {
  extern __shared__ unsigned char smem_raw[];
  T* Xs = (T*)smem_raw;                 // [npos][16]  X(v, p) at p*16 + v
  T* Msm = Xs + (size_t)npos_max * 16;  // [npos][16]  M(q0 + j, p) at p*16 + j (STAGE_M)
  __shared__ T Red[4][16][17];          // per-wave partial sums, [wave][q][v]
  __shared__ T Ss[16][17];              // rhs of the current block, [q][v]

  const int item = blockIdx.x / nstrips_max, strip = blockIdx.x % nstrips_max;
  const TileItem it = items[item];
  const int nvec = pr.side_left ? it.n : it.m;
  const int npos = pr.side_left ? it.m : it.n;
  const int v0 = strip * 16;
  if (v0 >= nvec) return;
  const int nv = min(16, nvec - v0);
  const T* Ab = A + it.a_off;
  T* Bb = B + it.b_off;
  const T* invt = invd + (size_t)it.gi * nJ * 256;  // triangle index travels in gi
  const long long sbv = pr.side_left ? ldb : 1, sbp = pr.side_left ? 1 : ldb;
  const bool cj = pr.cj != 0;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  auto Mv = [&](int q, int p) -> T {
    const int qq = pr.rev ? npos - 1 - q : q, pp = pr.rev ? npos - 1 - p : p;
    T v = Ab[(long long)qq * pr.sq + (long long)pp * pr.sp];
    return cj ? conj_(v) : v;
  };
  auto Bptr = [&](int v, int q) -> T* {
    const int qq = pr.rev ? npos - 1 - q : q;
    return Bb + (long long)(v0 + v) * sbv + (long long)qq * sbp;
  };
  const int av = tid & 15, aq = tid >> 4;  // (v, q) owned in the combine step

  for (int q0 = 0; q0 < npos; q0 += 16) {
    const int qb = min(16, npos - q0);
    // (1) partial contractions: wave w takes p-chunks [16c, 16c+16) with c % 4 == w
    Blk16<T> acc;
    acc.zero();
    if (STAGE_M) {
      // stage the block row M(q0 : q0+16, 0 : q0) in LDS with all 256 threads
      // (coalesced along q for the common sq == 1 layouts, 32+ loads in flight per thread)
      for (int e = tid; e < q0 * 16; e += 256) {
        const int j = e & 15, p = e >> 4;
        Msm[e] = (j < qb) ? Mv(q0 + j, p) : ST<T>::zero();
      }
      __syncthreads();
      auto X = [&](int i, int p) -> T { return Xs[p * 16 + i]; };   // i = v
      auto Y = [&](int j, int p) -> T { return Msm[p * 16 + j]; };  // j = q
      for (int c0 = w * 16; c0 < q0; c0 += 64) acc.add(X, Y, c0, min(c0 + 16, q0));
    } else {
      auto X = [&](int i, int p) -> T { return Xs[p * 16 + i]; };                          // i = v
      auto Y = [&](int j, int p) -> T { return (j < qb) ? Mv(q0 + j, p) : ST<T>::zero(); };  // j = q
      for (int c0 = w * 16; c0 < q0; c0 += 64) acc.add(X, Y, c0, min(c0 + 16, q0));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Red[w][Blk16<T>::bcol(l, r)][Blk16<T>::brow(l, r)] = acc.get(r);
    __syncthreads();
    // (2) rhs: S(q, v) = alpha B(v, q) - sum_w Red[w][q][v]
    {
      T s = ST<T>::zero();
      if (aq < qb && av < nv) s = mul(alpha, *Bptr(av, q0 + aq));
      s = sub(s, add(add(Red[0][aq][av], Red[1][aq][av]), add(Red[2][aq][av], Red[3][aq][av])));
      Ss[aq][av] = s;
    }
    __syncthreads();
    // (3) X(v, q0+q) = sum_{q'} invD[q][q'] S(q', v)
    {
      const T* inv = invt + (size_t)(q0 / 16) * 256;
      T x = ST<T>::zero();
#pragma unroll
      for (int k = 0; k < 16; ++k) x = fma_(inv[aq * 16 + k], Ss[k][av], x);
      if (aq < qb) Xs[(q0 + aq) * 16 + av] = (av < nv) ? x : ST<T>::zero();
    }
    __syncthreads();
  }
  // write back X
  for (int e = tid; e < npos * 16; e += 256) {
    const int v = e & 15, q = e >> 4;
    if (v < nv) *Bptr(v, q) = Xs[q * 16 + v];
  }
}

template <typename T>
static int trsm_launch(int side, int uplo, int trans, int diag, int nitems, const TileItem* items, int max_vec,
                       int max_pos, T alpha, const T* A, int lda, T* B, int ldb, int ntri, const long long* tri_off,
                       T* work, hipStream_t st) {
  if (nitems <= 0) return 0;
  TrsmParams pr;
  pr.side_left = side == DPL_LEFT;
  const bool tr = trans != DPL_NOTRANS;
  pr.cj = trans == DPL_CONJTRANS;
  pr.unit = diag == DPL_UNIT;
  // M(q,p) = op(A)(q,p) for left, op(A)(p,q) for right
  bool m_is_opA_T;  // M(q,p) = A[p + q*lda] ?
  if (pr.side_left) m_is_opA_T = tr;
  else m_is_opA_T = !tr;
  if (m_is_opA_T) { pr.sq = lda; pr.sp = 1; } else { pr.sq = 1; pr.sp = lda; }
  const bool a_lower = uplo == DPL_LOWER;
  const bool m_lower = m_is_opA_T ? !a_lower : a_lower;
  pr.rev = m_lower ? 0 : 1;
  const size_t xs = (size_t)16 * max_pos * sizeof(T);
  // staging M per 16-row strip re-streams the whole triangle per workgroup and
  // drops occupancy to 1 WG/CU; measured slower, so only for small triangles
  const bool stage = max_pos <= 128 && 2 * xs <= 64 * 1024;
  const size_t lds = stage ? 2 * xs : xs;
  if (lds > 128 * 1024) return -3;
  const int nJ = cdiv(max_pos, 16);
  hipLaunchKernelGGL((k_diag_inv16<T>), dim3(ntri * nJ), dim3(64), 0, st, tri_off, max_pos, nJ, A, pr, work);
  const int ns = cdiv(max_vec, 16);
  if (stage)
    hipLaunchKernelGGL((k_trsm_strip<T, true>), dim3(nitems * ns), dim3(256), lds, st, items, ns, A, lda, B, ldb,
                       alpha, pr, (const T*)work, nJ, max_pos);
  else
    hipLaunchKernelGGL((k_trsm_strip<T, false>), dim3(nitems * ns), dim3(256), lds, st, items, ns, A, lda, B, ldb,
                       alpha, pr, (const T*)work, nJ, max_pos);
  return (int)hipGetLastError();
}

// items: device TileItem array (gi = triangle index into tri_off); every item of
// a batch has the same triangle order (max_pos); tri_off: device int64[ntri];
// work: device scratch of ntri * ceil(order/16) * 256 elements.
DPL_API int dpl_trsm_batched(int prec, int side, int uplo, int trans, int diag, int nitems, const void* items,
                             int max_m, int max_n, const void* alpha, const void* A, int lda, void* B, int ldb,
                             int ntri, const void* tri_off, void* work, hipStream_t st) {
  const int max_vec = side == DPL_LEFT ? max_n : max_m;
  const int max_pos = side == DPL_LEFT ? max_m : max_n;
  const TileItem* it = (const TileItem*)items;
  const long long* to = (const long long*)tri_off;
  switch (prec) {
    case DPL_S: return trsm_launch<float>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const float*)alpha, (const float*)A, lda, (float*)B, ldb, ntri, to, (float*)work, st);
    case DPL_D: return trsm_launch<double>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const double*)alpha, (const double*)A, lda, (double*)B, ldb, ntri, to, (double*)work, st);
    case DPL_C: return trsm_launch<hipFloatComplex>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const hipFloatComplex*)alpha, (const hipFloatComplex*)A, lda, (hipFloatComplex*)B, ldb, ntri, to, (hipFloatComplex*)work, st);
    case DPL_Z: return trsm_launch<hipDoubleComplex>(side, uplo, trans, diag, nitems, it, max_vec, max_pos, *(const hipDoubleComplex*)alpha, (const hipDoubleComplex*)A, lda, (hipDoubleComplex*)B, ldb, ntri, to, (hipDoubleComplex*)work, st);
  }
  return -2;
}
