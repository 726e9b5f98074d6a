// Full-tile MFMA GEMM body shared by the batched engine (gemm.hip: one launch per step) and the
// device task runtime (dtr.hip: one persistent launch per factorisation): one 128x128 C sub-tile
// of 256 threads, fp64 / fp32 MFMA, buffer-load operand fetches, MFMA-paced LDS pipeline.  The
// LDS image is passed in (the persistent kernel overlays it with its other task bodies) and the
// k-run comes from a source functor: ks(t) -> KPair (the engine reads its KPair array, the task
// runtime computes Cholesky operand offsets from tile indices).
#pragma once
#include "common.h"

struct KPair {
  long long a_off, b_off;
  int k;
  int pad;
};
struct GemmItemK {
  long long c_off;
  int kt_beg, kt_cnt;  // run of KPair records
  int m, n;
  int flags;           // bits 0-1: C write mask (0 full, 1 lower, 2 upper)
  int pad;
};

typedef double d2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <typename T> struct MF;
template <> struct MF<double> {
  typedef d4_t acc_t;
  typedef d2v vec_t;
  static constexpr int VEC = 2;
  static __device__ inline acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // row (within a 16x16 block, along the D "row" axis) held by lane l, register r
  static __device__ inline int drow(int l, int r) { return (l >> 4) + 4 * r; }
};
template <> struct MF<float> {
  typedef f4_t acc_t;
  typedef f4v vec_t;
  static constexpr int VEC = 4;
  static __device__ inline acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) * 4 + r; }
};

#define GBM 128
#define GBN 128
#define GBK 16

// ------------------------------------------------------------------ full-tile fast path
// Used when every item of the launch is a whole number of 128x128 sub-tiles and every k-run a
// multiple of GBK (e.g. all NB=512 Cholesky / SUMMA updates).  Differences from k_gemm_mfma:
//  * no bounds logic anywhere in the k-loop;
//  * operands are fetched with buffer loads: the per-thread byte offset is loop-invariant (VGPR),
//    the k-advance is a scalar soffset and the k-tile base lives in the SGPR resource, so the
//    loop carries no 64-bit VALU address arithmetic;
//  * alpha is applied once in the epilogue (acc starts at (beta/alpha) C), not per staged block;
//  * k-contiguous operands (A^T / B untransposed) are fetched with 16 consecutive lanes on 16
//    different rows/columns so their transposed LDS stores hit 16 distinct bank slots; all LDS
//    images use the padded stride 144 (fragment reads of rows kr / kr+1 in opposite bank halves).
#define FLS 144

__device__ inline __amdgpu_buffer_rsrc_t mk_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

template <typename T> struct BufLd;
template <> struct BufLd<double> {
  typedef d2v vec_t;
  static __device__ inline vec_t ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(vec_t, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  }
};
template <> struct BufLd<float> {
  typedef f4v vec_t;
  static __device__ inline vec_t ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(vec_t, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  }
};

// LDS image size (elements of T) of gemm_subtile
template <typename T> constexpr int gemm_lds_elems() { return 2 * 2 * GBK * FLS; }

// C sub-tile (m0, n0) of an item whose C origin is Cb: C = beta*C + alpha * sum_t opA(A_t) opB(B_t),
// ks(t) = KPair{a_off, b_off, k} for t in [0, kt_cnt), k a multiple of GBK; uplo 1 / 2 masks the
// stores to the lower / upper triangle of the item (the caller skips sub-tiles wholly outside it).
// sm: gemm_lds_elems<T>() elements of LDS.  Ends with no LDS access pending on return only after
// the caller's next __syncthreads().
template <typename T, bool TA, bool TB, typename KS>
__device__ __forceinline__ void gemm_subtile(T* __restrict__ sm, const KS& ks, const int kt_cnt, const int m0,
                                             const int n0, const int uplo, T alpha, const T* __restrict__ A,
                                             int lda, const T* __restrict__ B, int ldb, T beta,
                                             T* __restrict__ Cb, int ldc, int tid_in = -1, bool wt = false) {
  typedef MF<T> M_;
  typedef typename M_::acc_t acc_t;
  typedef typename M_::vec_t vec_t;
  constexpr int VEC = M_::VEC;
  constexpr int NLD = (GBM * GBK) / (VEC * 256);
  constexpr int KG = GBK / VEC;      // 16-byte k-groups per row of a k-contiguous operand
  constexpr int OPB_ = GBK * FLS;    // sm: [buf][operand][GBK x FLS]

  // tid_in: a persistent caller passes threadIdx.x laundered through an asm barrier each task, so the
  // per-thread address arithmetic below is recomputed per task instead of being hoisted out of the
  // task loop and kept live across it (which spilled)
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;

  int nsteps = 0;
  for (int t = 0; t < kt_cnt; ++t) nsteps += ks(t).k / GBK;

  // ---- loop-invariant per-thread fetch offset (bytes) and LDS destination of the q=0 vector;
  // the q-th vector (thread c + 256q) is a fixed stride away: scalar for the fetch, immediate in LDS
  int voa, vob, lda0, ldb0;
  {
    const int c = tid;
    if (!TA) {  // op(A)(i, k) = A[i + k*lda]: 16-byte vectors along i
      const int kk = c / (GBM / VEC), i = (c % (GBM / VEC)) * VEC;
      voa = (i + kk * lda) * (int)sizeof(T);
      lda0 = kk * FLS + i;
    } else {    // op(A)(i, k) = A[k + i*lda]: 16 consecutive lanes on 16 different i
      const int i = (c & 15) | ((c / (16 * KG)) << 4), kk = ((c >> 4) % KG) * VEC;
      voa = (kk + i * lda) * (int)sizeof(T);
      lda0 = kk * FLS + i;
    }
    if (TB) {   // op(B)(k, j) = B[j + k*ldb]
      const int kk = c / (GBN / VEC), j = (c % (GBN / VEC)) * VEC;
      vob = (j + kk * ldb) * (int)sizeof(T);
      ldb0 = kk * FLS + j;
    } else {    // op(B)(k, j) = B[k + j*ldb]
      const int j = (c & 15) | ((c / (16 * KG)) << 4), kk = ((c >> 4) % KG) * VEC;
      vob = (kk + j * ldb) * (int)sizeof(T);
      ldb0 = kk * FLS + j;
    }
  }
  constexpr int LQA = TA ? 16 * VEC : 2 * VEC * FLS;   // LDS stride between q and q+1
  constexpr int LQB = TB ? 2 * VEC * FLS : 16 * VEC;
  const int GQA = (TA ? 16 * VEC : 2 * VEC) * lda * (int)sizeof(T);  // fetch stride (bytes)
  const int GQB = (TB ? 2 * VEC : 16 * VEC) * ldb * (int)sizeof(T);
  // scalar k-position of the next fetch
  int ld_kt = 0, ld_k0 = 0, ld_K = 0;
  __amdgpu_buffer_rsrc_t ra_rs = mk_rsrc(A), rb_rs = mk_rsrc(B);
  auto set_kt = [&]() {
    const KPair kp = ks(ld_kt);
    ld_K = kp.k;
    ra_rs = mk_rsrc(A + kp.a_off + (TA ? (long long)m0 * lda : (long long)m0));
    rb_rs = mk_rsrc(B + kp.b_off + (TB ? (long long)n0 : (long long)n0 * ldb));
  };
  if (nsteps > 0) set_kt();
  vec_t ra[NLD], rb[NLD];
  // fetch(): issue the block at the current position; advance(): step it (scalar), clamped at
  // the last block so the loop can fetch unconditionally (surplus fetches are never stored)
  auto fetch = [&]() {
    const int sa = (TA ? ld_k0 : ld_k0 * lda) * (int)sizeof(T);
    const int sb = (TB ? ld_k0 * ldb : ld_k0) * (int)sizeof(T);
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      ra[q] = BufLd<T>::ld(ra_rs, voa, sa + q * GQA);
      rb[q] = BufLd<T>::ld(rb_rs, vob, sb + q * GQB);
    }
  };
  auto advance = [&]() {
    if (ld_k0 + GBK < ld_K) {
      ld_k0 += GBK;
    } else if (ld_kt + 1 < kt_cnt) {
      ++ld_kt;
      ld_k0 = 0;
      set_kt();
    }
  };
  auto load = [&]() {
    fetch();
    advance();
  };
  auto store = [&](int buf) {
    T* sa = sm + (2 * buf) * OPB_;
    T* sb = sa + OPB_;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      if (!TA) {
        *(vec_t*)&sa[lda0 + q * LQA] = ra[q];
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) sa[lda0 + q * LQA + e * FLS] = ra[q][e];
      }
      if (TB) {
        *(vec_t*)&sb[ldb0 + q * LQB] = rb[q];
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) sb[ldb0 + q * LQB + e * FLS] = rb[q][e];
      }
    }
  };
  auto frag = [&](int buf, int kq, T* a, T* b) {
    const T* sa = sm + (2 * buf) * OPB_;
    const T* sb = sa + OPB_;
    const int kr = kq * 4 + (l >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = sa[kr * FLS + wm * 64 + i * 16 + (l & 15)];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = sb[kr * FLS + wn * 64 + j * 16 + (l & 15)];
  };

  if (nsteps > 0) load();
  // ---- C prologue: acc = (beta/alpha) C, finished by one multiply with alpha in the epilogue
  const int mrow = m0 + wm * 64 + (l & 15);
  const int ncol = n0 + wn * 64;
  T* cp = Cb + mrow + (long long)ncol * ldc;
  acc_t acc[4][4];
  if (beta == T(0)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = T(0);
  } else {
    const T bs = beta / alpha;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = cp[i * 16 + (long long)(j * 16 + M_::drow(l, r)) * ldc];
    // consume the C values here so the waitcnt pass drains them before the loop (vmcnt is a counter)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] *= bs;
  }
  if (nsteps > 0) store(0);
  if (nsteps > 1) load();
  // One basic block per k-step: barrier, then the step's 64 MFMAs/wave with the LDS writes of
  // block s+1, the buffer fetches of block s+2 and the fragment reads of quads 1..3 interleaved
  // one memory instruction per MFMA (sched_group_barrier), then the scalar advance.
  constexpr int NW = (TA ? NLD * VEC : NLD) + (TB ? NLD : NLD * VEC);  // LDS stores per step
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    __syncthreads();
    T a[3][4], b[3][4];
    frag(cur, 0, a[0], b[0]);
    store(cur ^ 1);
    frag(cur, 1, a[1], b[1]);
    fetch();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = M_::mma(b[0][j], a[0][i], acc[i][j]);
    frag(cur, 2, a[2], b[2]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = M_::mma(b[1][j], a[1][i], acc[i][j]);
    frag(cur, 3, a[0], b[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = M_::mma(b[2][j], a[2][i], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = M_::mma(b[0][j], a[0][i], acc[i][j]);
    // schedule: [quad-0 reads] then MFMA-paced: NW stores, 4 reads (q1), 2*NLD fetches,
    // pad to 24, 4 reads (q2), pad to 40, 4 reads (q3), rest
    constexpr int M1 = NW + 4 + 2 * NLD;            // MFMAs paced by stores / q1 reads / fetches
    constexpr int P1 = M1 < 24 ? 24 - M1 : 0;
    constexpr int M2 = M1 + P1 + 4;
    constexpr int P2 = M2 < 40 ? 40 - M2 : 0;
    constexpr int M3 = M2 + P2 + 4;
    static_assert(M3 < 64, "schedule overflows the step's MFMAs");
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int v = 0; v < 2 * NLD; ++v) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    if (P1 > 0) __builtin_amdgcn_sched_group_barrier(0x008, P1, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if (P2 > 0) __builtin_amdgcn_sched_group_barrier(0x008, P2, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 64 - M3, 0);
    advance();
  }

  const bool diag = (uplo == 1 && n0 + GBN > m0) || (uplo == 2 && m0 + GBM > n0);
  if (wt) {
    // write-through to memory (system scope) -- a measurement knob of the device task runtime
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = mrow + i * 16, nn = ncol + j * 16 + M_::drow(l, r);
          const bool ok = !diag || ((uplo == 1) ? (mm >= nn) : (mm <= nn));
          if (ok) __hip_atomic_store(Cb + mm + (long long)nn * ldc, alpha * acc[i][j][r], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
        }
  } else if (!diag) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cp[i * 16 + (long long)(j * 16 + M_::drow(l, r)) * ldc] = alpha * acc[i][j][r];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = mrow + i * 16, nn = ncol + j * 16 + M_::drow(l, r);
          const bool ok = (uplo == 1) ? (mm >= nn) : (mm <= nn);
          if (ok) Cb[mm + (long long)nn * ldc] = alpha * acc[i][j][r];
        }
  }
}

