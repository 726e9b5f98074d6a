// Batched tile GEMM engine: C_item = beta*C_item + alpha * sum_kt opA(A_kt) * opB(B_kt)
//
// This is the flop engine of every dplasma_amd algorithm (the role cublasZgemm
// plays inside the reference's JDF CUDA bodies, e.g. src/zpotrf_L.jdf:432-471,
// src/zgemm_NN_summa.jdf:209-242, src/zgetrf_nopiv.jdf:198-235).  Instead of one
// vendor call per tile, one launch covers every output tile of a step:
//
//   * each GemmItem names one C tile and a run of KPair records (the k-tiles to
//     contract), so a whole local SUMMA/GEMM, or one Cholesky trailing update,
//     is a single launch;
//   * f64 uses v_mfma_f64_16x16x4_f64, f32 uses v_mfma_f32_16x16x4_f32:
//     256-thread workgroups, 128x128 C sub-tile per workgroup, 4 waves in 2x2,
//     64x64 per wave = 4x4 MFMA blocks, BK=16 k-steps double-buffered in LDS
//     (row stride 144 elements => conflict-free ds_read_b64 halves);
//   * operand roles are swapped inside the MFMA (D = opB^T * opA^T) so the
//     accumulator's lane index runs along C's rows, i.e. along the contiguous
//     direction of column-major tiles: epilogue stores are 128-B segments;
//   * accumulators are initialised with beta*C (C is read once, up front, its
//     latency overlapping the first operand loads) and alpha is folded into the
//     A staging, so the epilogue is a pure store;
//   * blockIdx is remapped XCD-aware so the 16 sub-tiles of a 512x512 tile and
//     neighbouring tiles of a tile-row share one XCD's L2.
// Complex precisions run on the matrix cores too (zgemm.hip, four real MFMA products per complex one).
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

// LDS image of one operand block: [GBK][row-stride] per buffer.
//  f64: no padding, column index XOR-swizzled by ((kk >> 1) & 7) << 2.  Fragment reads (16
//       consecutive columns of row kr + the same of row kr+1 per 32 lanes) stay a permutation
//       of whole 16-column groups in opposite bank halves, and the transposed stores of a
//       k-contiguous operand (8 lanes = rows 0,2,..,14 of one column) land on 8 distinct
//       bank pairs -- conflict-free both ways (padding alone cannot do both for b64).
//  f32: padded row stride 144, no swizzle.
template <typename T> struct LdsL {
  static constexpr int LS = 144;
  static __device__ inline int at(int kk, int col) { return kk * LS + col; }
};
template <> struct LdsL<double> {
  static constexpr int LS = 128;
  static __device__ inline int at(int kk, int col) { return kk * LS + (col ^ (((kk >> 1) & 7) << 2)); }
};

template <typename T, bool TA, bool TB>
__global__ __launch_bounds__(256, 2) void k_gemm_mfma(const GemmItemK* __restrict__ items,
                                                      const KPair* __restrict__ kps, int nsm, int nsn,
                                                      int nwg, T alpha, const T* __restrict__ A, int lda,
                                                      const T* __restrict__ B, int ldb, T beta,
                                                      T* __restrict__ C, int ldc, int vec_ok) {
  typedef MF<T> M_;
  typedef typename M_::acc_t acc_t;
  typedef typename M_::vec_t vec_t;
  constexpr int VEC = M_::VEC;
  constexpr int NLD = (GBM * GBK) / (VEC * 256);  // 16-byte loads per thread per operand per k-step
  typedef LdsL<T> L_;
  constexpr int OPB_ = GBK * L_::LS;  // one operand image
  __shared__ T sm[2 * 2 * OPB_];      // [buf][operand][GBK x LS]

  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per = nsm * nsn;
  const GemmItemK it = items[wg / per];
  const int sub = wg % per;
  const int m0 = (sub % nsm) * GBM, n0 = (sub / nsm) * GBN;
  const int Mt = it.m, Nt = it.n;
  if (m0 >= Mt || n0 >= Nt) return;
  const int uplo = it.flags & 3;
  if (uplo == 1 && n0 >= m0 + GBM) return;
  if (uplo == 2 && m0 >= n0 + GBN) return;

  T* Cb = C + it.c_off;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const bool fullmn = vec_ok && (m0 + GBM <= Mt) && (n0 + GBN <= Nt);

  // flatten the (k-tile, k-block) iteration space
  int nsteps = 0;
  for (int t = 0; t < it.kt_cnt; ++t) nsteps += (kps[it.kt_beg + t].k + GBK - 1) / GBK;

  vec_t ra[NLD], rb[NLD];
  int ld_kt = it.kt_beg, ld_k0 = 0;  // position of the next load
  KPair kp;
  kp.a_off = 0; kp.b_off = 0; kp.k = 0;
  if (it.kt_cnt > 0) kp = kps[ld_kt];

  auto load = [&](void) {
    const T* Ab = A + kp.a_off;
    const T* Bb = B + kp.b_off;
    const int Kt = kp.k;
    const bool fk = fullmn && (ld_k0 + GBK <= Kt);
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q;
      // ---- A: op(A)(i, k), i in [0,128), k in [0,16)
      if (!TA) {
        const int kk = c / (GBM / VEC), i = (c % (GBM / VEC)) * VEC;
        const T* src = Ab + (m0 + i) + (long long)(ld_k0 + kk) * lda;
        if (fk) {
          ra[q] = *(const vec_t*)src;
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e)
            ra[q][e] = (m0 + i + e < Mt && ld_k0 + kk < Kt) ? src[e] : T(0);
        }
      } else {
        const int i = c / (GBK / VEC), kk = (c % (GBK / VEC)) * VEC;
        const T* src = Ab + (ld_k0 + kk) + (long long)(m0 + i) * lda;
        if (fk) {
          ra[q] = *(const vec_t*)src;
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e)
            ra[q][e] = (m0 + i < Mt && ld_k0 + kk + e < Kt) ? src[e] : T(0);
        }
      }
      // ---- B: op(B)(k, j)
      if (TB) {
        const int kk = c / (GBN / VEC), j = (c % (GBN / VEC)) * VEC;
        const T* src = Bb + (n0 + j) + (long long)(ld_k0 + kk) * ldb;
        if (fk) {
          rb[q] = *(const vec_t*)src;
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e)
            rb[q][e] = (n0 + j + e < Nt && ld_k0 + kk < Kt) ? src[e] : T(0);
        }
      } else {
        const int j = c / (GBK / VEC), kk = (c % (GBK / VEC)) * VEC;
        const T* src = Bb + (ld_k0 + kk) + (long long)(n0 + j) * ldb;
        if (fk) {
          rb[q] = *(const vec_t*)src;
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e)
            rb[q][e] = (n0 + j < Nt && ld_k0 + kk + e < Kt) ? src[e] : T(0);
        }
      }
    }
    // advance
    ld_k0 += GBK;
    if (ld_k0 >= Kt) {
      ld_k0 = 0;
      ++ld_kt;
      if (ld_kt < it.kt_beg + it.kt_cnt) kp = kps[ld_kt];
    }
  };
  auto store = [&](int buf) {
    T* sa = sm + (2 * buf) * OPB_;
    T* sb = sa + OPB_;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q;
      if (!TA) {
        const int kk = c / (GBM / VEC), i = (c % (GBM / VEC)) * VEC;
        vec_t v = ra[q] * alpha;
        *(vec_t*)&sa[L_::at(kk, i)] = v;
      } else {
        const int i = c / (GBK / VEC), kk = (c % (GBK / VEC)) * VEC;
#pragma unroll
        for (int e = 0; e < VEC; ++e) sa[L_::at(kk + e, i)] = ra[q][e] * alpha;
      }
      if (TB) {
        const int kk = c / (GBN / VEC), j = (c % (GBN / VEC)) * VEC;
        *(vec_t*)&sb[L_::at(kk, j)] = rb[q];
      } else {
        const int j = c / (GBK / VEC), kk = (c % (GBK / VEC)) * VEC;
#pragma unroll
        for (int e = 0; e < VEC; ++e) sb[L_::at(kk + e, j)] = rb[q][e];
      }
    }
  };
  // MFMA fragments of k-quad kq: a[i] = op(A)(wm*64 + i*16 + l%16, kq*4 + l/16), b[j] likewise
  auto frag = [&](int buf, int kq, T* a, T* b) {
    const T* sa = sm + (2 * buf) * OPB_;
    const T* sb = sa + OPB_;
    const int kr = kq * 4 + (l >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = sa[L_::at(kr, wm * 64 + i * 16 + (l & 15))];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = sb[L_::at(kr, wn * 64 + j * 16 + (l & 15))];
  };

  // first operand block in flight before the C prologue so both latencies overlap
  if (nsteps > 0) load();
  // C sub-tile origin of this lane: row mrow + i*16, columns ncol + j*16 + drow(l, r)
  const int mrow = m0 + wm * 64 + (l & 15);
  const int ncol = n0 + wn * 64;
  const bool fullc = (m0 + GBM <= Mt) && (n0 + GBN <= Nt);
  acc_t acc[4][4];
  if (beta == T(0)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = T(0);
  } else if (fullc) {
    // interior sub-tile: 64 independent loads in flight, one wait (the first MFMA's)
    const T* cp = Cb + mrow + (long long)ncol * ldc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[i][j][r] = cp[i * 16 + (long long)(j * 16 + M_::drow(l, r)) * ldc];
    // always scale (even by 1): consuming the C values here makes the waitcnt pass drain
    // them before the main loop; left pending, they are carried into the loop and every
    // iteration's MFMAs wait on the freshly issued prefetch (vmcnt is a plain counter)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] *= beta;
  } else {
    // ragged edge: clamp the address, select the value (no per-element branches)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = mrow + i * 16, nn = ncol + j * 16 + M_::drow(l, r);
          const bool in = mm < Mt && nn < Nt;
          const T v = Cb[(in ? mm : 0) + (long long)(in ? nn : 0) * ldc];
          acc[i][j][r] = in ? beta * v : T(0);
        }
  }

  if (nsteps > 0) store(0);
  if (nsteps > 1) load();
  // Pipeline (per k-step s): barrier -> fragments of quad 0 -> write block s+1 (loaded during
  // step s-1) into the other buffer -> issue the global loads of block s+2 -> 16 MFMAs per
  // quad with the next quad's fragments in flight.  The LDS writes and the global loads both
  // hide behind the step's 64 MFMAs/wave instead of sitting between the MFMAs and the barrier.
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    __syncthreads();
    T a[2][4], b[2][4];
    frag(cur, 0, a[0], b[0]);
    if (s + 1 < nsteps) store(cur ^ 1);
    if (s + 2 < nsteps) load();
#pragma unroll
    for (int kq = 0; kq < GBK / 4; ++kq) {
      if (kq + 1 < GBK / 4) frag(cur, kq + 1, a[(kq + 1) & 1], b[(kq + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = M_::mma(b[kq & 1][j], a[kq & 1][i], acc[i][j]);
    }
  }

  // epilogue: interior sub-tiles off the diagonal store unconditionally
  const bool diag = (uplo == 1 && n0 + GBN > m0) || (uplo == 2 && m0 + GBM > n0);
  if (fullc && !diag) {
    T* cp = Cb + mrow + (long long)ncol * ldc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cp[i * 16 + (long long)(j * 16 + M_::drow(l, r)) * ldc] = acc[i][j][r];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = mrow + i * 16, nn = ncol + j * 16 + M_::drow(l, r);
          bool ok = mm < Mt && nn < Nt;
          if (uplo == 1) ok = ok && (mm >= nn);
          if (uplo == 2) ok = ok && (mm <= nn);
          if (ok) Cb[mm + (long long)nn * ldc] = acc[i][j][r];
        }
  }
}

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

template <typename T, bool TA, bool TB>
__device__ __forceinline__ void gemm_full_tile(const int wg, const GemmItemK* __restrict__ items,
                                               const KPair* __restrict__ kps, int nsm, int nsn, T alpha,
                                               const T* __restrict__ A, int lda, const T* __restrict__ B,
                                               int ldb, T beta, T* __restrict__ C, int ldc) {
  typedef MF<T> M_;
  typedef typename M_::acc_t acc_t;
  typedef typename M_::vec_t vec_t;
  constexpr int VEC = M_::VEC;
  constexpr int NLD = (GBM * GBK) / (VEC * 256);
  constexpr int KG = GBK / VEC;      // 16-byte k-groups per row of a k-contiguous operand
  constexpr int OPB_ = GBK * FLS;
  __shared__ T sm[2 * 2 * OPB_];     // [buf][operand][GBK x FLS]

  const int per = nsm * nsn;
  const GemmItemK it = items[wg / per];
  const int sub = wg % per;
  const int m0 = (sub % nsm) * GBM, n0 = (sub / nsm) * GBN;
  const int Mt = it.m, Nt = it.n;
  if (m0 >= Mt || n0 >= Nt) return;
  const int uplo = it.flags & 3;
  if (uplo == 1 && n0 >= m0 + GBM) return;
  if (uplo == 2 && m0 >= n0 + GBN) return;

  T* Cb = C + it.c_off;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;

  int nsteps = 0;
  for (int t = 0; t < it.kt_cnt; ++t) nsteps += kps[it.kt_beg + t].k / GBK;

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
  int ld_kt = it.kt_beg, ld_k0 = 0, ld_K = 0;
  __amdgpu_buffer_rsrc_t ra_rs = mk_rsrc(A), rb_rs = mk_rsrc(B);
  auto set_kt = [&]() {
    const KPair kp = kps[ld_kt];
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
    } else if (ld_kt + 1 < it.kt_beg + it.kt_cnt) {
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
  if (!diag) {
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

// One 128x128 output sub-tile per workgroup (PERSIST = false: grid = every sub-tile), or a capped
// grid that walks the sub-tiles grid-stride (PERSIST = true, dpl_gemm_set_wg_cap): a bulk update
// launched that way never holds more than the cap's workgroup slots, so latency-bound critical-path
// kernels on a high-priority stream find free CUs at once instead of queueing behind ~0.5 ms
// GEMM workgroups (profiles/r2_potrf16k_timeline.txt).  The cap is a multiple of the 8 XCDs, so a
// workgroup keeps its XCD's share of xcd_remap's tile order on every pass.
template <typename T, bool TA, bool TB, bool PERSIST>
__global__ __launch_bounds__(256, 2) void k_gemm_full(const GemmItemK* __restrict__ items,
                                                      const KPair* __restrict__ kps, int nsm, int nsn,
                                                      int nwg, T alpha, const T* __restrict__ A, int lda,
                                                      const T* __restrict__ B, int ldb, T beta,
                                                      T* __restrict__ C, int ldc) {
  if (!PERSIST) {
    gemm_full_tile<T, TA, TB>(xcd_remap(blockIdx.x, nwg), items, kps, nsm, nsn, alpha, A, lda, B, ldb, beta, C,
                              ldc);
    return;
  }
  for (int b = blockIdx.x; b < nwg; b += gridDim.x) {
    gemm_full_tile<T, TA, TB>(xcd_remap(b, nwg), items, kps, nsm, nsn, alpha, A, lda, B, ldb, beta, C, ldc);
    __syncthreads();   // the next sub-tile's first LDS stores must not overtake this one's last reads
  }
}

// ------------------------------------------------------------------ generic
// 64x64 C tile per 256-thread workgroup, 4x4 outputs per thread, BK=16.
// OPA/OPB: 0 = N, 1 = T, 2 = C (conjugate transpose).
template <typename T, int OPA, int OPB>
__global__ __launch_bounds__(256) void k_gemm_generic(const GemmItemK* __restrict__ items,
                                                      const KPair* __restrict__ kps, int nsm, int nsn,
                                                      int nwg, T alpha, const T* __restrict__ A, int lda,
                                                      const T* __restrict__ B, int ldb, T beta,
                                                      T* __restrict__ C, int ldc) {
  constexpr int BM = 64, BN = 64, BK = 16;
  __shared__ T As[BK][BM + 1];
  __shared__ T Bs[BK][BN + 1];
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per = nsm * nsn;
  const GemmItemK it = items[wg / per];
  const int sub = wg % per;
  const int m0 = (sub % nsm) * BM, n0 = (sub / nsm) * BN;
  const int Mt = it.m, Nt = it.n;
  if (m0 >= Mt || n0 >= Nt) return;
  const int uplo = it.flags & 3;
  if (uplo == 1 && n0 >= m0 + BM) return;
  if (uplo == 2 && m0 >= n0 + BN) return;
  T* Cb = C + it.c_off;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  T acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ST<T>::zero();

  for (int t = 0; t < it.kt_cnt; ++t) {
    const KPair kp = kps[it.kt_beg + t];
    const T* Ab = A + kp.a_off;
    const T* Bb = B + kp.b_off;
    for (int k0 = 0; k0 < kp.k; k0 += BK) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = tid + 256 * q;
        int i, kk;
        if (OPA == 0) { i = e & 63; kk = e >> 6; } else { kk = e & 15; i = e >> 4; }
        T v = ST<T>::zero();
        if (m0 + i < Mt && k0 + kk < kp.k) {
          v = (OPA == 0) ? Ab[(m0 + i) + (long long)(k0 + kk) * lda]
                         : Ab[(k0 + kk) + (long long)(m0 + i) * lda];
          if (OPA == 2) v = conj_(v);
        }
        As[kk][i] = mul(alpha, v);
        int j;
        if (OPB == 0) { kk = e & 15; j = e >> 4; } else { j = e & 63; kk = e >> 6; }
        T u = ST<T>::zero();
        if (n0 + j < Nt && k0 + kk < kp.k) {
          u = (OPB == 0) ? Bb[(k0 + kk) + (long long)(n0 + j) * ldb]
                         : Bb[(n0 + j) + (long long)(k0 + kk) * ldb];
          if (OPB == 2) u = conj_(u);
        }
        Bs[kk][j] = u;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) {
        T a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = As[kk][tx + 16 * i];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = Bs[kk][ty + 16 * j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fma_(a[i], b[j], acc[i][j]);
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mm = m0 + tx + 16 * i, nn = n0 + ty + 16 * j;
      bool ok = mm < Mt && nn < Nt;
      if (uplo == 1) ok = ok && (mm >= nn);
      if (uplo == 2) ok = ok && (mm <= nn);
      if (ok) {
        T* p = Cb + mm + (long long)nn * ldc;
        T v = acc[i][j];
        if (!is_zero(beta)) v = add(v, mul(beta, *p));
        *p = v;
      }
    }
}

// ------------------------------------------------------------------ launchers
static inline int op_code(int trans) { return trans == DPL_NOTRANS ? 0 : (trans == DPL_TRANS ? 1 : 2); }

// Workgroup cap of the next full-tile MFMA launches (0 = none): set around a bulk trailing update
// by the host program that wants CUs kept free for its critical path.  Host-thread state, like the
// current stream: the task programs issue from one thread.
static int g_gemm_wg_cap = 0;
DPL_API int dpl_gemm_set_wg_cap(int cap) {
  const int old = g_gemm_wg_cap;
  g_gemm_wg_cap = cap > 0 ? (cap / 8) * 8 : 0;
  if (cap > 0 && g_gemm_wg_cap == 0) g_gemm_wg_cap = 8;
  return old;
}

template <typename T>
static int launch_mfma(int opa, int opb, int nitems, const GemmItemK* items, const KPair* kps, int max_m,
                       int max_n, T alpha, const T* A, int lda, const T* B, int ldb, T beta, T* C, int ldc,
                       int vec_ok, hipStream_t st) {
  // vec_ok bit 1: every item is whole 128x128 sub-tiles with k-runs multiple of GBK (host-checked)
  // (32-bit buffer offsets: the furthest fetch is < (GBM + GBK) leading dimensions away)
  const bool full = (vec_ok & 2) && (vec_ok & 1) && alpha != T(0) &&
                    (long long)(GBM + GBK) * (lda > ldb ? lda : ldb) * (long long)sizeof(T) < (1LL << 30);
  vec_ok &= 1;
  const int nsm = cdiv(max_m, GBM), nsn = cdiv(max_n, GBN);
  const long long nwgl = (long long)nitems * nsm * nsn;
  if (nwgl <= 0) return 0;
  if (nwgl > 0x7fffffffLL) return -1;
  const int nwg = (int)nwgl;
  dim3 g(nwg), b(256);
  const bool ta = opa != 0, tb = opb != 0;
  if (full) {
    const int cap = g_gemm_wg_cap;
    if (cap > 0 && nwg > cap) {
      g = dim3(cap);
      if (!ta && !tb) hipLaunchKernelGGL((k_gemm_full<T, false, false, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
      else if (!ta && tb) hipLaunchKernelGGL((k_gemm_full<T, false, true, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
      else if (ta && !tb) hipLaunchKernelGGL((k_gemm_full<T, true, false, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
      else hipLaunchKernelGGL((k_gemm_full<T, true, true, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
      return (int)hipGetLastError();
    }
    if (!ta && !tb) hipLaunchKernelGGL((k_gemm_full<T, false, false, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
    else if (!ta && tb) hipLaunchKernelGGL((k_gemm_full<T, false, true, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
    else if (ta && !tb) hipLaunchKernelGGL((k_gemm_full<T, true, false, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
    else hipLaunchKernelGGL((k_gemm_full<T, true, true, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
    return (int)hipGetLastError();
  }
  if (!ta && !tb) hipLaunchKernelGGL((k_gemm_mfma<T, false, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc, vec_ok);
  else if (!ta && tb) hipLaunchKernelGGL((k_gemm_mfma<T, false, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc, vec_ok);
  else if (ta && !tb) hipLaunchKernelGGL((k_gemm_mfma<T, true, false>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc, vec_ok);
  else hipLaunchKernelGGL((k_gemm_mfma<T, true, true>), g, b, 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc, vec_ok);
  return (int)hipGetLastError();
}

template <typename T, int OA, int OB>
static void lg1(dim3 g, hipStream_t st, const GemmItemK* items, const KPair* kps, int nsm, int nsn, int nwg,
                T alpha, const T* A, int lda, const T* B, int ldb, T beta, T* C, int ldc) {
  hipLaunchKernelGGL((k_gemm_generic<T, OA, OB>), g, dim3(256), 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B,
                     ldb, beta, C, ldc);
}

template <typename T>
static int launch_generic(int opa, int opb, int nitems, const GemmItemK* items, const KPair* kps, int max_m,
                          int max_n, T alpha, const T* A, int lda, const T* B, int ldb, T beta, T* C, int ldc,
                          hipStream_t st) {
  const int nsm = cdiv(max_m, 64), nsn = cdiv(max_n, 64);
  const long long nwgl = (long long)nitems * nsm * nsn;
  if (nwgl <= 0) return 0;
  if (nwgl > 0x7fffffffLL) return -1;
  const int nwg = (int)nwgl;
  dim3 g(nwg);
#define G_(a, b) \
  if (opa == a && opb == b) lg1<T, a, b>(g, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B, ldb, beta, C, ldc);
  G_(0, 0) G_(0, 1) G_(0, 2) G_(1, 0) G_(1, 1) G_(1, 2) G_(2, 0) G_(2, 1) G_(2, 2)
#undef G_
  return (int)hipGetLastError();
}

// complex precisions on the matrix cores (zgemm.hip)
DPL_API int dpl_cgemm_mfma(int prec, int opa, int opb, int nitems, const void* items, const void* kpairs, int max_m,
                           int max_n, const void* alpha, const void* A, int lda, const void* B, int ldb,
                           const void* beta, void* C, int ldc, hipStream_t st);

// alpha/beta: host pointers to one scalar of the launch precision (complex = 2 reals)
// force_generic: route every precision through the FMA kernel (testing / A-B).
DPL_API int dpl_gemm_batched(int prec, int transA, int transB, int nitems, const void* items, const void* kpairs,
                             int max_m, int max_n, const void* alpha, const void* A, int lda, const void* B,
                             int ldb, const void* beta, void* C, int ldc, int vec_ok, int force_generic,
                             hipStream_t st) {
  const int oa = op_code(transA), ob = op_code(transB);
  const GemmItemK* it = (const GemmItemK*)items;
  const KPair* kp = (const KPair*)kpairs;
  switch (prec) {
    case DPL_D:
      if (!force_generic)
        return launch_mfma<double>(oa, ob, nitems, it, kp, max_m, max_n, *(const double*)alpha, (const double*)A,
                                   lda, (const double*)B, ldb, *(const double*)beta, (double*)C, ldc, vec_ok, st);
      return launch_generic<double>(oa, ob, nitems, it, kp, max_m, max_n, *(const double*)alpha, (const double*)A,
                                    lda, (const double*)B, ldb, *(const double*)beta, (double*)C, ldc, st);
    case DPL_S:
      if (!force_generic)
        return launch_mfma<float>(oa, ob, nitems, it, kp, max_m, max_n, *(const float*)alpha, (const float*)A, lda,
                                  (const float*)B, ldb, *(const float*)beta, (float*)C, ldc, vec_ok, st);
      return launch_generic<float>(oa, ob, nitems, it, kp, max_m, max_n, *(const float*)alpha, (const float*)A, lda,
                                   (const float*)B, ldb, *(const float*)beta, (float*)C, ldc, st);
    case DPL_C:
      if (!force_generic)
        return dpl_cgemm_mfma(prec, oa, ob, nitems, items, kpairs, max_m, max_n, alpha, A, lda, B, ldb, beta, C, ldc,
                              st);
      return launch_generic<hipFloatComplex>(oa, ob, nitems, it, kp, max_m, max_n,
                                             *(const hipFloatComplex*)alpha, (const hipFloatComplex*)A, lda,
                                             (const hipFloatComplex*)B, ldb, *(const hipFloatComplex*)beta,
                                             (hipFloatComplex*)C, ldc, st);
    case DPL_Z:
      if (!force_generic)
        return dpl_cgemm_mfma(prec, oa, ob, nitems, items, kpairs, max_m, max_n, alpha, A, lda, B, ldb, beta, C, ldc,
                              st);
      return launch_generic<hipDoubleComplex>(oa, ob, nitems, it, kp, max_m, max_n,
                                              *(const hipDoubleComplex*)alpha, (const hipDoubleComplex*)A, lda,
                                              (const hipDoubleComplex*)B, ldb, *(const hipDoubleComplex*)beta,
                                              (hipDoubleComplex*)C, ldc, st);
  }
  return -2;
}
