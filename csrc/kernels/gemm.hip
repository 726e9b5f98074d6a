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
#include "gemm_tile.h"

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
// (the sub-tile body lives in gemm_tile.h, shared with the device task runtime)
template <typename T, bool TA, bool TB>
__device__ __forceinline__ void gemm_full_tile(const int wg, const GemmItemK* __restrict__ items,
                                               const KPair* __restrict__ kps, int nsm, int nsn, T alpha,
                                               const T* __restrict__ A, int lda, const T* __restrict__ B,
                                               int ldb, T beta, T* __restrict__ C, int ldc) {
  __shared__ T sm[gemm_lds_elems<T>()];
  const int per = nsm * nsn;
  const GemmItemK it = items[wg / per];
  const int sub = wg % per;
  const int m0 = (sub % nsm) * GBM, n0 = (sub / nsm) * GBN;
  if (m0 >= it.m || n0 >= it.n) return;
  const int uplo = it.flags & 3;
  if (uplo == 1 && n0 >= m0 + GBM) return;
  if (uplo == 2 && m0 >= n0 + GBN) return;
  const KPair* kp = kps + it.kt_beg;
  gemm_subtile<T, TA, TB>(sm, [kp](int t) { return kp[t]; }, it.kt_cnt, m0, n0, uplo, alpha, A, lda, B, ldb, beta,
                          C + it.c_off, ldc);
}

// One 128x128 output sub-tile per workgroup (PERSIST = false: grid = every sub-tile), or a capped
// grid that walks the sub-tiles grid-stride (PERSIST = true, dpl_gemm_set_wg_cap): a bulk update
// launched that way never holds more than the cap's workgroup slots, so latency-bound critical-path
// kernels on a high-priority stream find free CUs at once instead of queueing behind ~0.5 ms
// GEMM workgroups (profiles/r2_potrf16k_timeline.txt).  The cap is a multiple of the 8 XCDs, so a
// workgroup keeps its XCD's share of xcd_remap's tile order on every pass.
// wave-uniform copy of a value that a non-inlined call passed in VGPRs (any trivially copyable type)
template <typename V>
__device__ __forceinline__ V rfl_any(V v) {
  static_assert(sizeof(V) % 4 == 0, "32-bit words");
  unsigned w[sizeof(V) / 4];
  __builtin_memcpy(w, &v, sizeof(V));
#pragma unroll
  for (int q = 0; q < (int)(sizeof(V) / 4); ++q) w[q] = __builtin_amdgcn_readfirstlane(w[q]);
  V r;
  __builtin_memcpy(&r, w, sizeof(V));
  return r;
}

// One sub-tile of the capped (grid-stride) launch as a separate function: inlined into the
// grid-stride loop the body kept loop-invariant addressing live across iterations and spilled 63
// VGPRs to scratch (hipcc -Rpass-analysis=kernel-resource-usage), which is what made every capped
// bulk update slower than the uncapped one (profiles/r3_lu_rest_cap.txt).  Called, it is allocated on
// its own; the arguments arrive in VGPRs and are made wave-uniform again (buffer resources need SGPRs).
template <typename T, bool TA, bool TB>
__device__ __attribute__((noinline)) void gemm_full_tile_call(int wg, const GemmItemK* items, const KPair* kps,
                                                               int nsm, int nsn, T alpha, const T* A, int lda,
                                                               const T* B, int ldb, T beta, T* C, int ldc) {
  gemm_full_tile<T, TA, TB>(rfl_any(wg), rfl_any(items), rfl_any(kps), rfl_any(nsm), rfl_any(nsn), rfl_any(alpha),
                            rfl_any(A), rfl_any(lda), rfl_any(B), rfl_any(ldb), rfl_any(beta), rfl_any(C),
                            rfl_any(ldc));
}

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
    gemm_full_tile_call<T, TA, TB>(xcd_remap(b, nwg), items, kps, nsm, nsn, alpha, A, lda, B, ldb, beta, C, ldc);
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
