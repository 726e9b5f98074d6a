// Complex batched tile GEMM on the matrix cores: C_item = beta*C_item + alpha * sum_kt opA(A_kt) opB(B_kt)
// for hipDoubleComplex (v_mfma_f64_16x16x4_f64) and hipFloatComplex (v_mfma_f32_16x16x4_f32).
//
// Reference role: cublasZgemm / cublasCgemm inside the JDF CUDA bodies (src/zpotrf_L.jdf:432-471,
// src/zgemm_NN.jdf:168-199) -- z is the reference's template precision.  Same item protocol as the
// real engine (gemm.hip: GemmItemK / KPair, one launch per step of an algorithm).
//
// Design: a complex product is four real MFMA products on planar operands,
//     Cr += Ar Br - Ai Bi,   Ci += Ar Bi + Ai Br      (8 real flops per complex multiply-add,
// the LAPACK flop count of ZGEMM, so the complex rate equals the real MFMA rate).  Operands are
// staged in LDS as separate real / imaginary planes (padded row stride: the four 16-lane groups of
// a fragment read land in alternating bank halves), alpha and the conjugations are applied while
// staging A and B, and -Bi is formed once per fragment.  As in the real engine the MFMA computes
// D = opB^T opA^T, so the accumulator lanes run along C's rows (the contiguous direction of
// column-major tiles).  64x64 C sub-tile per 256-thread workgroup, 4 waves in 2x2 (32x32 each:
// 2x2 blocks x {re, im}), BK = 8 complex k per step, LDS double-buffered, XCD-aware block mapping.
#include "common.h"

struct KPairZ {
  long long a_off, b_off;
  int k;
  int pad;
};
struct GemmItemZ {
  long long c_off;
  int kt_beg, kt_cnt;
  int m, n;
  int flags;
  int pad;
};

namespace {
constexpr int ZBM = 64, ZBN = 64, ZBK = 8, ZLS = 80;  // tile, k-step, padded LDS row stride

template <typename R> struct ZT;
template <> struct ZT<double> {
  typedef hipDoubleComplex C;
  typedef d4_t acc_t;
  static __device__ inline acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) + 4 * r; }
};
template <> struct ZT<float> {
  typedef hipFloatComplex C;
  typedef f4_t acc_t;
  static __device__ inline acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) * 4 + r; }
};

template <typename R, int OPA, int OPB>
__global__ __launch_bounds__(256) void k_cgemm_mfma(const GemmItemZ* __restrict__ items,
                                                    const KPairZ* __restrict__ kps, int nsm, int nsn, int nwg,
                                                    typename ZT<R>::C alpha, const typename ZT<R>::C* __restrict__ A,
                                                    int lda, const typename ZT<R>::C* __restrict__ B, int ldb,
                                                    typename ZT<R>::C beta, typename ZT<R>::C* __restrict__ C,
                                                    int ldc) {
  typedef typename ZT<R>::C Cx;
  typedef typename ZT<R>::acc_t acc_t;
  // [buf][plane: Ar, Ai, Br, Bi][ZBK][ZLS]
  __shared__ R sm[2][4][ZBK][ZLS];

  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per = nsm * nsn;
  const GemmItemZ it = items[wg / per];
  const int sub = wg % per;
  const int m0 = (sub % nsm) * ZBM, n0 = (sub / nsm) * ZBN;
  const int Mt = it.m, Nt = it.n;
  if (m0 >= Mt || n0 >= Nt) return;
  const int uplo = it.flags & 3;
  if (uplo == 1 && n0 >= m0 + ZBM) return;
  if (uplo == 2 && m0 >= n0 + ZBN) return;
  Cx* Cb = C + it.c_off;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;

  int nsteps = 0;
  for (int t = 0; t < it.kt_cnt; ++t) nsteps += (kps[it.kt_beg + t].k + ZBK - 1) / ZBK;

  // ---- global -> registers (2 A and 2 B complex elements per thread per step)
  Cx ra[2], rb[2];
  int ld_kt = it.kt_beg, ld_k0 = 0;
  KPairZ kp;
  kp.a_off = 0; kp.b_off = 0; kp.k = 0;
  if (it.kt_cnt > 0) kp = kps[ld_kt];
  const Cx zero = ST<Cx>::zero();
  auto load = [&]() {
    const Cx* Ab = A + kp.a_off;
    const Cx* Bb = B + kp.b_off;
    const int Kt = kp.k;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + 256 * q;
      int i, kk;
      if (OPA == 0) { i = e & 63; kk = e >> 6; } else { kk = e & 7; i = e >> 3; }
      const bool ina = (m0 + i < Mt) && (ld_k0 + kk < Kt);
      const long long ia = (OPA == 0) ? (m0 + i) + (long long)(ld_k0 + kk) * lda
                                      : (ld_k0 + kk) + (long long)(m0 + i) * lda;
      ra[q] = ina ? Ab[ia] : zero;
      int j;
      if (OPB == 0) { kk = e & 7; j = e >> 3; } else { j = e & 63; kk = e >> 6; }
      const bool inb = (n0 + j < Nt) && (ld_k0 + kk < Kt);
      const long long ib = (OPB == 0) ? (ld_k0 + kk) + (long long)(n0 + j) * ldb
                                      : (n0 + j) + (long long)(ld_k0 + kk) * ldb;
      rb[q] = inb ? Bb[ib] : zero;
    }
    ld_k0 += ZBK;
    if (ld_k0 >= Kt) {
      ld_k0 = 0;
      ++ld_kt;
      if (ld_kt < it.kt_beg + it.kt_cnt) kp = kps[ld_kt];
    }
  };
  // ---- registers -> LDS planes (alpha on A, conjugation on C-ops)
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + 256 * q;
      int i, kk;
      if (OPA == 0) { i = e & 63; kk = e >> 6; } else { kk = e & 7; i = e >> 3; }
      Cx a = ra[q];
      if (OPA == 2) a = conj_(a);
      a = mul(alpha, a);
      sm[buf][0][kk][i] = realv(a);
      sm[buf][1][kk][i] = imagv(a);
      int j;
      if (OPB == 0) { kk = e & 7; j = e >> 3; } else { j = e & 63; kk = e >> 6; }
      Cx b = rb[q];
      if (OPB == 2) b = conj_(b);
      sm[buf][2][kk][j] = realv(b);
      sm[buf][3][kk][j] = imagv(b);
    }
  };

  if (nsteps > 0) load();
  const int mrow = m0 + wm * 32 + (l & 15);
  const int ncol = n0 + wn * 32;
  acc_t ar[2][2], ai[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = mrow + i * 16, nn = ncol + j * 16 + ZT<R>::drow(l, r);
        const bool in = mm < Mt && nn < Nt && !is_zero(beta);
        const Cx v = in ? mul(beta, Cb[mm + (long long)nn * ldc]) : zero;
        ar[i][j][r] = realv(v);
        ai[i][j][r] = imagv(v);
      }
  if (nsteps > 0) store(0);
  if (nsteps > 1) load();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    __syncthreads();
    if (s + 1 < nsteps) store(cur ^ 1);
    if (s + 2 < nsteps) load();
#pragma unroll
    for (int kq = 0; kq < ZBK / 4; ++kq) {
      const int kr = kq * 4 + (l >> 4);
      R fa_r[2], fa_i[2], fb_r[2], fb_i[2], fb_n[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa_r[i] = sm[cur][0][kr][wm * 32 + i * 16 + (l & 15)];
        fa_i[i] = sm[cur][1][kr][wm * 32 + i * 16 + (l & 15)];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb_r[j] = sm[cur][2][kr][wn * 32 + j * 16 + (l & 15)];
        fb_i[j] = sm[cur][3][kr][wn * 32 + j * 16 + (l & 15)];
        fb_n[j] = -fb_i[j];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          ar[i][j] = ZT<R>::mma(fb_r[j], fa_r[i], ar[i][j]);
          ai[i][j] = ZT<R>::mma(fb_i[j], fa_r[i], ai[i][j]);
          ar[i][j] = ZT<R>::mma(fb_n[j], fa_i[i], ar[i][j]);
          ai[i][j] = ZT<R>::mma(fb_r[j], fa_i[i], ai[i][j]);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = mrow + i * 16, nn = ncol + j * 16 + ZT<R>::drow(l, r);
        bool ok = mm < Mt && nn < Nt;
        if (uplo == 1) ok = ok && (mm >= nn);
        if (uplo == 2) ok = ok && (mm <= nn);
        if (ok) Cb[mm + (long long)nn * ldc] = make_sc<Cx>(ar[i][j][r], ai[i][j][r]);
      }
}

template <typename R, int OA, int OB>
void zl1(dim3 g, hipStream_t st, const GemmItemZ* items, const KPairZ* kps, int nsm, int nsn, int nwg,
         typename ZT<R>::C alpha, const typename ZT<R>::C* A, int lda, const typename ZT<R>::C* B, int ldb,
         typename ZT<R>::C beta, typename ZT<R>::C* C, int ldc) {
  hipLaunchKernelGGL((k_cgemm_mfma<R, OA, OB>), g, dim3(256), 0, st, items, kps, nsm, nsn, nwg, alpha, A, lda, B,
                     ldb, beta, C, ldc);
}

template <typename R>
int launch_cgemm(int opa, int opb, int nitems, const void* items, const void* kpairs, int max_m, int max_n,
                 const void* alpha, const void* A, int lda, const void* B, int ldb, const void* beta, void* C,
                 int ldc, hipStream_t st) {
  typedef typename ZT<R>::C Cx;
  const int nsm = cdiv(max_m, ZBM), nsn = cdiv(max_n, ZBN);
  const long long nwgl = (long long)nitems * nsm * nsn;
  if (nwgl <= 0) return 0;
  if (nwgl > 0x7fffffffLL) return -1;
  const int nwg = (int)nwgl;
  dim3 g(nwg);
  const GemmItemZ* it = (const GemmItemZ*)items;
  const KPairZ* kp = (const KPairZ*)kpairs;
  const Cx al = *(const Cx*)alpha, be = *(const Cx*)beta;
#define ZG_(a, b)                                                                                           \
  if (opa == a && opb == b)                                                                                 \
    zl1<R, a, b>(g, st, it, kp, nsm, nsn, nwg, al, (const Cx*)A, lda, (const Cx*)B, ldb, be, (Cx*)C, ldc);
  ZG_(0, 0) ZG_(0, 1) ZG_(0, 2) ZG_(1, 0) ZG_(1, 1) ZG_(1, 2) ZG_(2, 0) ZG_(2, 1) ZG_(2, 2)
#undef ZG_
  return (int)hipGetLastError();
}
}  // namespace

// prec: DPL_Z or DPL_C; op codes 0 = N, 1 = T, 2 = C (items / kpairs: the gemm.hip records)
DPL_API int dpl_cgemm_mfma(int prec, int opa, int opb, int nitems, const void* items, const void* kpairs, int max_m,
                           int max_n, const void* alpha, const void* A, int lda, const void* B, int ldb,
                           const void* beta, void* C, int ldc, hipStream_t st) {
  if (prec == DPL_Z)
    return launch_cgemm<double>(opa, opb, nitems, items, kpairs, max_m, max_n, alpha, A, lda, B, ldb, beta, C, ldc,
                                st);
  if (prec == DPL_C)
    return launch_cgemm<float>(opa, opb, nitems, items, kpairs, max_m, max_n, alpha, A, lda, B, ldb, beta, C, ldc,
                               st);
  return -2;
}
