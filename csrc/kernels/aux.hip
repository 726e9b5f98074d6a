// Element-wise / map kernels on batched tile items: matrix generators
// (plrnt/plghe/plgsy), laset, lacpy, geadd/tradd, lascal, and per-tile norm
// partials (max, column sums, row sums, scaled sum of squares).
//
// Reference roles: CORE_zplrnt/zplghe/zplgsy (src/cores/core_zplrnt.c:68-91,
// core_zplghe.c:72-154), CORE_zlaset/zlacpy/zgeadd/ztradd, the map2/apply
// taskpools (src/map2.jdf:31-123, src/zplrnt_wrapper.c:111), and the tile norm
// kernels CORE_zlange/zlansy/zlantr/zgessq (src/cores/core_zlange.c:72 ...).
//
// The generators reproduce the reference's 64-bit LCG with O(log n) skip-ahead
// (src/cores/random.h:20-41) bit for bit: every element's value depends only on
// its GLOBAL (row, col) and the seed, so a matrix generated on any P x Q grid,
// any tile size, on GPU or CPU, is identical (SURVEY.md §2.4 "RNG").
#include <algorithm>

#include "common.h"

#define RND64_A 6364136223846793005ULL
#define RND64_C 1ULL
#define RNDF_MUL 5.4210108624275222e-20f

__device__ inline unsigned long long rnd64_jump(unsigned long long n, unsigned long long seed) {
  unsigned long long a_k = RND64_A, c_k = RND64_C, ran = seed;
  for (; n; n >>= 1) {
    if (n & 1) ran = a_k * ran + c_k;
    c_k *= (a_k + 1);
    a_k *= a_k;
  }
  return ran;
}
// the reference computes "0.5f - ran * RndF_Mul" in float arithmetic
__device__ inline float rnd_val(unsigned long long ran) { return 0.5f - (float)ran * RNDF_MUL; }

template <typename T> struct IsCplx { static constexpr bool v = false; };
template <> struct IsCplx<hipFloatComplex> { static constexpr bool v = true; };
template <> struct IsCplx<hipDoubleComplex> { static constexpr bool v = true; };

template <typename T> __device__ inline T mk(float re, float im);
template <> __device__ inline float mk<float>(float re, float) { return re; }
template <> __device__ inline double mk<double>(float re, float) { return (double)re; }
template <> __device__ inline hipFloatComplex mk<hipFloatComplex>(float re, float im) { return make_hipFloatComplex(re, im); }
template <> __device__ inline hipDoubleComplex mk<hipDoubleComplex>(float re, float im) { return make_hipDoubleComplex((double)re, (double)im); }

// value of the random matrix at global (I, J) for the plrnt stream
template <typename T>
__device__ inline T rnd_at(long long I, long long J, long long gM, unsigned long long seed) {
  const unsigned long long nbe = IsCplx<T>::v ? 2ULL : 1ULL;
  unsigned long long ran = rnd64_jump(nbe * (unsigned long long)(I + J * gM), seed);
  float re = rnd_val(ran), im = 0.f;
  if (IsCplx<T>::v) {
    ran = RND64_A * ran + RND64_C;
    im = rnd_val(ran);
  }
  return mk<T>(re, im);
}

// gen kind: 0 plrnt, 1 plghe (Hermitian, real diag + bump), 2 plgsy (symmetric, diag + bump)
// Each thread produces a run of SEG consecutive rows of one column with the
// sequential LCG (one skip-ahead per run).
#define SEG 16
template <typename T>
__device__ inline void k_generate_one(long long gid, const TileItem* __restrict__ items, int nitems, int nseg_max,
                                                  int nmax, T* A, int lda, long long gM, unsigned long long seed,
                                                  int kind, T bump) {
  const int per_item = nseg_max * nmax;
  if (gid >= (long long)nitems * per_item) return;  // tail of the last block
  const int item = (int)(gid / per_item);
  const int r = (int)(gid % per_item);
  const int seg = r % nseg_max, j = r / nseg_max;
  const TileItem it = items[item];
  if (j >= it.n || seg * SEG >= it.m) return;
  T* col = A + it.a_off + (long long)j * lda;
  const long long J = it.gj + j;
  const unsigned long long nbe = IsCplx<T>::v ? 2ULL : 1ULL;
  const int i0 = seg * SEG, i1 = min(it.m, i0 + SEG);
  // runs in the strictly-lower (or any, for plrnt) part follow the column LCG
  bool have = false;
  unsigned long long ran = 0;
  for (int i = i0; i < i1; ++i) {
    const long long I = it.gi + i;
    T v;
    if (kind == 0 || I > J) {
      if (!have) {
        ran = rnd64_jump(nbe * (unsigned long long)(I + J * gM), seed);
        have = true;
      }
      float re = rnd_val(ran), im = 0.f;
      ran = RND64_A * ran + RND64_C;
      if (IsCplx<T>::v) {
        im = rnd_val(ran);
        ran = RND64_A * ran + RND64_C;
      }
      v = mk<T>(re, im);
    } else if (I == J) {
      T d = rnd_at<T>(I, J, gM, seed);
      if (kind == 1) v = from_real<T>(realv(d) + realv(bump));
      else v = add(d, bump);
      have = false;
    } else {  // upper: mirror of (J, I)
      T d = rnd_at<T>(J, I, gM, seed);
      v = (kind == 1) ? conj_(d) : d;
      have = false;
    }
    col[i] = v;
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_generate(const TileItem* __restrict__ items, int nitems, int nseg_max,
                                                  int nmax, T* A, int lda, long long gM, unsigned long long seed,
                                                  int kind, T bump) {
  // grid-stride: a launch covers at most 2^28 work-items (HSA grid sizes are 32-bit)
  const long long stride = (long long)gridDim.x * 256;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x;; gid += stride) {
    if (gid >= (long long)nitems * nseg_max * nmax) return;
    k_generate_one<T>(gid, items, nitems, nseg_max, nmax, A, lda, gM, seed, kind, bump);
  }
}

// ---------------------------------------------------------------- laset / lacpy / geadd / lascal
// part: 0 full, 1 lower incl diag, 2 upper incl diag, 3 strictly lower,
// 4 strictly upper, 5 diagonal only (global coordinates)
__device__ inline bool in_part(int part, long long I, long long J) {
  switch (part) {
    case 0: return true;
    case 1: return I >= J;
    case 2: return I <= J;
    case 3: return I > J;
    case 4: return I < J;
    default: return I == J;
  }
}
template <typename T>
__device__ inline void k_laset_one(long long gid, const TileItem* __restrict__ items, int nitems, int mmax, int nmax, T* A, int lda,
                                               int part, T alpha, T beta) {
  const int per = mmax * nmax;
  if (gid >= (long long)nitems * per) return;  // tail of the last block
  const int item = (int)(gid / per), r = (int)(gid % per);
  const int i = r % mmax, j = r / mmax;
  const TileItem it = items[item];
  if (i >= it.m || j >= it.n) return;
  const long long I = it.gi + i, J = it.gj + j;
  if (!in_part(part, I, J)) return;
  A[it.a_off + i + (long long)j * lda] = (I == J) ? beta : alpha;
}
template <typename T>
__global__ __launch_bounds__(256) void k_laset(const TileItem* __restrict__ items, int nitems, int mmax, int nmax, T* A, int lda,
                                               int part, T alpha, T beta) {
  // grid-stride: a launch covers at most 2^28 work-items (HSA grid sizes are 32-bit)
  const long long stride = (long long)gridDim.x * 256;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x;; gid += stride) {
    if (gid >= (long long)nitems * mmax * nmax) return;
    k_laset_one<T>(gid, items, nitems, mmax, nmax, A, lda, part, alpha, beta);
  }
}
// B = alpha * op(A) + beta * B on the part; trans: 0 N, 1 T, 2 C (A item tile is op-sized source)
template <typename T>
__device__ inline void k_geadd_one(long long gid, const TileItem* __restrict__ items, int nitems, int mmax, int nmax, const T* A,
                                               int lda, T* B, int ldb, int part, int trans, T alpha, T beta,
                                               int copy) {
  const int per = mmax * nmax;
  if (gid >= (long long)nitems * per) return;  // tail of the last block
  const int item = (int)(gid / per), r = (int)(gid % per);
  const int i = r % mmax, j = r / mmax;
  const TileItem it = items[item];
  if (i >= it.m || j >= it.n) return;
  const long long I = it.gi + i, J = it.gj + j;
  if (!in_part(part, I, J)) return;
  T a = (trans == 0) ? A[it.a_off + i + (long long)j * lda] : A[it.a_off + j + (long long)i * lda];
  if (trans == 2) a = conj_(a);
  T* pb = B + it.b_off + i + (long long)j * ldb;
  if (copy) { *pb = a; return; }
  T v = mul(alpha, a);
  if (!is_zero(beta)) v = add(v, mul(beta, *pb));
  *pb = v;
}
template <typename T>
__global__ __launch_bounds__(256) void k_geadd(const TileItem* __restrict__ items, int nitems, int mmax, int nmax, const T* A,
                                               int lda, T* B, int ldb, int part, int trans, T alpha, T beta,
                                               int copy) {
  // grid-stride: a launch covers at most 2^28 work-items (HSA grid sizes are 32-bit)
  const long long stride = (long long)gridDim.x * 256;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x;; gid += stride) {
    if (gid >= (long long)nitems * mmax * nmax) return;
    k_geadd_one<T>(gid, items, nitems, mmax, nmax, A, lda, B, ldb, part, trans, alpha, beta, copy);
  }
}
template <typename T>
__device__ inline void k_lascal_one(long long gid, const TileItem* __restrict__ items, int nitems, int mmax, int nmax, T* A, int lda,
                                                int part, T alpha) {
  const int per = mmax * nmax;
  if (gid >= (long long)nitems * per) return;  // tail of the last block
  const int item = (int)(gid / per), r = (int)(gid % per);
  const int i = r % mmax, j = r / mmax;
  const TileItem it = items[item];
  if (i >= it.m || j >= it.n) return;
  const long long I = it.gi + i, J = it.gj + j;
  if (!in_part(part, I, J)) return;
  T* p = A + it.a_off + i + (long long)j * lda;
  *p = mul(alpha, *p);
}
template <typename T>
__global__ __launch_bounds__(256) void k_lascal(const TileItem* __restrict__ items, int nitems, int mmax, int nmax, T* A, int lda,
                                                int part, T alpha) {
  // grid-stride: a launch covers at most 2^28 work-items (HSA grid sizes are 32-bit)
  const long long stride = (long long)gridDim.x * 256;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x;; gid += stride) {
    if (gid >= (long long)nitems * mmax * nmax) return;
    k_lascal_one<T>(gid, items, nitems, mmax, nmax, A, lda, part, alpha);
  }
}

// ---------------------------------------------------------------- diagonal scaling (LDL^H family)
// B(i, j) := B(i, j) / d, with d the diagonal of the tile at D + item.a_off:
// cols != 0: d = D(j, j) (B := B D^-1, CORE_ztrmdm / hetrf), else d = D(i, i) (B := D^-1 B, CORE_ztrdsm).
// item.b_off addresses the B tile; gi/gj its global coordinates for the part mask.
template <typename T>
__device__ inline void k_diag_scale_one(long long gid, const TileItem* __restrict__ items, int nitems, int mmax,
                                                    int nmax, const T* __restrict__ D, int ldd, T* B, int ldb,
                                                    int part, int cols) {
  const int per = mmax * nmax;
  if (gid >= (long long)nitems * per) return;
  const int item = (int)(gid / per), r = (int)(gid % per);
  const int i = r % mmax, j = r / mmax;
  const TileItem it = items[item];
  if (i >= it.m || j >= it.n) return;
  if (!in_part(part, it.gi + i, it.gj + j)) return;
  const int q = cols ? j : i;
  const T d = D[it.a_off + q + (long long)q * ldd];
  T* p = B + it.b_off + i + (long long)j * ldb;
  *p = divv(*p, d);
}
template <typename T>
__global__ __launch_bounds__(256) void k_diag_scale(const TileItem* __restrict__ items, int nitems, int mmax,
                                                    int nmax, const T* __restrict__ D, int ldd, T* B, int ldb,
                                                    int part, int cols) {
  // grid-stride: a launch covers at most 2^28 work-items (HSA grid sizes are 32-bit)
  const long long stride = (long long)gridDim.x * 256;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x;; gid += stride) {
    if (gid >= (long long)nitems * mmax * nmax) return;
    k_diag_scale_one<T>(gid, items, nitems, mmax, nmax, D, ldd, B, ldb, part, cols);
  }
}

// ---------------------------------------------------------------- norms
// kind 0: max |a| -> out[item]
// kind 1: column sums of |a| -> out[item*ostride + j]
// kind 2: row sums of |a| -> out[item*ostride + i]
// kind 3: (scale, ssq) with sum = scale^2 * ssq -> out[item*2 + {0,1}]
// part as above; unit: treat diagonal as 1 (lantr, diag = Unit)
template <typename T>
__global__ __launch_bounds__(256) void k_tile_norm(const TileItem* __restrict__ items, const T* A, int lda, int part,
                                                   int unit, int kind, double* out, int ostride) {
  typedef typename ST<T>::real R;
  const TileItem it = items[blockIdx.x];
  const T* Ab = A + it.a_off;
  const int tid = threadIdx.x;
  __shared__ double red[256];
  auto val = [&](int i, int j) -> double {
    const long long I = it.gi + i, J = it.gj + j;
    if (!in_part(part, I, J)) return 0.0;
    if (unit && I == J) return 1.0;
    return (double)absv(Ab[i + (long long)j * lda]);
  };
  if (kind == 0 || kind == 3) {
    double mx = 0.0;
    for (long long e = tid; e < (long long)it.m * it.n; e += 256) {
      const int i = (int)(e % it.m), j = (int)(e / it.m);
      mx = fmax(mx, val(i, j));
    }
    red[tid] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
      __syncthreads();
    }
    const double gmx = red[0];
    __syncthreads();
    if (kind == 0) {
      if (tid == 0) out[blockIdx.x] = gmx;
      return;
    }
    double ss = 0.0;
    if (gmx > 0.0) {
      for (long long e = tid; e < (long long)it.m * it.n; e += 256) {
        const int i = (int)(e % it.m), j = (int)(e / it.m);
        const double v = val(i, j) / gmx;
        ss += v * v;
      }
    }
    red[tid] = ss;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) red[tid] += red[tid + s];
      __syncthreads();
    }
    if (tid == 0) {
      out[2 * blockIdx.x] = gmx;
      out[2 * blockIdx.x + 1] = red[0];
    }
    return;
  }
  if (kind == 1) {
    for (int j = tid; j < it.n; j += 256) {
      double s = 0.0;
      for (int i = 0; i < it.m; ++i) s += val(i, j);
      out[(long long)blockIdx.x * ostride + j] = s;
    }
  } else {
    for (int i = tid; i < it.m; i += 256) {
      double s = 0.0;
      for (int j = 0; j < it.n; ++j) s += val(i, j);
      out[(long long)blockIdx.x * ostride + i] = s;
    }
  }
}

// ---------------------------------------------------------------- launchers
#define DISPATCH(prec, CALL)                                          \
  switch (prec) {                                                     \
    case DPL_S: { typedef float T; CALL; } break;                     \
    case DPL_D: { typedef double T; CALL; } break;                    \
    case DPL_C: { typedef hipFloatComplex T; CALL; } break;           \
    case DPL_Z: { typedef hipDoubleComplex T; CALL; } break;          \
    default: return -2;                                               \
  }

DPL_API int dpl_generate(int prec, int kind, int nitems, const void* items, int mmax, int nmax, void* A, int lda,
                         long long gM, unsigned long long seed, const void* bump, hipStream_t st) {
  if (nitems <= 0) return 0;
  const int nseg = cdiv(mmax, SEG);
  const long long total = (long long)nitems * nseg * nmax;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 1LL << 20);
  DISPATCH(prec, hipLaunchKernelGGL((k_generate<T>), dim3(blocks), dim3(256), 0, st, (const TileItem*)items, nitems, nseg,
                                    nmax, (T*)A, lda, gM, seed, kind, *(const T*)bump));
  return (int)hipGetLastError();
}

DPL_API int dpl_laset(int prec, int part, int nitems, const void* items, int mmax, int nmax, const void* alpha,
                      const void* beta, void* A, int lda, hipStream_t st) {
  if (nitems <= 0) return 0;
  const long long total = (long long)nitems * mmax * nmax;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 1LL << 20);
  DISPATCH(prec, hipLaunchKernelGGL((k_laset<T>), dim3(blocks), dim3(256), 0, st, (const TileItem*)items, nitems, mmax, nmax,
                                    (T*)A, lda, part, *(const T*)alpha, *(const T*)beta));
  return (int)hipGetLastError();
}

// copy != 0: B = op(A) (lacpy / latro); else B = alpha*op(A) + beta*B (geadd / tradd)
DPL_API int dpl_geadd(int prec, int part, int trans, int nitems, const void* items, int mmax, int nmax,
                      const void* alpha, const void* A, int lda, const void* beta, void* B, int ldb, int copy,
                      hipStream_t st) {
  if (nitems <= 0) return 0;
  const long long total = (long long)nitems * mmax * nmax;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 1LL << 20);
  const int tr = trans == DPL_NOTRANS ? 0 : (trans == DPL_TRANS ? 1 : 2);
  DISPATCH(prec, hipLaunchKernelGGL((k_geadd<T>), dim3(blocks), dim3(256), 0, st, (const TileItem*)items, nitems, mmax, nmax,
                                    (const T*)A, lda, (T*)B, ldb, part, tr, *(const T*)alpha, *(const T*)beta, copy));
  return (int)hipGetLastError();
}

DPL_API int dpl_lascal(int prec, int part, int nitems, const void* items, int mmax, int nmax, const void* alpha,
                       void* A, int lda, hipStream_t st) {
  if (nitems <= 0) return 0;
  const long long total = (long long)nitems * mmax * nmax;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 1LL << 20);
  DISPATCH(prec, hipLaunchKernelGGL((k_lascal<T>), dim3(blocks), dim3(256), 0, st, (const TileItem*)items, nitems, mmax,
                                    nmax, (T*)A, lda, part, *(const T*)alpha));
  return (int)hipGetLastError();
}

DPL_API int dpl_diag_scale(int prec, int part, int cols, int nitems, const void* items, int mmax, int nmax,
                           const void* D, int ldd, void* B, int ldb, hipStream_t st) {
  if (nitems <= 0) return 0;
  const long long total = (long long)nitems * mmax * nmax;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 1LL << 20);
  DISPATCH(prec, hipLaunchKernelGGL((k_diag_scale<T>), dim3(blocks), dim3(256), 0, st, (const TileItem*)items, nitems,
                                    mmax, nmax, (const T*)D, ldd, (T*)B, ldb, part, cols));
  return (int)hipGetLastError();
}

DPL_API int dpl_tile_norm(int prec, int kind, int part, int unit, int nitems, const void* items, const void* A,
                          int lda, double* out, int ostride, hipStream_t st) {
  if (nitems <= 0) return 0;
  DISPATCH(prec, hipLaunchKernelGGL((k_tile_norm<T>), dim3(nitems), dim3(256), 0, st, (const TileItem*)items,
                                    (const T*)A, lda, part, unit, kind, out, ostride));
  return (int)hipGetLastError();
}

// Stream restricted to a CU subset (CDNA CU masking): bit i of mask[i / 32] enables CU i.  Used to
// give the latency-bound diagonal-tile Cholesky its own CU(s), away from the CU-saturating trailing
// GEMM it would otherwise share SIMDs with.
// ---------------------------------------------------------------- tile-pair swap-transpose
// For each item: tile a (m x n at a_off) and tile b (n x m at b_off) become  a <- op(b)^T,
// b <- op(a)^T  (op = conj when cj, i.e. conjugate transposes); a_off == b_off transposes one square
// tile in place.  Grid (items, 32x32 sub-blocks of a): workgroup (r, c) exchanges sub-block (r, c) of
// a with sub-block (c, r) of b through LDS (coalesced 32-wide column reads and writes on both sides;
// row stride 33: conflict-free transposed reads).  In-place tiles: only r <= c works.
// Used by the upper Cholesky on one process: A^T (A^H) turns the upper triangle into the lower one,
// the lower schedule factors it, and the same exchange writes U = L^T (L^H) back while restoring the
// untouched strictly-lower triangle.
template <typename T>
__global__ __launch_bounds__(256) void k_swap_transpose(const TileItem* __restrict__ items, int nbc, T* __restrict__ A,
                                                        int ld, int cj) {
  __shared__ T sa[32 * 33], sb[32 * 33];
  const TileItem it = items[blockIdx.x];
  const int r = blockIdx.y / nbc, c = blockIdx.y % nbc;
  if (32 * r >= it.m || 32 * c >= it.n) return;
  const bool same = it.a_off == it.b_off;
  if (same && r > c) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int ra = 32 * r, ca = 32 * c;                  // sub-block origin in a; in b it is (ca, ra)
  const int mr = min(32, it.m - ra), nc = min(32, it.n - ca);
  T* a = A + it.a_off;
  T* b = A + it.b_off;
  const bool diag = same && r == c;
  // sa(i, j) = a(ra + i, ca + j);  sb(j, i) = b(ca + j, ra + i)
  for (int j = ty; j < 32; j += 8) {
    if (tx < mr && j < nc) sa[j * 33 + tx] = a[(long long)(ca + j) * ld + ra + tx];
    if (!diag && tx < nc && j < mr) sb[j * 33 + tx] = b[(long long)(ra + j) * ld + ca + tx];
  }
  __syncthreads();
  const T* src_for_a = diag ? sa : sb;
  for (int j = ty; j < 32; j += 8) {
    // a(ra + tx, ca + j) = op(b(ca + j, ra + tx)) = op(sb[tx * 33 + j])   (diag: op(sa[tx * 33 + j]))
    if (tx < mr && j < nc) {
      const T v = src_for_a[tx * 33 + j];
      a[(long long)(ca + j) * ld + ra + tx] = cj ? conj_(v) : v;
    }
    // b(ca + tx, ra + j) = op(a(ra + j, ca + tx)) = op(sa[tx * 33 + j])
    if (!diag && tx < nc && j < mr) {
      const T v = sa[tx * 33 + j];
      b[(long long)(ra + j) * ld + ca + tx] = cj ? conj_(v) : v;
    }
  }
}

DPL_API int dpl_swap_transpose(int prec, int nitems, const void* items, int mmax, int nmax, void* A, int ld, int cj,
                               hipStream_t st) {
  if (nitems <= 0) return 0;
  const int nbr = cdiv(mmax, 32), nbc = cdiv(nmax, 32);
  DISPATCH(prec, hipLaunchKernelGGL((k_swap_transpose<T>), dim3(nitems, nbr * nbc), dim3(256), 0, st,
                                    (const TileItem*)items, nbc, (T*)A, ld, cj));
  return (int)hipGetLastError();
}

// One-way transposed tile copy: for each item, tile y (n x m at b_off in Y) <- op(tile x)^T (x: m x n at
// a_off in X), op = conj when cj; upper_only writes only y(p, q), p <= q (a diagonal tile whose strictly
// lower part must stay).  Same LDS-staged 32x32 sub-block scheme as k_swap_transpose, half its traffic.
template <typename T>
__global__ __launch_bounds__(256) void k_copy_transpose(const TileItem* __restrict__ items, int nbc,
                                                        const T* __restrict__ X, int ldx, T* __restrict__ Y, int ldy,
                                                        int cj, int upper_only) {
  __shared__ T sa[32 * 33];
  const TileItem it = items[blockIdx.x];
  const int r = blockIdx.y / nbc, c = blockIdx.y % nbc;
  if (32 * r >= it.m || 32 * c >= it.n) return;
  if (upper_only && c > r) return;             // y block (c, r) lies strictly below the diagonal
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int ra = 32 * r, ca = 32 * c;
  const int mr = min(32, it.m - ra), nc = min(32, it.n - ca);
  const T* x = X + it.a_off;
  T* y = Y + it.b_off;
  for (int j = ty; j < 32; j += 8)
    if (tx < mr && j < nc) sa[j * 33 + tx] = x[(long long)(ca + j) * ldx + ra + tx];
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    // y(ca + tx, ra + j) = op(x(ra + j, ca + tx)) = op(sa[tx * 33 + j])
    if (tx < nc && j < mr && (!upper_only || ca + tx <= ra + j)) {
      const T v = sa[tx * 33 + j];
      y[(long long)(ra + j) * ldy + ca + tx] = cj ? conj_(v) : v;
    }
  }
}

DPL_API int dpl_copy_transpose(int prec, int nitems, const void* items, int mmax, int nmax, const void* X, int ldx,
                               void* Y, int ldy, int cj, int upper_only, hipStream_t st) {
  if (nitems <= 0) return 0;
  const int nbr = cdiv(mmax, 32), nbc = cdiv(nmax, 32);
  DISPATCH(prec, hipLaunchKernelGGL((k_copy_transpose<T>), dim3(nitems, nbr * nbc), dim3(256), 0, st,
                                    (const TileItem*)items, nbc, (const T*)X, ldx, (T*)Y, ldy, cj, upper_only));
  return (int)hipGetLastError();
}

DPL_API int dpl_stream_cumask(const unsigned* mask, int nwords, void** out) {
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  *out = (void*)s;
  return (int)e;
}

DPL_API int dpl_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

// Busy wait of a fixed wall-clock duration on a stream (tools/replay_potrf.py: stands in for an
// RCCL transfer of modelled duration -- occupying, like the RCCL kernel it replaces, nwg workgroup
// slots).  wall_clock64(): the 100 MHz constant-rate counter; bounded to 1 s.
__global__ __launch_bounds__(64) void k_delay(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  if (ticks > 100000000ull) ticks = 100000000ull;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

DPL_API int dpl_delay(double us, int nwg, hipStream_t st) {
  if (us <= 0.0) return 0;
  const unsigned long long ticks = (unsigned long long)(us * 100.0);   // 10 ns per tick
  hipLaunchKernelGGL(k_delay, dim3(nwg < 1 ? 1 : nwg), dim3(64), 0, st, ticks);
  return (int)hipGetLastError();
}

// out[i] = in[i] + delta, i < n (pivot index bookkeeping: panel-relative <-> global, 0 <-> 1-based)
__global__ __launch_bounds__(256) void k_ipiv_shift(const int* __restrict__ in, int* __restrict__ out, int n,
                                                    int delta) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = in[i] + delta;
}

DPL_API int dpl_ipiv_shift(const int* in, int* out, int n, int delta, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_ipiv_shift, dim3((n + 255) / 256), dim3(256), 0, st, in, out, n, delta);
  return (int)hipGetLastError();
}
