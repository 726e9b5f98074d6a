// LU with incremental (tile-pairwise) pivoting: tile kernels on DAG items.
//
// Reference roles (PLASMA core_blas, src/zgetrf_incpiv.jdf task classes
// zgetrf(k) :52, zgessm(k,n) :102, ztstrf(k,m) :156, zssssm(k,m,n) :234):
//   GETRF  partial-pivoting LU of the diagonal tile; IPIV 1-based tile rows
//   GESSM  apply a GETRF tile's row interchanges and unit-lower L^-1 to a tile of its row
//   TSTRF  LU of [U; A] (U upper triangular, A square): pivots are searched
//          between U's diagonal and A's column, IB columns at a time; the
//          multiplier histories of rows swapped into U ("swap behind") form the
//          unit-lower IB x IB blocks of the L tile; IPIV entries are ii+i+1 (no
//          swap) or NB+im+1 (swap with A row im)   (core_ztstrf.c:100-240)
//   SSSSM  replay a TSTRF on [A1; A2]: per IB block, the swaps, A1 := L1^-1 A1,
//          A2 -= L2 A1   (core_zssssm.c)
// Semantics match the PLASMA routines so that L / IPIV descriptors have the
// reference's shapes (L: mt*ib x nt*nb, IPIV: m x nt).  Round-1 kernels are
// VALU: one column per lane for GESSM/SSSSM (columns are independent), one
// 256-thread workgroup per TSTRF / GETRF tile.
#include "common.h"

struct LuItem {  // = DAG_ITEM (96 bytes)
  long long p0, p1, p2, p3;
  int ld0, ld1, ld2, ld3;
  int m, n, k, pad;
  long long p4, p5;
  int ld4, ld5, aux0, aux1;
};
static_assert(sizeof(LuItem) == 96, "LuItem layout = DAG_ITEM");

#define LUT 256
template <typename T>
__device__ inline T& el(T* b, int ld, int i, int j) { return b[i + (long long)j * ld]; }

// block-wide argmax of abs1 over rows [r0, r1) of column j (ties -> smallest row)
template <typename T>
__device__ inline int block_argmax(const T* A, int ld, int j, int r0, int r1, typename ST<T>::real* sv, int* si) {
  typedef typename ST<T>::real R;
  const int tid = threadIdx.x;
  R best = -1;
  int bi = r0;
  for (int r = r0 + tid; r < r1; r += LUT) {
    const R v = abs1(A[r + (long long)j * ld]);
    if (v > best) {
      best = v;
      bi = r;
    }
  }
  sv[tid] = best;
  si[tid] = bi;
  __syncthreads();
  for (int s = LUT / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const R a = sv[tid], b = sv[tid + s];
      if (b > a || (b == a && si[tid + s] < si[tid])) {
        sv[tid] = b;
        si[tid] = si[tid + s];
      }
    }
    __syncthreads();
  }
  const int p = si[0];
  __syncthreads();
  return p;
}

// ------------------------------------------------------------------ GETRF (tile)
// item: p1 = A (m x n), p3 = IPIV (int), k = global column offset (for info)
template <typename T>
__global__ __launch_bounds__(LUT) void k_getrf_tile(const LuItem* __restrict__ items, int* __restrict__ info) {
  typedef typename ST<T>::real R;
  __shared__ R sv[LUT];
  __shared__ int si[LUT];
  const LuItem it = items[blockIdx.x];
  T* A = (T*)it.p1;
  int* ipiv = (int*)it.p3;
  const int m = it.m, n = it.n, ld = it.ld1, tid = threadIdx.x;
  const int kmax = min(m, n);
  for (int j = 0; j < kmax; ++j) {
    const int p = block_argmax(A, ld, j, j, m, sv, si);
    if (p != j)
      for (int c = tid; c < n; c += LUT) {
        const T t = el(A, ld, j, c);
        el(A, ld, j, c) = el(A, ld, p, c);
        el(A, ld, p, c) = t;
      }
    if (tid == 0) ipiv[j] = p + 1;
    __syncthreads();
    const T d = el(A, ld, j, j);
    if (is_zero(d)) {
      if (tid == 0 && info) atomicCAS(info, 0, it.k + j + 1);
    } else {
      const T inv = divv(ST<T>::one(), d);
      for (int r = j + 1 + tid; r < m; r += LUT) el(A, ld, r, j) = mul(el(A, ld, r, j), inv);
    }
    __syncthreads();
    const int rows = m - j - 1, cols = n - j - 1;
    for (int e = tid; e < rows * cols; e += LUT) {
      const int r = j + 1 + e % rows, c = j + 1 + e / rows;
      el(A, ld, r, c) = sub(el(A, ld, r, c), mul(el(A, ld, r, j), el(A, ld, j, c)));
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ GESSM
// item: p1 = C (m x n) (tile of row k), p2 = LU tile (m x kk, unit lower L), p3 = IPIV; k = kk
// grid: items x ceil(n / 64); one lane per column.
template <typename T>
__global__ __launch_bounds__(64) void k_gessm(const LuItem* __restrict__ items, int nchunk) {
  const LuItem it = items[blockIdx.x / nchunk];
  const int c = (blockIdx.x % nchunk) * 64 + threadIdx.x;
  if (c >= it.n) return;
  T* C = (T*)it.p1;
  const T* L = (const T*)it.p2;
  const int* ipiv = (const int*)it.p3;
  const int m = it.m, kk = it.k, ldc = it.ld1, ldl = it.ld2;
  for (int i = 0; i < kk; ++i) {
    const int p = ipiv[i] - 1;
    if (p != i) {
      const T t = el(C, ldc, i, c);
      el(C, ldc, i, c) = el(C, ldc, p, c);
      el(C, ldc, p, c) = t;
    }
  }
  for (int i = 0; i < kk; ++i) {
    const T x = el(C, ldc, i, c);
    for (int r = i + 1; r < m; ++r) el(C, ldc, r, c) = sub(el(C, ldc, r, c), mul(L[r + (long long)i * ldl], x));
  }
}

// ------------------------------------------------------------------ SSSSM
// item: p0 = A1 (>= K rows x n), p1 = A2 (m x n), p2 = L1 tile (ib x K), p3 = IPIV, p4 = L2 (m x K)
//       m = rows of A2, n = cols, k = K; launch: ib, NB (row count of A1 in the IPIV encoding)
template <typename T>
__global__ __launch_bounds__(64) void k_ssssm(const LuItem* __restrict__ items, int nchunk, int ib, int NB) {
  const LuItem it = items[blockIdx.x / nchunk];
  const int c = (blockIdx.x % nchunk) * 64 + threadIdx.x;
  if (c >= it.n) return;
  T* A1 = (T*)it.p0;
  T* A2 = (T*)it.p1;
  const T* L1 = (const T*)it.p2;
  const int* ipiv = (const int*)it.p3;
  const T* L2 = (const T*)it.p4;
  const int m = it.m, K = it.k, ld1 = it.ld0, ld2 = it.ld1, ldl1 = it.ld2, ldl2 = it.ld4;
  for (int ii = 0; ii < K; ii += ib) {
    const int sb = min(ib, K - ii);
    for (int i = 0; i < sb; ++i) {
      const int im = ipiv[ii + i] - 1;
      if (im != ii + i) {
        const int r2 = im - NB;
        const T t = el(A1, ld1, ii + i, c);
        el(A1, ld1, ii + i, c) = el(A2, ld2, r2, c);
        el(A2, ld2, r2, c) = t;
      }
    }
    for (int i = 1; i < sb; ++i) {
      T s = el(A1, ld1, ii + i, c);
      for (int j = 0; j < i; ++j) s = sub(s, mul(L1[i + (long long)(ii + j) * ldl1], el(A1, ld1, ii + j, c)));
      el(A1, ld1, ii + i, c) = s;
    }
    for (int r = 0; r < m; ++r) {
      T s = el(A2, ld2, r, c);
      for (int i = 0; i < sb; ++i) s = sub(s, mul(L2[r + (long long)(ii + i) * ldl2], el(A1, ld1, ii + i, c)));
      el(A2, ld2, r, c) = s;
    }
  }
}

// ------------------------------------------------------------------ TSTRF
// item: p0 = U (NB x n, upper), p1 = A (m x n), p2 = L tile (ib x n), p3 = IPIV; m, n, k = global col offset
// launch: ib (<= 32), NB; one 256-thread workgroup per item, W (m x ib) in LDS (m <= 256)
template <typename T>
__global__ __launch_bounds__(LUT) void k_tstrf(const LuItem* __restrict__ items, int ib, int NB,
                                               int* __restrict__ info) {
  typedef typename ST<T>::real R;
  __shared__ R sv[LUT];
  __shared__ int si[LUT];
  __shared__ T W[32][257];
  const LuItem it = items[blockIdx.x];
  T* U = (T*)it.p0;
  T* A = (T*)it.p1;
  T* L = (T*)it.p2;
  int* ipiv = (int*)it.p3;
  const int m = it.m, n = it.n, ldu = it.ld0, lda = it.ld1, ldl = it.ld2, tid = threadIdx.x;
  for (int e = tid; e < ib * n; e += LUT) el(L, ldl, e % ib, e / ib) = ST<T>::zero();
  __syncthreads();
  for (int ii = 0; ii < n; ii += ib) {
    const int sb = min(n - ii, ib);
    for (int i = 0; i < sb; ++i) {
      const int col = ii + i;
      const int im = block_argmax(A, lda, col, 0, m, sv, si);
      const bool sw = absv(el(A, lda, im, col)) > absv(el(U, ldu, col, col));
      __syncthreads();  // every thread has decided before anyone swaps
      if (sw) {
        for (int j = tid; j < i; j += LUT) {  // swap behind
          const T t = el(L, ldl, i, ii + j);
          el(L, ldl, i, ii + j) = W[j][im];
          W[j][im] = t;
        }
        for (int j = i + tid; j < sb; j += LUT) {  // swap ahead
          const T t = el(U, ldu, col, ii + j);
          el(U, ldu, col, ii + j) = el(A, lda, im, ii + j);
          el(A, lda, im, ii + j) = t;
        }
      }
      __syncthreads();
      if (sw)
        for (int j = tid; j < i; j += LUT) el(A, lda, im, ii + j) = ST<T>::zero();
      if (tid == 0) {
        ipiv[col] = sw ? NB + im + 1 : col + 1;
        if (info && is_zero(el(U, ldu, col, col))) atomicCAS(info, 0, it.k + col + 1);
      }
      __syncthreads();
      const T u = el(U, ldu, col, col);
      const T alpha = is_zero(u) ? ST<T>::zero() : divv(ST<T>::one(), u);
      for (int r = tid; r < m; r += LUT) {
        const T x = mul(el(A, lda, r, col), alpha);
        el(A, lda, r, col) = x;
        W[i][r] = x;
      }
      __syncthreads();
      const int rest = sb - i - 1;
      for (int e = tid; e < m * rest; e += LUT) {
        const int r = e % m, j = col + 1 + e / m;
        el(A, lda, r, j) = sub(el(A, lda, r, j), mul(el(A, lda, r, col), el(U, ldu, col, j)));
      }
      __syncthreads();
    }
    // replay the block on the trailing columns (one thread per column)
    for (int c = ii + sb + tid; c < n; c += LUT) {
      for (int i = 0; i < sb; ++i) {
        const int p = ipiv[ii + i] - 1;
        if (p != ii + i) {
          const int r2 = p - NB;
          const T t = el(U, ldu, ii + i, c);
          el(U, ldu, ii + i, c) = el(A, lda, r2, c);
          el(A, lda, r2, c) = t;
        }
      }
      for (int i = 1; i < sb; ++i) {
        T s = el(U, ldu, ii + i, c);
        for (int j = 0; j < i; ++j) s = sub(s, mul(el(L, ldl, i, ii + j), el(U, ldu, ii + j, c)));
        el(U, ldu, ii + i, c) = s;
      }
      for (int r = 0; r < m; ++r) {
        T s = el(A, lda, r, c);
        for (int i = 0; i < sb; ++i) s = sub(s, mul(el(A, lda, r, ii + i), el(U, ldu, ii + i, c)));
        el(A, lda, r, c) = s;
      }
    }
    __syncthreads();
  }
}

#define DISPATCH(prec, CALL)                                          \
  switch (prec) {                                                     \
    case DPL_S: { typedef float T; CALL; } break;                     \
    case DPL_D: { typedef double T; CALL; } break;                    \
    case DPL_C: { typedef hipFloatComplex T; CALL; } break;           \
    case DPL_Z: { typedef hipDoubleComplex T; CALL; } break;          \
    default: return -2;                                               \
  }

DPL_API int dpl_getrf_tile(int prec, int nitems, const void* items, int* info, hipStream_t st) {
  if (nitems <= 0) return 0;
  DISPATCH(prec, hipLaunchKernelGGL((k_getrf_tile<T>), dim3(nitems), dim3(LUT), 0, st, (const LuItem*)items, info));
  return (int)hipGetLastError();
}

DPL_API int dpl_gessm(int prec, int nitems, const void* items, int max_n, hipStream_t st) {
  if (nitems <= 0) return 0;
  const int nchunk = cdiv(max_n, 64);
  DISPATCH(prec, hipLaunchKernelGGL((k_gessm<T>), dim3(nitems * nchunk), dim3(64), 0, st, (const LuItem*)items,
                                    nchunk));
  return (int)hipGetLastError();
}

DPL_API int dpl_ssssm(int prec, int nitems, const void* items, int max_n, int ib, int NB, hipStream_t st) {
  if (nitems <= 0) return 0;
  const int nchunk = cdiv(max_n, 64);
  DISPATCH(prec, hipLaunchKernelGGL((k_ssssm<T>), dim3(nitems * nchunk), dim3(64), 0, st, (const LuItem*)items,
                                    nchunk, ib, NB));
  return (int)hipGetLastError();
}

DPL_API int dpl_tstrf(int prec, int nitems, const void* items, int ib, int NB, int max_m, int* info, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > 32 || ib <= 0 || max_m > 256) return -3;
  DISPATCH(prec, hipLaunchKernelGGL((k_tstrf<T>), dim3(nitems), dim3(LUT), 0, st, (const LuItem*)items, ib, NB, info));
  return (int)hipGetLastError();
}
