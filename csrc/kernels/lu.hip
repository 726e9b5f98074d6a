// LU kernels: panel factorisation with partial pivoting (or none) and row gather.
//
// Reference roles: CORE_zgetrf_rectil / _reclap (multithreaded recursive panel,
// src/cores/core_zgetrf_rectil.c:120-279), CORE_zgetrf_nopiv (core_zgetrf_nopiv.c:69),
// CORE_zlaswp / zlaswp_ontile (core_zlaswp.c:62-224), the GETRF_MAX/RDC/SND
// pivot search of src/zgetrf_ptgpanel.jdf:206-590.
//
// Panel: one 1024-thread workgroup factors an m x n column-major panel
// (the concatenation of the panel's tiles): for each column a workgroup-wide
// |max| reduction in LDS picks the pivot, the two rows are swapped across the
// panel, the column is scaled and the trailing panel columns get a rank-1
// update.  Pivot indices are 0-based panel rows.  (Round-1 implementation:
// correctness first; the trailing update is not yet blocked.)
// Row gather: dst row r_i := src row s_i for a list of (dst, src) row offsets,
// used to apply a panel's net permutation to the other columns.
#include "common.h"

#define LT 1024
template <typename T>
__global__ __launch_bounds__(LT) void k_getrf_panel(T* __restrict__ A, int m, int n, int lda,
                                                    int* __restrict__ ipiv, int* __restrict__ info, int info_base,
                                                    int pivot) {
  typedef typename ST<T>::real R;
  __shared__ R sv[LT];
  __shared__ int si[LT];
  __shared__ int s_p;
  const int tid = threadIdx.x;
  const int kmax = min(m, n);
  for (int j = 0; j < kmax; ++j) {
    int p = j;
    if (pivot) {
      R best = -1;
      int bi = j;
      for (int i = j + tid; i < m; i += LT) {
        const R v = abs1(A[i + (long long)j * lda]);
        if (v > best) { best = v; bi = i; }
      }
      sv[tid] = best;
      si[tid] = bi;
      __syncthreads();
      for (int s = LT / 2; s > 0; s >>= 1) {
        if (tid < s) {
          const R a = sv[tid], b = sv[tid + s];
          // ties -> smaller row index (LAPACK idamax picks the first maximum)
          if (b > a || (b == a && si[tid + s] < si[tid])) { sv[tid] = b; si[tid] = si[tid + s]; }
        }
        __syncthreads();
      }
      if (tid == 0) s_p = si[0];
      __syncthreads();
      p = s_p;
      // swap rows j and p across the whole panel
      if (p != j) {
        for (int c = tid; c < n; c += LT) {
          T t = A[j + (long long)c * lda];
          A[j + (long long)c * lda] = A[p + (long long)c * lda];
          A[p + (long long)c * lda] = t;
        }
      }
    }
    if (tid == 0 && ipiv) ipiv[j] = p;
    __syncthreads();
    const T d = A[j + (long long)j * lda];
    if (is_zero(d)) {
      if (tid == 0 && info && *info == 0) *info = info_base + j + 1;
    } else {
      for (int i = j + 1 + tid; i < m; i += LT) A[i + (long long)j * lda] = divv(A[i + (long long)j * lda], d);
    }
    __syncthreads();
    // rank-1 update of the trailing panel
    const int rows = m - j - 1, cols = n - j - 1;
    if (rows > 0 && cols > 0) {
      for (long long e = tid; e < (long long)rows * cols; e += LT) {
        const int i = j + 1 + (int)(e % rows), c = j + 1 + (int)(e / rows);
        A[i + (long long)c * lda] = sub(A[i + (long long)c * lda], mul(A[i + (long long)j * lda], A[j + (long long)c * lda]));
      }
    }
    __syncthreads();
  }
}

struct RowPair {
  long long dst, src;  // element offsets of the row starts
};
template <typename T>
__global__ __launch_bounds__(256) void k_row_gather(T* __restrict__ dst, const T* __restrict__ src,
                                                    const RowPair* __restrict__ rows, int nrows, int ncols,
                                                    int ld_dst, int ld_src) {
  const int r = blockIdx.y;
  if (r >= nrows) return;
  const RowPair rp = rows[r];
  for (int c = blockIdx.x * 256 + threadIdx.x; c < ncols; c += gridDim.x * 256)
    dst[rp.dst + (long long)c * ld_dst] = src[rp.src + (long long)c * ld_src];
}

#define DISPATCH(prec, CALL)                                          \
  switch (prec) {                                                     \
    case DPL_S: { typedef float T; CALL; } break;                     \
    case DPL_D: { typedef double T; CALL; } break;                    \
    case DPL_C: { typedef hipFloatComplex T; CALL; } break;           \
    case DPL_Z: { typedef hipDoubleComplex T; CALL; } break;          \
    default: return -2;                                               \
  }

DPL_API int dpl_getrf_panel(int prec, int m, int n, void* A, long long a_off, int lda, int* ipiv, int* info,
                            int info_base, int pivot, hipStream_t st) {
  if (m <= 0 || n <= 0) return 0;
  DISPATCH(prec, hipLaunchKernelGGL((k_getrf_panel<T>), dim3(1), dim3(LT), 0, st, (T*)A + a_off, m, n, lda, ipiv,
                                    info, info_base, pivot));
  return (int)hipGetLastError();
}

// rows: device RowPair[nrows]; dst/src may alias only if no dst row is also a src row
DPL_API int dpl_row_gather(int prec, void* dst, const void* src, const void* rows, int nrows, int ncols, int ld_dst,
                           int ld_src, hipStream_t st) {
  if (nrows <= 0 || ncols <= 0) return 0;
  dim3 g((ncols + 255) / 256 > 64 ? 64 : (ncols + 255) / 256, nrows);
  DISPATCH(prec, hipLaunchKernelGGL((k_row_gather<T>), g, dim3(256), 0, st, (T*)dst, (const T*)src,
                                    (const RowPair*)rows, nrows, ncols, ld_dst, ld_src));
  return (int)hipGetLastError();
}
