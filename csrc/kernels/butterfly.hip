// Random butterfly transformation, one level, applied element-wise in O(m n) (reference: the HEBUT /
// GEBUT / GEBMM task classes, src/zhebut.jdf, src/zgebut.jdf, src/zgebmm.jdf, whose bodies are the
// per-segment updates of src/cores/core_zhebut.c:21-46).
//
// Level l of the recursive butterfly U = B_0 B_1 ... B_{d-1} is block diagonal with 2^l blocks of order
// size = n / 2^l, each  W = 1/sqrt(2) [R0  R1; R0  -R1]  with R0 = diag(r[base .. base+h)),
// R1 = diag(r[base+h .. base+size)), h = size / 2.  A row (LEFT) or column (RIGHT) pair (p, p + h) of
// a block mixes with itself only, so a level is one pass over the matrix: one thread per element pair,
// two loads, two stores, no workspace.  Two update forms cover the four (side, trans) cases:
//   form 0  (B A, A B^T):     x0' = s (r0 x0 + r1 x1),   x1' = s (r0 x0 - r1 x1)
//   form 1  (B^T A, A B):     x0' = s r0 (x0 + x1),      x1' = s r1 (x0 - x1)
// (r real, so Trans and ConjTrans coincide).  Any tiled storage whose element (I, J) sits at
//   base + (I / mb) si + (J / nb) sj + I % mb + (J % nb) ld
// -- TILE storage (si = mb nb, sj = local tile rows * mb nb, ld = mb), LAPACK (si = mb, sj = nb ld) and
// the native library's column-major buffers (mb = nb = 2^30).
#include "common.h"

namespace {

struct ButGeom {
  long long si, sj;
  int mb, nb, ld;
};

__device__ inline long long eoff(const ButGeom& g, long long I, long long J) {
  return (I / g.mb) * g.si + (J / g.nb) * g.sj + (I % g.mb) + (J % g.nb) * (long long)g.ld;
}

// m x n matrix; the butterfly acts on rows (left) or columns (right) of order nb_ord = m or n.
// Thread layout: x over the "other" index (contiguous in memory for LEFT: rows of one column), y over pairs.
template <typename T>
__global__ __launch_bounds__(256) void k_butterfly(T* A, ButGeom g, int m, int n, int left, int form, int size,
                                                   const double* __restrict__ r) {
  typedef typename ST<T>::real R;
  const int h = size >> 1;
  const R s = (R)0.70710678118654752440;
  const long long npairs = (long long)(left ? m : n) / 2;
  const long long nother = left ? n : m;
  const long long total = npairs * nother;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    // LEFT: e -> (pair, column) with the pair index fastest, so a wave reads consecutive rows of a column
    // RIGHT: e -> (row, pair) with the row fastest (consecutive rows of two columns)
    long long pr, oth;
    if (left) {
      pr = e % npairs;
      oth = e / npairs;
    } else {
      oth = e % nother;
      pr = e / nother;
    }
    const long long blk = pr / h, q = pr % h;
    const long long i0 = blk * size + q, i1 = i0 + h;
    const R r0 = (R)r[i0], r1 = (R)r[i1];
    const long long o0 = left ? eoff(g, i0, oth) : eoff(g, oth, i0);
    const long long o1 = left ? eoff(g, i1, oth) : eoff(g, oth, i1);
    const T x0 = A[o0], x1 = A[o1];
    T y0, y1;
    if (form == 0) {
      const T a = mul(from_real<T>(r0), x0), b = mul(from_real<T>(r1), x1);
      y0 = mul(from_real<T>(s), add(a, b));
      y1 = mul(from_real<T>(s), sub(a, b));
    } else {
      y0 = mul(from_real<T>(s * r0), add(x0, x1));
      y1 = mul(from_real<T>(s * r1), sub(x0, x1));
    }
    A[o0] = y0;
    A[o1] = y1;
  }
}

template <typename T>
int launch(void* A, const ButGeom& g, int m, int n, int left, int form, int size, const double* r, hipStream_t st) {
  const long long pairs = (long long)(left ? m : n) / 2 * (long long)(left ? n : m);
  if (pairs <= 0) return 0;
  const long long want = (pairs + 255) / 256;
  const int grid = (int)(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(k_butterfly<T>, dim3(grid), dim3(256), 0, st, (T*)A, g, m, n, left, form, size, r);
  return (int)hipGetLastError();
}

}  // namespace

// One butterfly level on an m x n matrix: side LEFT (B_l or B_l^T times A) or RIGHT (A times B_l or B_l^T);
// trans NOTRANS / TRANS / CONJTRANS; size = order / 2^l (even, divides the order); r = the level's n real
// diagonal entries on the device.  Returns -2 on a bad shape (nothing launched).
DPL_API int dpl_butterfly(int prec, int side, int trans, int m, int n, int size, const double* r, void* A,
                          long long si, long long sj, int mb, int nb, int ld, hipStream_t st) {
  const int left = side == DPL_LEFT;
  const int ord = left ? m : n;
  if (m < 0 || n < 0 || size < 2 || (size & 1) || ord % size || !r || !A || mb <= 0 || nb <= 0 || ld <= 0)
    return -2;
  // B A and A B^T share form 0; B^T A and A B form 1
  const int form = (left == (trans == DPL_NOTRANS)) ? 0 : 1;
  const ButGeom g{si, sj, mb, nb, ld};
  switch (prec) {
    case DPL_S: return launch<float>(A, g, m, n, left, form, size, r, st);
    case DPL_D: return launch<double>(A, g, m, n, left, form, size, r, st);
    case DPL_C: return launch<hipFloatComplex>(A, g, m, n, left, form, size, r, st);
    case DPL_Z: return launch<hipDoubleComplex>(A, g, m, n, left, form, size, r, st);
    default: return -2;
  }
}
