// Householder QR tile kernels (and, through transposed/conjugated views, LQ).
//
// Reference roles (PLASMA core_blas semantics, inner blocking IB, T stored as
// IB x NB tiles of upper-triangular IB x IB blocks):
//   CORE_zgeqrt  src/cores/core_zgeqrt.c:86     QR of a tile, V below the diagonal
//   CORE_zunmqr  src/cores/core_zunmqr.c:108    apply Q / Q^H of a geqrt tile
//   CORE_ztsqrt  src/cores/core_ztsqrt.c:97     QR of [R; A2] (triangle on square)
//   CORE_ztsmqr  src/cores/core_ztsmqr.c:124    apply the TS reflectors to [A1; A2]
//   CORE_zttqrt / CORE_zttmqr (core_zttqrt.c:116, core_zttmqr.c:116): TT variants
//   (A2 / V2 upper triangular) -- same kernels with the `tri` flag, which never
//   reads or writes below the diagonal of A2 (it holds other reflectors in HQR).
//   LQ kernels (gelqt/tslqt/tsmlq/ttlqt/ttmlq/unmlq) are these kernels applied to
//   the conjugate-transposed view of the tile (row stride <-> column stride).
//
// Every operand is a strided view  X(i,j) = conj?( base[off + i*rs + j*cs] ),
// so one Left-side kernel serves left/right application and QR/LQ.  One
// 256-thread workgroup per item; reductions through LDS.  Round-1 kernels are
// VALU (all four precisions); the reflector application is blocked by IB.
#include "common.h"

struct View {
  int tr, cj;  // transposed access (element (i,j) at i*ld + j) and conjugation of the view
};
// Items carry absolute device addresses so that tiles may live in descriptor
// storage or in exchange receive buffers within one launch.
struct QrItem {
  long long a1, a2, v, t;  // addresses of A (or A1), A2, V (V2), T tile
  int lda1, lda2, ldv, ldt;
  int m, n, k, pad;        // problem extents (meaning per kernel)
  long long p4, p5;        // extra operand slots (DAG_ITEM tail, unused here)
  int ld4, ld5, aux0, aux1;
};
static_assert(sizeof(QrItem) == 96, "QrItem layout = DAG_ITEM");

template <typename T>
__device__ inline T vget(const T* b, int ld, View v, int i, int j) {
  T x = v.tr ? b[(long long)i * ld + j] : b[i + (long long)j * ld];
  return v.cj ? conj_(x) : x;
}
template <typename T>
__device__ inline void vset(T* b, int ld, View v, int i, int j, T x) {
  x = v.cj ? conj_(x) : x;
  if (v.tr) b[(long long)i * ld + j] = x;
  else b[i + (long long)j * ld] = x;
}
// T tiles are plain column-major
template <typename T>
__device__ inline T& tref(T* b, int ldt, int i, int j) { return b[i + (long long)j * ldt]; }

#define QT 256
template <typename T>
__device__ inline T wg_sum(T x, T* red) {
  const int tid = threadIdx.x;
  red[tid] = x;
  __syncthreads();
  for (int s = QT / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] = add(red[tid], red[tid + s]);
    __syncthreads();
  }
  T r = red[0];
  __syncthreads();
  return r;
}

// Householder generator (LAPACK zlarfg semantics, no over/underflow rescaling):
// given alpha and ||x||^2, returns beta, tau, and the scale 1/(alpha - beta) for x.
template <typename T>
__device__ inline void larfg(T alpha, typename ST<T>::real xnorm2, T& beta_o, T& tau_o, T& scal_o) {
  typedef typename ST<T>::real R;
  const R ar = realv(alpha), ai = imagv(alpha);
  if (xnorm2 == 0 && ai == 0) {
    tau_o = ST<T>::zero();
    beta_o = alpha;
    scal_o = ST<T>::zero();
    return;
  }
  R nrm = sqrt(ar * ar + ai * ai + xnorm2);
  const R beta = ar >= 0 ? -nrm : nrm;
  T tau;
  tau = make_sc<T>((beta - ar) / beta, -ai / beta);
  beta_o = from_real<T>(beta);
  tau_o = tau;
  scal_o = divv(ST<T>::one(), sub(alpha, from_real<T>(beta)));
}

// ------------------------------------------------------------------ GEQRT
// item: a1 = tile A (m x n), t = T tile; extents m, n.  k = min(m, n).
template <typename T>
__global__ __launch_bounds__(QT) void k_geqrt(const QrItem* __restrict__ items, View va, int ib) {
  typedef typename ST<T>::real R;
  __shared__ T red[QT];
  __shared__ T s_w[64];     // per-column dot products within an IB block (ib <= 64)
  __shared__ T s_tau[64];
  const QrItem it = items[blockIdx.x];
  const int m = it.m, n = it.n, kk = min(m, n), tid = threadIdx.x;
  T* Ab = (T*)it.a2;  // A travels in the A2 slot (shared item layout with qr_mfma.hip)
  T* Tb = (T*)it.t;
  const int ao = it.lda2, ldt = it.ldt;
  for (int i0 = 0; i0 < kk; i0 += ib) {
    const int sb = min(ib, kk - i0);
    for (int j = i0; j < i0 + sb; ++j) {
      // ||A(j+1:m, j)||^2
      R part = 0;
      for (int r = j + 1 + tid; r < m; r += QT) {
        const T x = vget(Ab, ao, va, r, j);
        part += realv(mul(conj_(x), x));
      }
      const R xn2 = realv(wg_sum(from_real<T>(part), red));
      T beta, tau, scal;
      larfg(vget(Ab, ao, va, j, j), xn2, beta, tau, scal);
      for (int r = j + 1 + tid; r < m; r += QT) vset(Ab, ao, va, r, j, mul(vget(Ab, ao, va, r, j), scal));
      __syncthreads();
      if (tid == 0) {
        vset(Ab, ao, va, j, j, beta);
        s_tau[j - i0] = tau;
        tref(Tb, ldt, j - i0, j) = tau;
      }
      __syncthreads();
      // apply H^H = I - conj(tau) v v^H to the rest of the IB block
      const int c1 = i0 + sb;
      for (int c = j + 1; c < c1; ++c) {
        T p = ST<T>::zero();
        for (int r = j + tid; r < m; r += QT) {
          const T vr = (r == j) ? ST<T>::one() : vget(Ab, ao, va, r, j);
          p = add(p, mul(conj_(vr), vget(Ab, ao, va, r, c)));
        }
        const T w = wg_sum(p, red);
        const T f = mul(conj_(tau), w);
        for (int r = j + tid; r < m; r += QT) {
          const T vr = (r == j) ? ST<T>::one() : vget(Ab, ao, va, r, j);
          vset(Ab, ao, va, r, c, sub(vget(Ab, ao, va, r, c), mul(vr, f)));
        }
        __syncthreads();
      }
    }
    // T block (zlarft forward columnwise): T(0:jj, j) = -tau_j T(0:jj,0:jj) V(:,0:jj)^H v_j
    for (int jj = 1; jj < sb; ++jj) {
      const int j = i0 + jj;
      // y(a) = V(:, i0+a)^H v_j, a < jj ; rows r >= j (v_j has 1 at row j, zeros above)
      for (int a = 0; a < jj; ++a) {
        T p = ST<T>::zero();
        for (int r = j + tid; r < m; r += QT) {
          const T va_ = vget(Ab, ao, va, r, i0 + a);  // r > i0+a always here (r >= j > i0+a)
          const T vj = (r == j) ? ST<T>::one() : vget(Ab, ao, va, r, j);
          p = add(p, mul(conj_(va_), vj));
        }
        const T y = wg_sum(p, red);
        if (tid == 0) s_w[a] = y;
      }
      __syncthreads();
      if (tid < jj) {
        // T(tid, j) = -tau_j * sum_{b>=tid, b<jj} T(tid, i0+b) y(b)
        T s = ST<T>::zero();
        for (int b = tid; b < jj; ++b) s = add(s, mul(tref(Tb, ldt, tid, i0 + b), s_w[b]));
        tref(Tb, ldt, tid, j) = mul(sub(ST<T>::zero(), s_tau[jj]), s);
      }
      __syncthreads();
    }
    // zero the strictly lower part of the T block (PLASMA leaves it unused; keep it clean)
    for (int e = tid; e < sb * sb; e += QT) {
      const int r = e % sb, c = e / sb;
      if (r > c) tref(Tb, ldt, r, i0 + c) = ST<T>::zero();
    }
    __syncthreads();
    // block reflector on trailing columns: C = A(i0:m, i0+sb:n); W = V^H C; W = T^H W; C -= V W
    for (int c = i0 + sb; c < n; ++c) {
      // W(a) for a < sb
      for (int a = 0; a < sb; ++a) {
        T p = ST<T>::zero();
        for (int r = i0 + a + tid; r < m; r += QT) {
          const T vr = (r == i0 + a) ? ST<T>::one() : vget(Ab, ao, va, r, i0 + a);
          p = add(p, mul(conj_(vr), vget(Ab, ao, va, r, c)));
        }
        const T w = wg_sum(p, red);
        if (tid == 0) s_w[a] = w;
      }
      __syncthreads();
      // W = T^H W  (T upper): (T^H W)(a) = sum_{b<=a} conj(T(b,a)) W(b)
      if (tid < sb) {
        T s = ST<T>::zero();
        for (int b = 0; b <= tid; ++b) s = add(s, mul(conj_(tref(Tb, ldt, b, i0 + tid)), s_w[b]));
        red[tid] = s;
      }
      __syncthreads();
      if (tid < sb) s_w[tid] = red[tid];
      __syncthreads();
      for (int r = i0 + tid; r < m; r += QT) {
        T s = ST<T>::zero();
        for (int a = 0; a < sb && i0 + a <= r; ++a) {
          const T vr = (r == i0 + a) ? ST<T>::one() : vget(Ab, ao, va, r, i0 + a);
          s = add(s, mul(vr, s_w[a]));
        }
        vset(Ab, ao, va, r, c, sub(vget(Ab, ao, va, r, c), s));
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ UNMQR (left)
// C (m x nc) := op(Q) C with Q from a geqrt tile: V (m x k, unit lower), T (ib x k).
// trans: 0 -> Q C (blocks backward, T), 1 -> Q^H C (blocks forward, T^H).
// item: a1 = C tile, v = V tile, t = T tile; m = rows of C (= rows of V), n = cols of C, k = reflectors.
template <typename T>
__global__ __launch_bounds__(QT) void k_unmqr(const QrItem* __restrict__ items, View vc, View vv, int ib,
                                              int conjtrans) {
  __shared__ T Ws[64 * 33];  // W block: sb x (column chunk of 32)
  __shared__ T Tl[64][65];
  const QrItem it = items[blockIdx.x];
  const int m = it.m, nc = it.n, kk = it.k, tid = threadIdx.x;
  T* Cb = (T*)it.a2;  // C travels in the A2 slot (shared item layout with the MFMA kernel)
  const T* Vb = (const T*)it.v;
  const T* Tb = (const T*)it.t;
  const int ldc = it.lda2, ldv = it.ldv, ldt = it.ldt;
  const int nblk = (kk + ib - 1) / ib;
  for (int bi = 0; bi < nblk; ++bi) {
    const int blk = conjtrans ? bi : nblk - 1 - bi;
    const int i0 = blk * ib, sb = min(ib, kk - i0);
    for (int e = tid; e < sb * sb; e += QT) {
      const int r = e % sb, c = e / sb;
      Tl[r][c] = (r <= c) ? Tb[r + (long long)(i0 + c) * ldt] : ST<T>::zero();
    }
    __syncthreads();
    for (int c0 = 0; c0 < nc; c0 += 32) {
      const int cw = min(32, nc - c0);
      // W(a, c) = sum_r conj(V(r, i0+a)) C(r, c0+c), r >= i0+a
      for (int e = tid; e < sb * cw; e += QT) {
        const int a = e % sb, c = e / sb;
        T s = ST<T>::zero();
        for (int r = i0 + a; r < m; ++r) {
          const T vr = (r == i0 + a) ? ST<T>::one() : vget(Vb, ldv, vv, r, i0 + a);
          s = add(s, mul(conj_(vr), vget(Cb, ldc, vc, r, c0 + c)));
        }
        Ws[a * 33 + c] = s;
      }
      __syncthreads();
      // W = op(T) W : op = T^H (conjtrans) or T
      T tmp[8];  // sb*cw <= 64*32 = 8 per thread
      int ne = 0;
      for (int e = tid; e < sb * cw; e += QT, ++ne) {
        const int a = e % sb, c = e / sb;
        T s = ST<T>::zero();
        if (conjtrans) {
          for (int b = 0; b <= a; ++b) s = add(s, mul(conj_(Tl[b][a]), Ws[b * 33 + c]));
        } else {
          for (int b = a; b < sb; ++b) s = add(s, mul(Tl[a][b], Ws[b * 33 + c]));
        }
        tmp[ne] = s;
      }
      __syncthreads();
      ne = 0;
      for (int e = tid; e < sb * cw; e += QT, ++ne) {
        const int a = e % sb, c = e / sb;
        Ws[a * 33 + c] = tmp[ne];
      }
      __syncthreads();
      // C(r, c) -= sum_a V(r, i0+a) W(a, c)
      for (int e = tid; e < (m - i0) * cw; e += QT) {
        const int r = i0 + e % (m - i0), c = e / (m - i0);
        T s = ST<T>::zero();
        for (int a = 0; a < sb && i0 + a <= r; ++a) {
          const T vr = (r == i0 + a) ? ST<T>::one() : vget(Vb, ldv, vv, r, i0 + a);
          s = add(s, mul(vr, Ws[a * 33 + c]));
        }
        vset(Cb, ldc, vc, r, c0 + c, sub(vget(Cb, ldc, vc, r, c0 + c), s));
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ TSQRT / TTQRT
// QR of [A1; A2], A1 (n x n) upper triangular, A2 (m x n) (tri: upper triangular).
// V2 overwrites A2 (for tri only its upper triangle), R overwrites A1, T (ib x n).
// item: a1, a2, t; m = rows of A2, n = cols.
template <typename T>
__global__ __launch_bounds__(QT) void k_tsqrt(const QrItem* __restrict__ items, View v1, View v2, int ib, int tri) {
  typedef typename ST<T>::real R;
  __shared__ T red[QT];
  __shared__ T s_w[64];
  __shared__ T s_tau[64];
  const QrItem it = items[blockIdx.x];
  const int m = it.m, n = it.n, tid = threadIdx.x;
  T* P1 = (T*)it.a1;
  T* P2 = (T*)it.a2;
  T* Tb = (T*)it.t;
  const int ld1 = it.lda1, ld2 = it.lda2, ldt = it.ldt;
  auto A1 = [&](int i, int j) { return vget(P1, ld1, v1, i, j); };
  auto A2 = [&](int i, int j) { return (tri && i > j) ? ST<T>::zero() : vget(P2, ld2, v2, i, j); };
  auto rows2 = [&](int j) { return tri ? min(m, j + 1) : m; };  // rows of column j of V2 that can be nonzero
  for (int i0 = 0; i0 < n; i0 += ib) {
    const int sb = min(ib, n - i0);
    for (int j = i0; j < i0 + sb; ++j) {
      const int mj = rows2(j);
      R part = 0;
      for (int r = tid; r < mj; r += QT) {
        const T x = A2(r, j);
        part += realv(mul(conj_(x), x));
      }
      const R xn2 = realv(wg_sum(from_real<T>(part), red));
      T beta, tau, scal;
      larfg(A1(j, j), xn2, beta, tau, scal);
      for (int r = tid; r < mj; r += QT) vset(P2, ld2, v2, r, j, mul(A2(r, j), scal));
      __syncthreads();
      if (tid == 0) {
        vset(P1, ld1, v1, j, j, beta);
        s_tau[j - i0] = tau;
        tref(Tb, ldt, j - i0, j) = tau;
      }
      __syncthreads();
      // apply H^H to columns c in (j, i0+sb): rows j of A1 and 0..mj-1 of A2
      for (int c = j + 1; c < i0 + sb; ++c) {
        T p = ST<T>::zero();
        for (int r = tid; r < mj; r += QT) p = add(p, mul(conj_(A2(r, j)), A2(r, c)));
        T w = wg_sum(p, red);
        w = add(w, A1(j, c));
        const T f = mul(conj_(tau), w);
        if (tid == 0) vset(P1, ld1, v1, j, c, sub(A1(j, c), f));
        for (int r = tid; r < mj; r += QT) vset(P2, ld2, v2, r, c, sub(A2(r, c), mul(A2(r, j), f)));
        __syncthreads();
      }
    }
    // T block: T(0:jj, j) = -tau_j T(0:jj,0:jj) (V2(:, i0:j)^H v2_j)  (identity parts are orthogonal)
    for (int jj = 1; jj < sb; ++jj) {
      const int j = i0 + jj, mj = rows2(j);
      for (int a = 0; a < jj; ++a) {
        T p = ST<T>::zero();
        for (int r = tid; r < mj; r += QT) p = add(p, mul(conj_(A2(r, i0 + a)), A2(r, j)));
        const T y = wg_sum(p, red);
        if (tid == 0) s_w[a] = y;
      }
      __syncthreads();
      if (tid < jj) {
        T s = ST<T>::zero();
        for (int b = tid; b < jj; ++b) s = add(s, mul(tref(Tb, ldt, tid, i0 + b), s_w[b]));
        tref(Tb, ldt, tid, j) = mul(sub(ST<T>::zero(), s_tau[jj]), s);
      }
      __syncthreads();
    }
    for (int e = tid; e < sb * sb; e += QT) {
      const int r = e % sb, c = e / sb;
      if (r > c) tref(Tb, ldt, r, i0 + c) = ST<T>::zero();
    }
    __syncthreads();
    // apply the block to trailing columns c >= i0+sb: rows i0..i0+sb of A1, all (nonzero) rows of A2
    const int mblk = rows2(i0 + sb - 1);
    for (int c = i0 + sb; c < n; ++c) {
      for (int a = 0; a < sb; ++a) {
        const int ma = rows2(i0 + a);
        T p = ST<T>::zero();
        for (int r = tid; r < ma; r += QT) p = add(p, mul(conj_(A2(r, i0 + a)), A2(r, c)));
        const T w = wg_sum(p, red);
        if (tid == 0) s_w[a] = add(w, A1(i0 + a, c));
      }
      __syncthreads();
      if (tid < sb) {
        T s = ST<T>::zero();
        for (int b = 0; b <= tid; ++b) s = add(s, mul(conj_(tref(Tb, ldt, b, i0 + tid)), s_w[b]));
        red[tid] = s;
      }
      __syncthreads();
      if (tid < sb) {
        s_w[tid] = red[tid];
        vset(P1, ld1, v1, i0 + tid, c, sub(A1(i0 + tid, c), red[tid]));
      }
      __syncthreads();
      for (int r = tid; r < mblk; r += QT) {
        T s = ST<T>::zero();
        for (int a = 0; a < sb; ++a) s = add(s, mul(A2(r, i0 + a), s_w[a]));
        if (!(tri && r > c)) vset(P2, ld2, v2, r, c, sub(A2(r, c), s));
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ TSMQR / TTMQR (left)
// [A1; A2] := op(H) [A1; A2], H from tsqrt: V = [I; V2] (k reflectors), T (ib x k).
// A1 (k rows used) x nc, A2 (m x nc), V2 (m x k) (tri: upper triangular).
// item: a1, a2, v, t; m = rows of A2, n = nc, k.
template <typename T>
__global__ __launch_bounds__(QT) void k_tsmqr(const QrItem* __restrict__ items, View v1, View v2, View vv, int ib,
                                              int conjtrans, int tri) {
  __shared__ T Ws[64 * 33];
  __shared__ T Tl[64][65];
  const QrItem it = items[blockIdx.x];
  const int m = it.m, nc = it.n, kk = it.k, tid = threadIdx.x;
  T* P1 = (T*)it.a1;
  T* P2 = (T*)it.a2;
  const T* Vb = (const T*)it.v;
  const T* Tb = (const T*)it.t;
  const int ld1 = it.lda1, ld2 = it.lda2, ldv = it.ldv, ldt = it.ldt;
  auto V2 = [&](int i, int j) { return (tri && i > j) ? ST<T>::zero() : vget(Vb, ldv, vv, i, j); };
  const int nblk = (kk + ib - 1) / ib;
  for (int bi = 0; bi < nblk; ++bi) {
    const int blk = conjtrans ? bi : nblk - 1 - bi;
    const int i0 = blk * ib, sb = min(ib, kk - i0);
    const int mrows = tri ? min(m, i0 + sb) : m;
    for (int e = tid; e < sb * sb; e += QT) {
      const int r = e % sb, c = e / sb;
      Tl[r][c] = (r <= c) ? Tb[r + (long long)(i0 + c) * ldt] : ST<T>::zero();
    }
    __syncthreads();
    for (int c0 = 0; c0 < nc; c0 += 32) {
      const int cw = min(32, nc - c0);
      // W(a, c) = A1(i0+a, c) + sum_r conj(V2(r, i0+a)) A2(r, c)
      for (int e = tid; e < sb * cw; e += QT) {
        const int a = e % sb, c = e / sb;
        T s = vget(P1, ld1, v1, i0 + a, c0 + c);
        const int ma = tri ? min(m, i0 + a + 1) : m;
        for (int r = 0; r < ma; ++r) s = add(s, mul(conj_(V2(r, i0 + a)), vget(P2, ld2, v2, r, c0 + c)));
        Ws[a * 33 + c] = s;
      }
      __syncthreads();
      T tmp[8];  // sb*cw <= 64*32 = 8 per thread
      int ne = 0;
      for (int e = tid; e < sb * cw; e += QT, ++ne) {
        const int a = e % sb, c = e / sb;
        T s = ST<T>::zero();
        if (conjtrans) {
          for (int b = 0; b <= a; ++b) s = add(s, mul(conj_(Tl[b][a]), Ws[b * 33 + c]));
        } else {
          for (int b = a; b < sb; ++b) s = add(s, mul(Tl[a][b], Ws[b * 33 + c]));
        }
        tmp[ne] = s;
      }
      __syncthreads();
      ne = 0;
      for (int e = tid; e < sb * cw; e += QT, ++ne) {
        const int a = e % sb, c = e / sb;
        Ws[a * 33 + c] = tmp[ne];
        vset(P1, ld1, v1, i0 + a, c0 + c, sub(vget(P1, ld1, v1, i0 + a, c0 + c), tmp[ne]));
      }
      __syncthreads();
      for (int e = tid; e < mrows * cw; e += QT) {
        const int r = e % mrows, c = e / mrows;
        T s = ST<T>::zero();
        for (int a = 0; a < sb; ++a) s = add(s, mul(V2(r, i0 + a), Ws[a * 33 + c]));
        vset(P2, ld2, v2, r, c0 + c, sub(vget(P2, ld2, v2, r, c0 + c), s));
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ launchers
#define DISPATCH(prec, CALL)                                          \
  switch (prec) {                                                     \
    case DPL_S: { typedef float T; CALL; } break;                     \
    case DPL_D: { typedef double T; CALL; } break;                    \
    case DPL_C: { typedef hipFloatComplex T; CALL; } break;           \
    case DPL_Z: { typedef hipDoubleComplex T; CALL; } break;          \
    default: return -2;                                               \
  }

static inline View mkview(int tr, int cj) {
  View v;
  v.tr = tr;
  v.cj = cj;
  return v;
}

// Every launcher: items = device QrItem[nitems]; ib in [1, 64].
DPL_API int dpl_geqrt(int prec, int nitems, const void* items, int a_tr, int a_cj, int ib, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > 64 || ib <= 0) return -3;
  DISPATCH(prec, hipLaunchKernelGGL((k_geqrt<T>), dim3(nitems), dim3(QT), 0, st, (const QrItem*)items,
                                    mkview(a_tr, a_cj), ib));
  return (int)hipGetLastError();
}

DPL_API int dpl_unmqr(int prec, int nitems, const void* items, int c_tr, int c_cj, int v_tr, int v_cj, int ib,
                      int conjtrans, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > 64 || ib <= 0) return -3;
  DISPATCH(prec, hipLaunchKernelGGL((k_unmqr<T>), dim3(nitems), dim3(QT), 0, st, (const QrItem*)items,
                                    mkview(c_tr, c_cj), mkview(v_tr, v_cj), ib, conjtrans));
  return (int)hipGetLastError();
}

DPL_API int dpl_tsqrt(int prec, int nitems, const void* items, int a_tr, int a_cj, int ib, int tri, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > 64 || ib <= 0) return -3;
  DISPATCH(prec, hipLaunchKernelGGL((k_tsqrt<T>), dim3(nitems), dim3(QT), 0, st, (const QrItem*)items,
                                    mkview(a_tr, a_cj), mkview(a_tr, a_cj), ib, tri));
  return (int)hipGetLastError();
}

DPL_API int dpl_tsmqr(int prec, int nitems, const void* items, int a_tr, int a_cj, int v_tr, int v_cj, int ib,
                      int conjtrans, int tri, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > 64 || ib <= 0) return -3;
  DISPATCH(prec, hipLaunchKernelGGL((k_tsmqr<T>), dim3(nitems), dim3(QT), 0, st, (const QrItem*)items,
                                    mkview(a_tr, a_cj), mkview(a_tr, a_cj), mkview(v_tr, v_cj), ib, conjtrans, tri));
  return (int)hipGetLastError();
}
