// MFMA block-reflector application for the QR family (real precisions).
//
// Covers CORE_ztsmqr / CORE_zttmqr / CORE_zunmqr (core_ztsmqr.c:124,
// core_zttmqr.c:116, core_zunmqr.c:108) -- the dominant flops of geqrf
// (the reference's CUDA path loops cublas calls per IB
// block; here the whole IB loop runs inside one kernel).
//
// One workgroup (256 threads, 4 waves) owns one 32-column chunk of one item:
//   * the A2 chunk (m <= 256 rows x 32 columns) stays resident in LDS for the
//     whole IB loop; it is read from HBM once and written once;
//   * per IB block (<= 32 reflectors) the V block is staged in LDS with the
//     mode's structure applied (TS: full, TT: upper triangle, UNMQR: unit
//     lower), T is staged upper-triangular, then
//        W  = A1(blk rows, chunk) + V^H A2      (MFMA, K = m)
//        W  = op(T) W                            (MFMA, K = ib)
//        A1(blk rows, chunk) -= W                (straight from accumulators)
//        A2 -= V W                               (MFMA, K = ib; acc = A2 tile)
//   * v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32, operand roles arranged so
//     the accumulator lane index runs along rows (column-major friendly);
//   * the item's chunks are consecutive block ids, remapped XCD-aware so the
//     chunks sharing V/T hit the same L2.
// Items / views are those of qr.hip (absolute addresses, per-operand ld).
#include "common.h"

struct View2 {
  int tr, cj;
};
struct QrItemM {
  long long a1, a2, v, t;
  int lda1, lda2, ldv, ldt;
  int m, n, k, pad;
  long long p4, p5;
  int ld4, ld5, aux0, aux1;
};
static_assert(sizeof(QrItemM) == 96, "QrItemM layout = DAG_ITEM");

template <typename T>
__device__ inline T vld(const T* b, int ld, View2 v, int i, int j) {
  return v.tr ? b[(long long)i * ld + j] : b[i + (long long)j * ld];
}
template <typename T>
__device__ inline void vst(T* b, int ld, View2 v, int i, int j, T x) {
  if (v.tr) b[(long long)i * ld + j] = x;
  else b[i + (long long)j * ld] = x;
}

template <typename T> struct QMF;
template <> struct QMF<double> {
  typedef d4_t acc_t;
  static __device__ inline acc_t mma(double x, double y, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) + 4 * r; }
};
template <> struct QMF<float> {
  typedef f4_t acc_t;
  static __device__ inline acc_t mma(float x, float y, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) * 4 + r; }
};

#define QM_CW 32    // columns per workgroup
#define QM_MR 256   // max rows of A2 / V
#define QM_IB 32    // max inner block
#define QM_LDM (QM_MR + 2)
#define QM_LDW (QM_IB + 2)

// One IB block applied to one LDS-resident A2 chunk (columns c0.. of the item):
//   W = A1(i0.., chunk) + V^H A2 ; W = op(T) W ; A1 -= W ; A2 -= V W.
// Vs holds the structured V block (zeros where V is structurally zero), Ts the
// upper-triangular T block.  A1 == nullptr: no A1 term (UNMQR / GEQRT mode).
// Caller guarantees Vs/Ts/A2s are complete (barrier before the call); returns
// after a barrier with A2s updated.
// a1pre: the A1 values of this lane's W entries, already loaded (or nullptr: load here).
template <typename T>
__device__ inline void apply_block(T (*A2s)[QM_LDM], const T (*Vs)[QM_LDM], T (*Ws)[QM_LDW], const T (*Ts)[QM_LDW],
                                   int mp, int sb, int conjtrans, T* A1, int lda1, View2 va, int i0, int c0, int cw,
                                   const T* a1pre = nullptr) {
  typedef QMF<T> M_;
  typedef typename M_::acc_t acc_t;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int ta = (w & 1) * 16, tc = (w >> 1) * 16;
  acc_t acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int a = ta + (l & 15), c = tc + M_::drow(l, r);
    acc[r] = a1pre ? a1pre[r] : ((A1 && a < sb && c < cw) ? vld(A1, lda1, va, i0 + a, c0 + c) : T(0));
  }
  {
    // four independent accumulation chains over the row range (more MFMA/LDS overlap)
    acc_t acc1, acc2, acc3;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc1[r] = acc2[r] = acc3[r] = T(0);
    int r0 = 0;
    for (; r0 + 16 <= mp; r0 += 16) {
      const int rr = r0 + (l >> 4);
      const T x0 = A2s[tc + (l & 15)][rr], y0 = Vs[ta + (l & 15)][rr];
      const T x1 = A2s[tc + (l & 15)][rr + 4], y1 = Vs[ta + (l & 15)][rr + 4];
      const T x2 = A2s[tc + (l & 15)][rr + 8], y2 = Vs[ta + (l & 15)][rr + 8];
      const T x3 = A2s[tc + (l & 15)][rr + 12], y3 = Vs[ta + (l & 15)][rr + 12];
      acc = M_::mma(x0, y0, acc);
      acc1 = M_::mma(x1, y1, acc1);
      acc2 = M_::mma(x2, y2, acc2);
      acc3 = M_::mma(x3, y3, acc3);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] += acc1[r] + acc2[r] + acc3[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) Ws[tc + M_::drow(l, r)][ta + (l & 15)] = acc[r];
  __syncthreads();
  {
    acc_t t2;
#pragma unroll
    for (int r = 0; r < 4; ++r) t2[r] = T(0);
    for (int b0 = 0; b0 < QM_IB; b0 += 4) {
      const int b = b0 + (l >> 4), a = ta + (l & 15);
      const T opT = conjtrans ? Ts[a][b] : Ts[b][a];  // T^H(a,b) = T(b,a) = Ts[a][b]; T(a,b) = Ts[b][a]
      t2 = M_::mma(Ws[tc + (l & 15)][b], opT, t2);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = ta + (l & 15), c = tc + M_::drow(l, r);
      Ws[c][a] = t2[r];
      if (A1 && a < sb && c < cw) {
        const T old = a1pre ? a1pre[r] : vld(A1, lda1, va, i0 + a, c0 + c);
        vst(A1, lda1, va, i0 + a, c0 + c, old - t2[r]);
      }
    }
  }
  __syncthreads();
  for (int rt = w; rt < mp / 16; rt += 4) {
#pragma unroll
    for (int ct = 0; ct < QM_CW; ct += 16) {
      acc_t a2;
#pragma unroll
      for (int r = 0; r < 4; ++r) a2[r] = A2s[ct + M_::drow(l, r)][rt * 16 + (l & 15)];
#pragma unroll
      for (int a0 = 0; a0 < QM_IB; a0 += 4) {
        const int a = a0 + (l >> 4);
        a2 = M_::mma(Ws[ct + (l & 15)][a], -Vs[a][rt * 16 + (l & 15)], a2);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) A2s[ct + M_::drow(l, r)][rt * 16 + (l & 15)] = a2[r];
    }
  }
  __syncthreads();
}

template <typename T>
__device__ inline void load_chunk(T (*A2s)[QM_LDM], const T* A2, int lda2, View2 va, int m, int mp, int c0, int cw) {
  for (int e = threadIdx.x; e < QM_CW * mp; e += 256) {
    const int c = e / mp, r = e % mp;
    A2s[c][r] = (r < m && c < cw) ? vld(A2, lda2, va, r, c0 + c) : T(0);
  }
}
template <typename T>
__device__ inline void store_chunk(const T (*A2s)[QM_LDM], T* A2, int lda2, View2 va, int m, int mp, int c0, int cw) {
  for (int e = threadIdx.x; e < QM_CW * mp; e += 256) {
    const int c = e / mp, r = e % mp;
    if (r < m && c < cw) vst(A2, lda2, va, r, c0 + c, A2s[c][r]);
  }
}
template <typename T>
__device__ inline void load_T(T (*Ts)[QM_LDW], const T* Tt, int ldt, int i0, int sb) {
  for (int e = threadIdx.x; e < QM_IB * QM_IB; e += 256) {
    const int col = e / QM_IB, row = e % QM_IB;
    Ts[col][row] = (row <= col && col < sb) ? Tt[row + (long long)(i0 + col) * ldt] : T(0);
  }
}

// mode: 0 TS (A1 present, V2 full), 1 TT (A1 present, V2 upper), 2 UNMQR (no A1, V unit lower)
// The next IB block's V, T and A1 values are prefetched into registers while
// the current block computes (one wave per SIMD: registers are plentiful).
template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_apply_mfma(const QrItemM* __restrict__ items, int nchunk, int nwg,
                                                          View2 va, View2 vv, int ib, int conjtrans, int mode) {
  typedef QMF<T> M_;
  __shared__ T A2s[QM_CW][QM_LDM];
  __shared__ T Vs[QM_IB][QM_LDM];
  __shared__ T Ws[QM_CW][QM_LDW];
  __shared__ T Ts[QM_IB][QM_LDW];
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int item = bid / nchunk, chunk = bid % nchunk;
  const QrItemM it = items[item];
  const int m = it.m, kk = it.k;
  const int c0 = chunk * QM_CW;
  if (c0 >= it.n) return;
  const int cw = min(QM_CW, it.n - c0);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  T* A1 = mode == 2 ? nullptr : (T*)it.a1;
  T* A2 = (T*)it.a2;
  const T* V = (const T*)it.v;
  const T* Tt = (const T*)it.t;
  const int mp = (m + 15) & ~15;  // rows padded to 16
  const int nblk = (kk + ib - 1) / ib;
  const int ta = (w & 1) * 16, tc = (w >> 1) * 16;
  T vreg[QM_IB * QM_MR / 256];
  T treg[QM_IB * QM_IB / 256];
  T areg[4];
  auto fetch = [&](int bi) {
    const int blk = conjtrans ? bi : nblk - 1 - bi;
    const int i0 = blk * ib, sb = min(ib, kk - i0);
#pragma unroll
    for (int q = 0; q < QM_IB * QM_MR / 256; ++q) {
      const int e = tid + 256 * q;
      const int a = e / mp, r = e % mp;
      T x = T(0);
      if (e < QM_IB * mp && a < sb && r < m) {
        const int ag = i0 + a;
        if (mode == 0) x = vld(V, it.ldv, vv, r, ag);
        else if (mode == 1) x = (r <= ag) ? vld(V, it.ldv, vv, r, ag) : T(0);
        else x = (r == ag) ? T(1) : (r > ag ? vld(V, it.ldv, vv, r, ag) : T(0));
      }
      vreg[q] = x;
    }
#pragma unroll
    for (int q = 0; q < QM_IB * QM_IB / 256; ++q) {
      const int e = tid + 256 * q;
      const int col = e / QM_IB, row = e % QM_IB;
      treg[q] = (row <= col && col < sb) ? Tt[row + (long long)(i0 + col) * it.ldt] : T(0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = ta + (l & 15), c = tc + M_::drow(l, r);
      areg[r] = (A1 && a < sb && c < cw) ? vld(A1, it.lda1, va, i0 + a, c0 + c) : T(0);
    }
  };
  fetch(0);
  load_chunk(A2s, A2, it.lda2, va, m, mp, c0, cw);
  for (int bi = 0; bi < nblk; ++bi) {
    const int blk = conjtrans ? bi : nblk - 1 - bi;
    const int i0 = blk * ib, sb = min(ib, kk - i0);
    // registers -> LDS (the previous block finished with Vs / Ts: apply_block ends with a barrier)
#pragma unroll
    for (int q = 0; q < QM_IB * QM_MR / 256; ++q) {
      const int e = tid + 256 * q;
      if (e < QM_IB * mp) Vs[e / mp][e % mp] = vreg[q];
    }
#pragma unroll
    for (int q = 0; q < QM_IB * QM_IB / 256; ++q) {
      const int e = tid + 256 * q;
      Ts[e / QM_IB][e % QM_IB] = treg[q];
    }
    T a1cur[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) a1cur[r] = areg[r];
    __syncthreads();
    if (bi + 1 < nblk) fetch(bi + 1);  // in flight during this block's MFMA work
    apply_block(A2s, Vs, Ws, Ts, mp, sb, conjtrans, A1, it.lda1, va, i0, c0, cw, a1cur);
  }
  store_chunk(A2s, A2, it.lda2, va, m, mp, c0, cw);
}

// ------------------------------------------------------------------ panel kernels (GEQRT, TSQRT, TTQRT)
template <typename T>
__device__ inline T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
// block-wide sum over 256 threads; red4 has 4 slots; ends with all threads holding the sum
template <typename T>
__device__ inline T block_sum(T x, T* red4) {
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = x;
  __syncthreads();
  const T r = red4[0] + red4[1] + red4[2] + red4[3];
  __syncthreads();
  return r;
}

// Factor one IB-column block held in Vs (column a = global column i0+a of the tile).
//   geqrt (ts=false): column j's reflector acts on rows >= jr = i0+j: alpha = A(jr, j),
//          x = rows > jr; the R part lies above.
//   tsqrt: alpha = R1[j][j] (A1 diagonal block), x = Vs[j][0..re) with
//          re = tri ? min(m, jr+1) : m.
// Two barriers per column: phase 1 computes, per (column c, row segment), the
// partial dot products d_c = sum x_r A(r, c) -- c = j gives ||x||^2 -- and
// snapshots A(jr, c); phase 2 lets every thread derive tau / scale redundantly
// and apply  A(r, c) -= v_r f_c  with  f_c = tau (A(jr, c) + scale d_c),
// v_r = scale x_r, while the column-j threads scale x in place.  A segment's
// rows belong to one wave, so a wave reads x_r before it overwrites it.
template <typename T>
__device__ inline void factor_block(T (*Vs)[QM_LDM], T (*R1)[QM_LDW], T (*Red)[33], T* tau, T* red4, int m, int i0,
                                    int sb, bool ts, bool tri) {
  const int tid = threadIdx.x;
  const int c = tid & 31, seg = tid >> 5;
  (void)red4;
  for (int j = 0; j < sb; ++j) {
    const int jr = i0 + j;
    const int rb = ts ? 0 : jr + 1;
    const int re = ts ? (tri ? min(m, jr + 1) : m) : m;
    const int cc = j + c;
    // ---- phase 1
    T p = T(0);
    if (cc < sb)
      for (int r = rb + seg; r < re; r += 8) p += Vs[j][r] * Vs[cc][r];
    Red[seg][c] = p;
    if (seg == 0 && cc < sb) Red[8][c] = ts ? R1[j][cc] : Vs[cc][jr];
    __syncthreads();
    // ---- phase 2 (every thread: tau, scale)
    T xn2 = T(0);
#pragma unroll
    for (int q = 0; q < 8; ++q) xn2 += Red[q][0];
    const T alpha = Red[8][0];
    T beta = alpha, tj = T(0), scal = T(0);
    if (xn2 != T(0)) {
      const T nrm = sqrt(alpha * alpha + xn2);
      beta = alpha >= T(0) ? -nrm : nrm;
      tj = (beta - alpha) / beta;
      scal = T(1) / (alpha - beta);
    }
    if (c != 0 && cc < sb) {
      T d = T(0);
#pragma unroll
      for (int q = 0; q < 8; ++q) d += Red[q][c];
      const T f = tj * (Red[8][c] + scal * d);
      const T fs = f * scal;
      for (int r = rb + seg; r < re; r += 8) Vs[cc][r] -= Vs[j][r] * fs;
      if (seg == 0) {
        if (ts) R1[j][cc] -= f;
        else Vs[cc][jr] -= f;
      }
    }
    // after the reconvergence point: every lane of this wave has read x_r already
    if (c == 0) {
      for (int r = rb + seg; r < re; r += 8) Vs[j][r] *= scal;
      if (seg == 0) {
        tau[j] = tj;
        if (ts) R1[j][j] = beta;
        else Vs[j][jr] = beta;
      }
    }
    __syncthreads();
  }
}

// T block from the taus and the Gram matrix of the (structured) V block: T(0:j, j) = -tau_j T(0:j,0:j) y_j
template <typename T>
__device__ inline void build_T(const T (*Vs)[QM_LDM], T (*Ts)[QM_LDW], T (*G)[33], const T* tau, int mp, int sb,
                               bool ts) {
  const int tid = threadIdx.x;
  // G(a, j) = V(:, a)^T V(:, j) for a < j (TS: identity parts are orthogonal, V = V2 only)
  for (int e = tid; e < QM_IB * QM_IB; e += 256) {
    const int a = e % QM_IB, j = e / QM_IB;
    T s = T(0);
    if (a < j && j < sb)
      for (int r = 0; r < mp; ++r) s += Vs[a][r] * Vs[j][r];
    G[a][j] = s;
  }
  for (int e = tid; e < QM_IB * QM_IB; e += 256) Ts[e / QM_IB][e % QM_IB] = T(0);
  __syncthreads();
  for (int j = 0; j < sb; ++j) {
    if (tid < j) {
      T s = T(0);
      for (int b = tid; b < j; ++b) s += Ts[b][tid] * G[b][j];  // Ts[col][row]
      Ts[j][tid] = -tau[j] * s;
    }
    if (tid == 0) Ts[j][j] = tau[j];
    __syncthreads();
  }
  (void)ts;
}

// GEQRT (ts=false) / TSQRT (ts=true, tri=false) / TTQRT (ts=true, tri=true), one item per workgroup.
//   geqrt: item.a2 = A (m x n), t = T ; tsqrt: item.a1 = A1 (n x n), a2 = A2 (m x n), t = T.
template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_panel_mfma(const QrItemM* __restrict__ items, View2 va, int ib, int ts,
                                                          int tri) {
  __shared__ T A2s[QM_CW][QM_LDM];
  __shared__ T Vs[QM_IB][QM_LDM];
  __shared__ T Ws[QM_CW][QM_LDW];
  __shared__ T Ts[QM_IB][QM_LDW];
  __shared__ T R1[QM_IB][QM_LDW];
  __shared__ T tau[QM_IB];
  __shared__ T red4[4];
  T (*Red)[33] = reinterpret_cast<T (*)[33]>(&A2s[0][0]);  // scratch while A2s is idle
  T (*G)[33] = reinterpret_cast<T (*)[33]>(&Ws[0][0]);
  const QrItemM it = items[blockIdx.x];
  const int m = it.m, n = it.n, tid = threadIdx.x;
  const int kk = ts ? n : min(m, n);
  T* A = (T*)it.a2;
  T* A1 = ts ? (T*)it.a1 : nullptr;
  T* Tt = (T*)it.t;
  const int mp = (m + 15) & ~15;
  for (int i0 = 0; i0 < kk; i0 += ib) {
    const int sb = min(ib, kk - i0);
    // ---- stage the block columns (and the A1 diagonal block)
    for (int e = tid; e < QM_IB * mp; e += 256) {
      const int a = e / mp, r = e % mp;
      T x = T(0);
      if (a < sb && r < m && !(tri && r > i0 + a)) x = vld(A, it.lda2, va, r, i0 + a);
      Vs[a][r] = x;
    }
    if (ts)
      for (int e = tid; e < QM_IB * QM_IB; e += 256) {
        const int a = e / QM_IB, b = e % QM_IB;  // R1[a][b] = A1(i0+a, i0+b)
        R1[a][b] = (a < sb && b < sb) ? vld(A1, it.lda1, va, i0 + a, i0 + b) : T(0);
      }
    __syncthreads();
    factor_block(Vs, R1, Red, tau, red4, m, i0, sb, ts, tri);
    // ---- write the factored block back (geqrt: R above / beta / V below; ts: V2 and R1 block)
    for (int e = tid; e < sb * m; e += 256) {
      const int a = e / m, r = e % m;
      if (!(tri && r > i0 + a)) vst(A, it.lda2, va, r, i0 + a, Vs[a][r]);
    }
    if (ts)
      for (int e = tid; e < sb * sb; e += 256) {
        const int a = e / sb, b = e % sb;
        if (a <= b) vst(A1, it.lda1, va, i0 + a, i0 + b, R1[a][b]);
      }
    __syncthreads();
    // ---- structured V for the Gram matrix / trailing update (geqrt: unit lower from row i0+a)
    if (!ts)
      for (int e = tid; e < QM_IB * mp; e += 256) {
        const int a = e / mp, r = e % mp;
        if (a < sb) Vs[a][r] = (r < i0 + a) ? T(0) : (r == i0 + a ? T(1) : Vs[a][r]);
      }
    __syncthreads();
    build_T(Vs, Ts, G, tau, mp, sb, ts);
    for (int e = tid; e < sb * sb; e += 256) {
      const int row = e % sb, col = e / sb;
      Tt[row + (long long)(i0 + col) * it.ldt] = row <= col ? Ts[col][row] : T(0);
    }
    __syncthreads();
    // ---- trailing columns i0+sb .. n-1, 32 at a time: [A1 rows i0..; A] -= block reflector
    for (int c0 = i0 + sb; c0 < n; c0 += QM_CW) {
      const int cw = min(QM_CW, n - c0);
      load_chunk(A2s, A, it.lda2, va, m, mp, c0, cw);
      __syncthreads();
      apply_block(A2s, Vs, Ws, Ts, mp, sb, 1, A1, it.lda1, va, i0, c0, cw);
      // TT: columns c0.. are right of the diagonal block, rows < mp all belong to the triangle
      store_chunk(A2s, A, it.lda2, va, m, mp, c0, cw);
      __syncthreads();
    }
  }
}

DPL_API int dpl_qr_panel_mfma(int prec, int nitems, const void* items, int a_tr, int ib, int ts, int tri,
                              hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > QM_IB || ib <= 0) return -3;
  View2 va{a_tr, 0};
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_qr_panel_mfma<double>), dim3(nitems), dim3(256), 0, st, (const QrItemM*)items, va, ib, ts,
                       tri);
  else if (prec == DPL_S)
    hipLaunchKernelGGL((k_qr_panel_mfma<float>), dim3(nitems), dim3(256), 0, st, (const QrItemM*)items, va, ib, ts,
                       tri);
  else
    return -2;
  return (int)hipGetLastError();
}

DPL_API int dpl_qr_apply_mfma_ok(int prec, int max_m, int ib) {
  return (prec == DPL_D || prec == DPL_S) && max_m <= QM_MR && ib <= QM_IB && ib > 0;
}

// items: device QrItemM[nitems]; mode 0 TS, 1 TT, 2 UNMQR (A1 unused); max_n = widest item
DPL_API int dpl_qr_apply_mfma(int prec, int nitems, const void* items, int max_n, int a_tr, int v_tr, int ib,
                              int conjtrans, int mode, hipStream_t st) {
  if (nitems <= 0) return 0;
  if (ib > QM_IB || ib <= 0) return -3;
  const int nchunk = cdiv(max_n, QM_CW);
  const int nwg = nitems * nchunk;
  View2 va{a_tr, 0}, vv{v_tr, 0};
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_qr_apply_mfma<double>), dim3(nwg), dim3(256), 0, st, (const QrItemM*)items, nchunk, nwg, va,
                       vv, ib, conjtrans, mode);
  else if (prec == DPL_S)
    hipLaunchKernelGGL((k_qr_apply_mfma<float>), dim3(nwg), dim3(256), 0, st, (const QrItemM*)items, nchunk, nwg, va,
                       vv, ib, conjtrans, mode);
  else
    return -2;
  return (int)hipGetLastError();
}
