// Householder QR of one tall column-major panel in ONE persistent launch -- complex precisions.
//
// Same schedule as the real kernel (qr_panel.hip; reference roles CORE_zgeqrt / CORE_ztsqrt chains of
// src/zgeqrf.jdf:98-443 and LAPACK zgeqr2 / zlarfg / zlarft): workgroup w owns rows
// [w R, w R + R) of the panel for the whole launch (R <= 256, one row per thread), every column
// step is one grid barrier on the partial dot products, and each block of reflectors is applied
// to the rest of the panel from a cross-workgroup reduction of Y = V_b^H [V_b | V_prev | A_rest].
// Differences for complex data:
//  * 16-column blocks (a complex 256-row block in LDS is twice the bytes of a real one: two
//    16 x 257 complex double blocks + T / W blocks = 144 KB of the 160 KB LDS);
//  * dot products are x^H a, the reflector is zlarfg's (complex tau, real beta), the panel gets
//    H^H = I - conj(tau) v v^H (zgeqr2), the block update A -= V (T^H (V^H A)) and T is zlarft's
//    forward / columnwise T from the Gram block V^H V;
//  * the small block products (Y partials, T^H Y, V W) run on the VALU with complex FMAs: the
//    panel is latency bound, the bulk of the factorisation's flops are the trailing updates on
//    the complex MFMA GEMM engine (zgemm.hip);
//  * values handed across workgroups travel as two agent-scope relaxed scalars (real, imag).
// Output as the real kernel: P holds R (upper) and V (strictly below), V the explicit reflectors
// (unit diagonal, zeros above), Tm the kf x kf upper-triangular T.
#include "common.h"
#include "grid_sync.h"

#define QZ_R 256          // rows per workgroup (max)
#define QZ_B 16           // block width
#define QZ_LD (QZ_R + 1)  // LDS column stride (complex elements)

namespace {

__device__ inline hipDoubleComplex shfl_xor_c(hipDoubleComplex v, int m) {
  return make_hipDoubleComplex(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64));
}
__device__ inline hipFloatComplex shfl_xor_c(hipFloatComplex v, int m) {
  return make_hipFloatComplex(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64));
}
template <typename T> __device__ inline void st_c(T* p, T v) {
  typedef typename ST<T>::real R;
  st_sc1(&((R*)p)[0], v.x);
  st_sc1(&((R*)p)[1], v.y);
}
template <typename T> __device__ inline T ld_c(const T* p) {
  typedef typename ST<T>::real R;
  return make_sc<T>(ld_sc1(&((const R*)p)[0]), ld_sc1(&((const R*)p)[1]));
}
// conj(a) * b + c
template <typename T> __device__ inline T cfma(T a, T b, T c) { return fma_(conj_(a), b, c); }

template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_panel_z(T* __restrict__ P0, int ldp, int rbl, long long rstride, int M,
                                                       int nc, int kf, int R, T* __restrict__ V, int ldv,
                                                       T* __restrict__ Tm, int ldt, T* __restrict__ part1,
                                                       T* __restrict__ rowj, T* __restrict__ part2,
                                                       T* __restrict__ Yg, T* __restrict__ Xc, int* __restrict__ cnt,
                                                       int* __restrict__ info) {
  typedef typename ST<T>::real Rl;
  __shared__ T Ab[QZ_B][QZ_LD];     // finished block columns (R / beta / V), later explicit V_b
  __shared__ T Xs[QZ_B][QZ_LD];     // explicit V_b during the column steps, later streamed chunks
  __shared__ T Ts[QZ_B][QZ_B + 1];  // T_b, Ts[col][row]
  __shared__ T Ws[QZ_B][QZ_B + 1];  // Gram block / Y chunk / T_b^H Y chunk, Ws[col][k]
  __shared__ T red[16][QZ_B + 1];
  __shared__ T fin[2 * QZ_B];
  __shared__ T ff[QZ_B], taus[QZ_B];
  const T zero = ST<T>::zero(), one = ST<T>::one();
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int rbase = w * R;
  const int nr = max(0, min(R, M - rbase));
  const int grow = rbase + tid;
  const bool rowok = tid < nr;
  T* const P = P0 + (long long)(grow / rbl) * rstride + (grow % rbl) - grow;
  int nsync = 0;
  const int nblk = (kf + QZ_B - 1) / QZ_B;

  for (int b = 0; b < nblk; ++b) {
    const int b0 = b * QZ_B;
    const int cb = min(QZ_B, nc - b0);
    const int bw = min(QZ_B, kf - b0);
    T a[QZ_B];   // the row's block, rotated so that the active column is a[0]
#pragma unroll
    for (int c = 0; c < QZ_B; ++c) a[c] = (rowok && c < cb) ? P[grow + (long long)(b0 + c) * ldp] : zero;
    for (int e = tid; e < QZ_B * QZ_LD; e += 256) {
      (&Xs[0][0])[e] = zero;
      (&Ab[0][0])[e] = zero;
    }
    for (int e = tid; e < QZ_B * (QZ_B + 1); e += 256) (&Ts[0][0])[e] = zero;
    __syncthreads();
    // ------------------------------------------------------------ column steps
    for (int jj = 0; jj < bw; ++jj) {
      const int j = b0 + jj;
      const int par = nsync & 1;
      const int sh = QZ_B - jj;   // live slots: slot s is column jj + s
      {
        const T x = (rowok && grow > j) ? a[0] : zero;
        T v[QZ_B];
#pragma unroll
        for (int s = 0; s < QZ_B; ++s) v[s] = s < sh ? mul(conj_(x), a[s]) : zero;
        // wave transpose-reduction: lane l ends with slot l >> 2 summed over its 4-lane group
#pragma unroll
        for (int wdt = QZ_B / 2, m = 32; wdt >= 1; wdt >>= 1, m >>= 1) {
          const bool hi = (l & m) != 0;
#pragma unroll
          for (int i = 0; i < wdt; ++i) {
            const T send = hi ? v[i] : v[wdt + i];
            const T keep = hi ? v[wdt + i] : v[i];
            v[i] = add(keep, shfl_xor_c(send, m));
          }
        }
        v[0] = add(v[0], shfl_xor_c(v[0], 1));
        v[0] = add(v[0], shfl_xor_c(v[0], 2));
        if ((l & 3) == 0) red[wv][l >> 2] = v[0];
        if (rowok && grow == j) {
          T* rj = rowj + par * QZ_B;
#pragma unroll
          for (int s = 0; s < QZ_B; ++s)
            if (s < sh) st_c(&rj[s], a[s]);
        }
      }
      __syncthreads();
      if (tid < QZ_B) {
        const T d = add(add(red[0][tid], red[1][tid]), add(red[2][tid], red[3][tid]));
        st_c(&part1[((long long)par * G + w) * QZ_B + tid], d);
      }
      if (G > 1) {
        ++nsync;
        grid_sync_counter(cnt, nsync * G, info);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      {
        // thread (slot s, group q) sums partials q, q+16, ...
        const int s = tid & 15, q = tid >> 4;
        T acc = zero;
        if (s < sh) {
          const T* src = part1 + (long long)par * G * QZ_B + s;
          for (int bb = q; bb < G; bb += 16) acc = add(acc, ld_c(&src[(long long)bb * QZ_B]));
        }
        red[q][s] = acc;
        if (tid < QZ_B) fin[QZ_B + tid] = tid < sh ? ld_c(&rowj[par * QZ_B + tid]) : zero;
      }
      __syncthreads();
      if (tid < QZ_B) {
        T d = zero;
#pragma unroll
        for (int q = 0; q < 16; ++q) d = add(d, red[q][tid]);
        fin[tid] = d;
      }
      __syncthreads();
      // zlarfg (every thread derives the same scalars); slot 0 is column jj
      const T alpha = fin[QZ_B];
      const Rl x2 = realv(fin[0]);
      const Rl ar = realv(alpha), ai = imagv(alpha);
      T tau, scale;
      Rl beta;
      if (x2 == Rl(0) && ai == Rl(0)) {
        beta = ar;
        tau = zero;
        scale = zero;
      } else {
        const Rl nrm = sqrt(ar * ar + ai * ai + x2);
        beta = ar >= Rl(0) ? -nrm : nrm;
        tau = make_sc<T>((beta - ar) / beta, -ai / beta);
        scale = divv(one, sub(alpha, from_real<T>(beta)));
      }
      if (tid < QZ_B) {
        // H^H a_s = a_s - conj(tau) v (v^H a_s),  v^H a_s = a(j, s) + conj(scale) (x^H a_s)
        ff[tid] = (tid >= 1 && tid < sh && jj + tid < cb)
                      ? mul(conj_(tau), add(fin[QZ_B + tid], mul(conj_(scale), fin[tid])))
                      : zero;
        if (tid == 0) taus[jj] = tau;
      }
      __syncthreads();
      if (rowok) {
        const T x = a[0];
        const T vr = grow > j ? mul(scale, x) : (grow == j ? one : zero);
#pragma unroll
        for (int s = 1; s < QZ_B; ++s) a[s] = sub(a[s], mul(vr, ff[s]));
        Ab[jj][tid] = grow < j ? x : (grow == j ? from_real<T>(beta) : vr);
        Xs[jj][tid] = vr;
      }
#pragma unroll
      for (int s = 0; s < QZ_B - 1; ++s) a[s] = a[s + 1];
      a[QZ_B - 1] = zero;
    }
    if (rowok)
#pragma unroll
      for (int s = 0; s < QZ_B; ++s)
        if (s < cb - bw) Ab[(bw + s) & (QZ_B - 1)][tid] = a[s];
    __syncthreads();
    // ------------------------------------------------------------ block results
    if (rowok) {
#pragma unroll
      for (int c = 0; c < QZ_B; ++c) {
        if (c < cb) P[grow + (long long)(b0 + c) * ldp] = Ab[c][tid];
        if (c < bw) V[grow + (long long)(b0 + c) * ldv] = Xs[c][tid];
      }
    }
    if (tid < nr)
      for (int c = 0; c < QZ_B; ++c) Ab[c][tid] = c < bw ? Xs[c][tid] : zero;
    __syncthreads();
    // ------------------------------------------------------------ Y partials: V_b^H [V_b | V_prev | A_rest]
    const int nA = nc - b0 - cb;
    const int nX = QZ_B + b0 + nA;
    const bool act = rbase + nr > b0;
    const long long E = (long long)QZ_B * nX;
    for (int x0 = 0; x0 < nX; x0 += QZ_B) {
      const int cw = min(QZ_B, nX - x0);
      T* pw = part2 + (long long)w * E;
      if (act) {
        if (tid < nr) {
          const bool live = grow >= b0;
          if (x0 < QZ_B) {
            for (int c = 0; c < QZ_B; ++c) Xs[c][tid] = Ab[c][tid];
          } else {
            const T* src = x0 < QZ_B + b0 ? V + grow + (long long)(x0 - QZ_B) * ldv
                                          : P + grow + (long long)(cb + x0 - QZ_B) * ldp;
            const long long ld = x0 < QZ_B + b0 ? ldv : ldp;
            T t[QZ_B];
#pragma unroll
            for (int c = 0; c < QZ_B; ++c) t[c] = (live && c < cw) ? src[c * ld] : zero;
#pragma unroll
            for (int c = 0; c < QZ_B; ++c) Xs[c][tid] = t[c];
          }
        }
        __syncthreads();
        {
          // thread (p, q) of the 16 x 16 chunk: sum over my rows of conj(V_b(r, p)) X(r, q)
          const int p = tid & 15, q = tid >> 4;
          T s0 = zero, s1 = zero;
          int r = 0;
          for (; r + 1 < nr; r += 2) {
            s0 = cfma(Ab[p][r], Xs[q][r], s0);
            s1 = cfma(Ab[p][r + 1], Xs[q][r + 1], s1);
          }
          if (r < nr) s0 = cfma(Ab[p][r], Xs[q][r], s0);
          if (q < cw) st_c(&pw[(long long)p * nX + x0 + q], add(s0, s1));
        }
        __syncthreads();
      } else {
        const int p = tid & 15, q = tid >> 4;
        if (q < cw) st_c(&pw[(long long)p * nX + x0 + q], zero);
      }
    }
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    // ------------------------------------------------------------ Y = sum of partials
    {
      const long long epw = (E + G - 1) / G;
      const long long e_beg = (long long)w * epw, e_end = min(E, e_beg + epw);
      for (long long base = e_beg; base < e_end; base += 16) {
        const long long e = base + (tid & 15);
        const int g = tid >> 4;
        T s = zero;
        if (e < e_end)
          for (int bb = g; bb < G; bb += 16) s = add(s, ld_c(&part2[(long long)bb * E + e]));
        red[g][tid & 15] = s;
        __syncthreads();
        if (tid < 16 && e < e_end) {
          T y = zero;
#pragma unroll
          for (int gg = 0; gg < 16; ++gg) y = add(y, red[gg][tid]);
          st_c(&Yg[e], y);
          const int p = (int)(e / nX), xc = (int)(e - (long long)p * nX);
          if (xc >= QZ_B && xc < QZ_B + b0) st_c(&Xc[((long long)b * QZ_B + p) * kf + xc - QZ_B], y);
        }
        __syncthreads();
      }
    }
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    // ------------------------------------------------------------ T_b (zlarft) from taus and G = V_b^H V_b
    for (int e = tid; e < QZ_B * QZ_B; e += 256) {
      const int c = e >> 4, k = e & 15;
      Ws[c][k] = ld_c(&Yg[(long long)k * nX + c]);   // G(k, c) = v_k^H v_c
    }
    __syncthreads();
    if (tid < bw) {
      // lane i builds row i of T_b: T(i, j) = -tau_j sum_{k=i}^{j-1} T(i, k) G(k, j)
      const int i = tid;
      Ts[i][i] = taus[i];
      for (int jc = i + 1; jc < bw; ++jc) {
        T z = zero;
        for (int k = i; k < jc; ++k) z = fma_(Ts[k][i], Ws[jc][k], z);
        Ts[jc][i] = mul(make_sc<T>(-realv(taus[jc]), -imagv(taus[jc])), z);
      }
    }
    __syncthreads();
    if (w == 0)
      for (int e = tid; e < bw * bw; e += 256) {
        const int c = e / bw, i = e - c * bw;
        st_c(&Tm[(b0 + i) + (long long)(b0 + c) * ldt], i <= c ? Ts[c][i] : zero);
      }
    // ------------------------------------------------------------ A_rest -= V_b (T_b^H Y)
    if (nA > 0 && act) {
      const int ycol0 = QZ_B + b0;
      for (int a0 = 0; a0 < nA; a0 += QZ_B) {
        const int cw = min(QZ_B, nA - a0);
        for (int e = tid; e < QZ_B * QZ_B; e += 256) {
          const int q = e >> 4, i = e & 15;
          Ws[q][i] = q < cw ? ld_c(&Yg[(long long)i * nX + ycol0 + a0 + q]) : zero;
        }
        if (tid < nr) {
          const bool live = grow >= b0;
          const T* src = P + grow + (long long)(b0 + cb + a0) * ldp;
          T t[QZ_B];
#pragma unroll
          for (int c = 0; c < QZ_B; ++c) t[c] = (live && c < cw) ? src[(long long)c * ldp] : zero;
#pragma unroll
          for (int c = 0; c < QZ_B; ++c) Xs[c][tid] = t[c];
        }
        __syncthreads();
        T o;
        {
          // (T^H Y)(k, q) = sum_{i <= k} conj(T(i, k)) Y(i, q)
          const int q = tid & 15, k = tid >> 4;
          T z = zero;
          for (int i = 0; i <= k; ++i) z = cfma(Ts[k][i], Ws[q][i], z);
          o = z;
        }
        __syncthreads();
        Ws[tid & 15][tid >> 4] = o;
        __syncthreads();
        if (rowok && grow >= b0) {
          T* dst = P + grow + (long long)(b0 + cb + a0) * ldp;
          for (int q = 0; q < cw; ++q) {
            T acc = Xs[q][tid];
#pragma unroll
            for (int k = 0; k < QZ_B; ++k) acc = sub(acc, mul(Ab[k][tid], Ws[q][k]));
            dst[(long long)q * ldp] = acc;
          }
        }
        __syncthreads();
      }
    }
  }
  // ------------------------------------------------------------ off-diagonal T blocks
  // T(i, blk) = -T(i, 0:b0) Z, Z = X_b T_b, X_b = V_prev^H V_b = conj(Y(p, xc))^T; rows w, w+G, ...
  if (nblk > 1) {
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    for (int b = 1; b < nblk; ++b) {
      const int b0 = b * QZ_B, bw = min(QZ_B, kf - b0);
      if (w >= b0) continue;
      for (int e = tid; e < QZ_B * QZ_B; e += 256) {
        const int c = e >> 4, k = e & 15;
        Ts[c][k] = (k <= c && c < bw) ? ld_c(&Tm[(b0 + k) + (long long)(b0 + c) * ldt]) : zero;
      }
      __syncthreads();
      // X_b = conj(Y)^T staged in LDS (Ab is free here), then Z(jx, c) = sum_{k <= c} X_b(jx, k) T_b(k, c)
      for (int e = tid; e < QZ_B * b0; e += 256) {
        const int k = e / b0, jx = e - k * b0;
        Ab[k][jx] = k < bw ? conj_(ld_c(&Xc[((long long)b * QZ_B + k) * kf + jx])) : zero;
      }
      __syncthreads();
      for (int e = tid; e < QZ_B * b0; e += 256) {
        const int c = e / b0, jx = e - c * b0;
        T z = zero;
        for (int k = 0; k <= c; ++k) z = fma_(Ab[k][jx], Ts[c][k], z);
        Xs[c][jx] = z;
      }
      __syncthreads();
      const int nown = (b0 - w + G - 1) / G;
      for (int o = 0; o < nown; ++o) {
        const int i = w + o * G;
        // thread (c, part): partial sum over jx = i + part, i + part + 16, ...
        const int c = tid & 15, part = tid >> 4;
        T s = zero;
        for (int jx = i + part; jx < b0; jx += 16) s = fma_(ld_c(&Tm[i + (long long)jx * ldt]), Xs[c][jx], s);
        red[part][c] = s;
        __syncthreads();
        if (tid < QZ_B && tid < bw) {
          T t = zero;
#pragma unroll
          for (int pp = 0; pp < 16; ++pp) t = add(t, red[pp][tid]);
          st_c(&Tm[i + (long long)(b0 + tid) * ldt], make_sc<T>(-realv(t), -imagv(t)));
        }
        __syncthreads();
      }
    }
  }
}

int g_qz_cus = 0;
int qz_cus() {
  if (g_qz_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_qz_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_qz_cus <= 0) g_qz_cus = 1;
    if (g_qz_cus > 256) g_qz_cus = 256;
  }
  return g_qz_cus;
}

inline long long qz_align(long long x) { return (x + 255) & ~255LL; }

// part1 [2][256][16], rowj [2][16], part2 [256][16 (nc+16)], Yg [16 (nc+16)], Xc [nblk][16][kf], counter
inline void qz_layout(long long es, int nc, int kf, long long off[6]) {
  const long long nblk = (kf + QZ_B - 1) / QZ_B;
  off[0] = 0;
  off[1] = off[0] + qz_align(es * 2 * 256 * QZ_B);
  off[2] = off[1] + qz_align(es * 2 * QZ_B);
  off[3] = off[2] + qz_align(es * 256LL * QZ_B * (nc + QZ_B));
  off[4] = off[3] + qz_align(es * QZ_B * (nc + QZ_B));
  off[5] = off[4] + qz_align(es * nblk * QZ_B * kf);
}

}  // namespace

DPL_API long long dpl_qr_panel_z_ws_bytes(int prec, int nc, int kf) {
  long long off[6];
  qz_layout(prec == DPL_Z ? 16 : 8, nc, kf, off);
  return off[5] + 256;
}

DPL_API int dpl_qr_panel_z(int prec, void* P, int ldp, int rbl, long long rstride, int M, int nc, int kf, void* V,
                           int ldv, void* Tm, int ldt, void* ws, int* info, hipStream_t st) {
  if (kf <= 0) return 0;
  if (prec != DPL_Z && prec != DPL_C) return -2;
  if (rbl <= 0 || rbl >= M) {
    rbl = 1 << 30;
    rstride = 0;
    if (ldp < M) return -3;
  } else if (ldp < rbl) {
    return -3;
  }
  if (kf > M || kf > nc || kf > QZ_R || ldv < M || ldt < kf) return -3;
  int G = (M + QZ_R - 1) / QZ_R;
  if (G > qz_cus()) return -4;
  if (G < 1) G = 1;
  const int R = (M + G - 1) / G;
  long long off[6];
  qz_layout(prec == DPL_Z ? 16 : 8, nc, kf, off);
  char* b = (char*)ws;
  void *part1 = b + off[0], *rowj = b + off[1], *part2 = b + off[2], *Yg = b + off[3], *Xc = b + off[4];
  int* cnt = (int*)(b + off[5]);
  if (hipMemsetAsync(cnt, 0, sizeof(int), st) != hipSuccess) return -1;
  if (prec == DPL_Z)
    hipLaunchKernelGGL((k_qr_panel_z<hipDoubleComplex>), dim3(G), dim3(256), 0, st, (hipDoubleComplex*)P, ldp, rbl,
                       rstride, M, nc, kf, R, (hipDoubleComplex*)V, ldv, (hipDoubleComplex*)Tm, ldt,
                       (hipDoubleComplex*)part1, (hipDoubleComplex*)rowj, (hipDoubleComplex*)part2,
                       (hipDoubleComplex*)Yg, (hipDoubleComplex*)Xc, cnt, info);
  else
    hipLaunchKernelGGL((k_qr_panel_z<hipFloatComplex>), dim3(G), dim3(256), 0, st, (hipFloatComplex*)P, ldp, rbl,
                       rstride, M, nc, kf, R, (hipFloatComplex*)V, ldv, (hipFloatComplex*)Tm, ldt,
                       (hipFloatComplex*)part1, (hipFloatComplex*)rowj, (hipFloatComplex*)part2,
                       (hipFloatComplex*)Yg, (hipFloatComplex*)Xc, cnt, info);
  return (int)hipGetLastError();
}
