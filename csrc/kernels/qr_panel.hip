// Householder QR of one tall column-major panel in ONE persistent launch (real precisions).
//
// Reference roles: the panel kernels of the tile QR (CORE_zgeqrt / CORE_ztsqrt chains of
// src/zgeqrf.jdf:98-443, core_zgeqrt.c, core_ztsqrt.c) and the compact-WY T construction of
// LAPACK dlarft.  On MI355X the tile chain (one workgroup walks the panel tile by tile, one
// column at a time) is latency bound, so a TS domain of the elimination tree is factored as
// ONE stacked panel here (models/qr_panel.py), spread over up to one workgroup per CU:
//
//  * rows are partitioned once: workgroup w owns rows [w*R, w*R+R) (R <= 256, one row per
//    thread in the column steps) for the whole launch, so every cross-workgroup hand-off is a
//    small reduction (grid_sync.h) and the matrix itself never crosses workgroups;
//  * 32-column blocks live in LDS.  Column j: every workgroup forms 32 partial dot products of
//    its part of x = A(j+1:, j) with the block columns (c < j: the T column, c == j: ||x||^2,
//    c > j: the reflector's effect) plus a snapshot of row j; ONE grid barrier; every
//    workgroup reduces the partials redundantly, derives beta/tau/scale (dlarfg) and applies
//    the reflector to its rows;
//  * after a block: Y = V_b^T [V_prev | A_rest] is formed with fp64 MFMA (K = the workgroup's
//    rows), reduced in two barriers (each workgroup sums a slice), then A_rest -= V_b T_b^T Y
//    with MFMA, rows stay resident per workgroup; Y's V_prev part is the T coupling input;
//  * the off-diagonal T blocks T(0:b0, blk) = -T(0:b0,0:b0) (V_prev^T V_b) T_b are formed at
//    the end, each workgroup owning T rows w, w+G, ... (no barrier between blocks).
// Output: P holds R (upper) and V (strictly below the diagonal), V holds V explicitly (unit
// diagonal, zeros above) for the trailing GEMMs, Tm the full upper-triangular kf x kf T
// (its strictly-lower part is left untouched: callers keep it zero).
#include "common.h"
#include "grid_sync.h"

#define QP_R 256          // rows per workgroup (max)
#define QP_B 32           // block width
#define QP_LD (QP_R + 2)  // LDS column stride (conflict-free MFMA operand reads)
#define QP_WL (QP_B + 2)

template <typename T> struct QPM;
template <> struct QPM<double> {
  typedef d4_t acc_t;
  static __device__ inline acc_t mma(double x, double y, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) + 4 * r; }
};
template <> struct QPM<float> {
  typedef f4_t acc_t;
  static __device__ inline acc_t mma(float x, float y, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c, 0, 0, 0);
  }
  static __device__ inline int drow(int l, int r) { return (l >> 4) * 4 + r; }
};

// mma(x, y, acc): D(p, q) += sum_k x(p, k) y(q, k); input lane l carries p (resp. q) = l & 15,
// k = l >> 4; output acc[r] of lane l is D(drow(l, r), l & 15).
template <typename T>
__global__ __launch_bounds__(256, 1) void k_qr_panel_persist(T* __restrict__ P, int ldp, int M, int nc, int kf, int R,
                                                             T* __restrict__ V, int ldv, T* __restrict__ Tm, int ldt,
                                                             T* __restrict__ part1, T* __restrict__ part2,
                                                             T* __restrict__ Yg, T* __restrict__ Xc,
                                                             int* __restrict__ cnt, int* __restrict__ info) {
  typedef QPM<T> MM;
  typedef typename MM::acc_t acc_t;
  __shared__ T Ab[QP_B][QP_LD];   // current block columns (later: explicit V_b)
  __shared__ T Xs[QP_B][QP_LD];   // streamed chunk of other columns
  __shared__ T Ts[QP_B][QP_B + 1];  // T_b, Ts[col][row]
  __shared__ T Ws[QP_B][QP_WL];   // Y / T_b^T Y chunk, Ws[col][k]
  __shared__ T red[8][QP_B + 1];
  __shared__ T fin[2 * QP_B];
  __shared__ T ff[QP_B], tv[QP_B];
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int rbase = w * R;
  const int nr = max(0, min(R, M - rbase));
  const int R16 = (nr + 15) & ~15;
  int nsync = 0;
  const int nblk = (kf + QP_B - 1) / QP_B;

  for (int b = 0; b < nblk; ++b) {
    const int b0 = b * QP_B;
    const int cb = min(QP_B, nc - b0);   // block columns held in LDS
    const int bw = min(QP_B, kf - b0);   // of which reflectors
    for (int e = tid; e < QP_B * R16; e += 256) {
      const int c = e / R16, r = e % R16;
      Ab[c][r] = (c < cb && r < nr) ? P[(rbase + r) + (long long)(b0 + c) * ldp] : T(0);
    }
    for (int e = tid; e < QP_B * (QP_B + 1); e += 256) (&Ts[0][0])[e] = T(0);
    __syncthreads();
    // ------------------------------------------------------------ column steps
    for (int jj = 0; jj < bw; ++jj) {
      const int j = b0 + jj;
      const int par = nsync & 1;
      {
        const int c = tid & 31, g = tid >> 5;
        const int rs = j + 1 - rbase;  // first local row strictly below the diagonal
        T s = T(0);
        if (c < cb)
          for (int rl = g; rl < nr; rl += 8)
            if (rl >= rs) s += Ab[jj][rl] * Ab[c][rl];
        red[g][c] = s;
      }
      __syncthreads();
      if (tid < QP_B) {
        T d = T(0);
#pragma unroll
        for (int g = 0; g < 8; ++g) d += red[g][tid];
        const bool own = j >= rbase && j < rbase + nr;
        const T rv = (own && tid < cb) ? Ab[tid][j - rbase] : T(0);
        T* pp = part1 + ((long long)par * G + w) * (2 * QP_B);
        st_sc1(&pp[tid], d);
        st_sc1(&pp[QP_B + tid], rv);
      }
      ++nsync;
      grid_sync_counter(cnt, nsync * G, info);
      {
        const int v = tid & 63, q = tid >> 6;
        T s = T(0);
        for (int bb = q; bb < G; bb += 4) s += ld_sc1(&part1[((long long)par * G + bb) * (2 * QP_B) + v]);
        (&red[0][0])[q * 64 + v] = s;
      }
      __syncthreads();
      if (tid < 2 * QP_B) {
        const T* rf = &red[0][0];
        fin[tid] = (rf[tid] + rf[64 + tid]) + (rf[128 + tid] + rf[192 + tid]);
      }
      __syncthreads();
      // dlarfg (every thread derives the same scalars)
      const T alpha = fin[QP_B + jj], x2 = fin[jj];
      T beta, tau, scale;
      if (x2 == T(0)) {
        beta = alpha;
        tau = T(0);
        scale = T(0);
      } else {
        const T nrm = sqrt(alpha * alpha + x2);
        beta = alpha >= T(0) ? -nrm : nrm;
        tau = (beta - alpha) / beta;
        scale = T(1) / (alpha - beta);
      }
      if (tid < QP_B) {
        const T t = fin[QP_B + tid] + scale * fin[tid];   // v^T A(:, tid) (c > jj), V(:, tid)^T v (c < jj)
        ff[tid] = (tid > jj && tid < cb) ? tau * t : T(0);
        tv[tid] = tid < jj ? t : T(0);
      }
      __syncthreads();
      if (tid < jj) {
        T z = T(0);
        for (int k = tid; k < jj; ++k) z += Ts[k][tid] * tv[k];
        Ts[jj][tid] = -tau * z;
      } else if (tid == jj) {
        Ts[jj][jj] = tau;
      }
      if (tid < nr) {
        const int grow = rbase + tid;
        if (grow > j) {
          const T vr = scale * Ab[jj][tid];
          Ab[jj][tid] = vr;
          for (int c = jj + 1; c < cb; ++c) Ab[c][tid] -= vr * ff[c];
        } else if (grow == j) {
          Ab[jj][tid] = beta;
          for (int c = jj + 1; c < cb; ++c) Ab[c][tid] -= ff[c];
        }
      }
      __syncthreads();
    }
    // ------------------------------------------------------------ block results
    if (w == 0)
      for (int e = tid; e < bw * bw; e += 256) {
        const int i = e % bw, c = e / bw;
        st_sc1(&Tm[(b0 + i) + (long long)(b0 + c) * ldt], i <= c ? Ts[c][i] : T(0));
      }
    for (int e = tid; e < cb * R16; e += 256) {
      const int c = e / R16, r = e % R16;
      const int grow = rbase + r, gc = b0 + c;
      const T a = Ab[c][r];
      T vex = T(0);
      if (r < nr) {
        P[grow + (long long)gc * ldp] = a;
        if (c < bw) {
          vex = grow > gc ? a : (grow == gc ? T(1) : T(0));
          V[grow + (long long)gc * ldv] = vex;
        }
      }
      Ab[c][r] = vex;
    }
    __syncthreads();
    const int nA = nc - b0 - cb;   // trailing panel columns
    const int nX = b0 + nA;        // columns of [V_prev | A_rest]
    if (nX <= 0) continue;
    const bool act = rbase + nr > b0;
    const long long E = (long long)QP_B * nX;
    // ------------------------------------------------------------ Y partials (MFMA, K = own rows)
    for (int x0 = 0; x0 < nX; x0 += QP_B) {
      const int cw = min(QP_B, nX - x0);
      if (act) {
        for (int e = tid; e < QP_B * R16; e += 256) {
          const int c = e / R16, r = e % R16;
          const int grow = rbase + r, xc = x0 + c;
          T v = T(0);
          if (c < cw && r < nr && grow >= b0)
            v = xc < b0 ? V[grow + (long long)xc * ldv] : P[grow + (long long)(cb + xc) * ldp];
          Xs[c][r] = v;
        }
        __syncthreads();
        const int pt = wv & 1, qt = wv >> 1;
        acc_t a0, a1, a2, a3;
#pragma unroll
        for (int r = 0; r < 4; ++r) a0[r] = a1[r] = a2[r] = a3[r] = T(0);
        for (int r0 = 0; r0 < R16; r0 += 16) {
          const int rr = r0 + (l >> 4);
          a0 = MM::mma(Ab[pt * 16 + (l & 15)][rr], Xs[qt * 16 + (l & 15)][rr], a0);
          a1 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 4], Xs[qt * 16 + (l & 15)][rr + 4], a1);
          a2 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 8], Xs[qt * 16 + (l & 15)][rr + 8], a2);
          a3 = MM::mma(Ab[pt * 16 + (l & 15)][rr + 12], Xs[qt * 16 + (l & 15)][rr + 12], a3);
        }
        T* pw = part2 + (long long)w * E;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = pt * 16 + MM::drow(l, r), q = qt * 16 + (l & 15);
          if (q < cw) st_sc1(&pw[(long long)p * nX + x0 + q], (a0[r] + a1[r]) + (a2[r] + a3[r]));
        }
        __syncthreads();
      } else {
        T* pw = part2 + (long long)w * E;
        for (int e = tid; e < QP_B * cw; e += 256) st_sc1(&pw[(long long)(e / cw) * nX + x0 + e % cw], T(0));
      }
    }
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    // ------------------------------------------------------------ Y = sum of partials (slice per workgroup)
    {
      const long long epw = (E + G - 1) / G;
      const long long e_beg = (long long)w * epw, e_end = min(E, e_beg + epw);
      for (long long base = e_beg; base < e_end; base += 32) {
        const long long e = base + (tid & 31);
        const int g = tid >> 5;
        T s = T(0);
        if (e < e_end)
          for (int bb = g; bb < G; bb += 8) s += ld_sc1(&part2[(long long)bb * E + e]);
        red[g][tid & 31] = s;
        __syncthreads();
        if (tid < 32 && e < e_end) {
          T y = T(0);
#pragma unroll
          for (int gg = 0; gg < 8; ++gg) y += red[gg][tid];
          st_sc1(&Yg[e], y);
          const int p = (int)(e / nX), xc = (int)(e % nX);
          if (xc < b0) st_sc1(&Xc[((long long)b * QP_B + p) * kf + xc], y);
        }
        __syncthreads();
      }
    }
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    // ------------------------------------------------------------ A_rest -= V_b (T_b^T Y)
    if (nA > 0 && act) {
      for (int a0 = 0; a0 < nA; a0 += QP_B) {
        const int cw = min(QP_B, nA - a0);
        for (int e = tid; e < QP_B * QP_B; e += 256) {
          const int q = e / QP_B, i = e % QP_B;
          Ws[q][i] = q < cw ? ld_sc1(&Yg[(long long)i * nX + b0 + a0 + q]) : T(0);
        }
        for (int e = tid; e < QP_B * R16; e += 256) {
          const int c = e / R16, r = e % R16;
          const int grow = rbase + r;
          Xs[c][r] = (c < cw && r < nr && grow >= b0) ? P[grow + (long long)(b0 + cb + a0 + c) * ldp] : T(0);
        }
        __syncthreads();
        T o[4];
        {
          const int q = tid & 31, kg = tid >> 5;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int k = kg * 4 + u;
            T z = T(0);
            for (int i = 0; i <= k; ++i) z += Ts[k][i] * Ws[q][i];
            o[u] = z;
          }
        }
        __syncthreads();
        {
          const int q = tid & 31, kg = tid >> 5;
#pragma unroll
          for (int u = 0; u < 4; ++u) Ws[q][kg * 4 + u] = o[u];
        }
        __syncthreads();
        const int RT = R16 / 16;
        for (int t = wv; t < RT * 2; t += 4) {
          const int rt = t >> 1, qt = t & 1;
          acc_t acc;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = Xs[qt * 16 + (l & 15)][rt * 16 + MM::drow(l, r)];
#pragma unroll
          for (int k0 = 0; k0 < QP_B; k0 += 4) {
            const int k = k0 + (l >> 4);
            acc = MM::mma(-Ab[k][rt * 16 + (l & 15)], Ws[qt * 16 + (l & 15)][k], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) Xs[qt * 16 + (l & 15)][rt * 16 + MM::drow(l, r)] = acc[r];
        }
        __syncthreads();
        for (int e = tid; e < cw * R16; e += 256) {
          const int c = e / R16, r = e % R16;
          const int grow = rbase + r;
          if (r < nr && grow >= b0) P[grow + (long long)(b0 + cb + a0 + c) * ldp] = Xs[c][r];
        }
        __syncthreads();
      }
    }
  }
  // ------------------------------------------------------------ off-diagonal T blocks
  if (nblk > 1) {
    ++nsync;
    grid_sync_counter(cnt, nsync * G, info);
    for (int b = 1; b < nblk; ++b) {
      const int b0 = b * QP_B, bw = min(QP_B, kf - b0);
      if (w >= b0) continue;   // owns no T row above this block
      for (int e = tid; e < QP_B * QP_B; e += 256) {
        const int c = e / QP_B, k = e % QP_B;
        Ts[c][k] = (k <= c && c < bw) ? ld_sc1(&Tm[(b0 + k) + (long long)(b0 + c) * ldt]) : T(0);
      }
      for (int e = tid; e < QP_B * b0; e += 256) {
        const int k = e / b0, j = e % b0;
        Ab[k][j] = k < bw ? ld_sc1(&Xc[((long long)b * QP_B + k) * kf + j]) : T(0);
      }
      __syncthreads();
      // Z(j, c) = sum_k X(j, k) T_b(k, c), X = V_prev^T V_b
      for (int e = tid; e < QP_B * b0; e += 256) {
        const int c = e / b0, j = e % b0;
        T z = T(0);
        for (int k = 0; k <= c; ++k) z += Ab[k][j] * Ts[c][k];
        Xs[c][j] = z;
      }
      __syncthreads();
      T* trow = &Ws[0][0];
      for (int i = w; i < b0; i += G) {
        for (int j = tid; j < b0; j += 256) trow[j] = j >= i ? ld_sc1(&Tm[i + (long long)j * ldt]) : T(0);
        __syncthreads();
        const int c = tid & 31, g = tid >> 5;
        T s = T(0);
        for (int j = i + g; j < b0; j += 8) s += trow[j] * Xs[c][j];
        red[g][c] = s;
        __syncthreads();
        if (tid < bw) {
          T t = T(0);
#pragma unroll
          for (int gg = 0; gg < 8; ++gg) t += red[gg][tid];
          st_sc1(&Tm[i + (long long)(b0 + tid) * ldt], -t);
        }
        __syncthreads();
      }
    }
  }
}

static int g_qp_cus = 0;
static int qp_cus() {
  if (g_qp_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_qp_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_qp_cus <= 0) g_qp_cus = 1;
    if (g_qp_cus > 256) g_qp_cus = 256;
  }
  return g_qp_cus;
}

static inline long long qp_align(long long x) { return (x + 255) & ~255LL; }

// Workspace layout (bytes, 256-aligned parts): part1 [2][256][64], part2 [256][32*nc], Yg [32*nc],
// Xc [nblk][32][kf] elements of the precision, then the barrier counter.
DPL_API long long dpl_qr_panel_ws_bytes(int prec, int nc, int kf) {
  const long long es = prec == DPL_D ? 8 : 4;
  const long long nblk = (kf + QP_B - 1) / QP_B;
  return qp_align(es * 2 * 256 * 2 * QP_B) + qp_align(es * 256LL * QP_B * nc) + qp_align(es * QP_B * nc) +
         qp_align(es * nblk * QP_B * kf) + 256;
}

// Largest panel height the single-launch kernel takes (one workgroup per CU, <= 256 rows each).
DPL_API int dpl_qr_panel_max_rows() { return qp_cus() * QP_R; }

DPL_API int dpl_qr_panel(int prec, void* P, int ldp, int M, int nc, int kf, void* V, int ldv, void* Tm, int ldt,
                         void* ws, int* info, hipStream_t st) {
  if (kf <= 0) return 0;
  if (prec != DPL_D && prec != DPL_S) return -2;
  if (kf > M || kf > nc || kf > QP_R || ldp < M || ldv < M || ldt < kf) return -3;
  const int cus = qp_cus();
  int G = (M + QP_R - 1) / QP_R;
  if (G > cus) return -4;
  if (G < 1) G = 1;
  const int R = (M + G - 1) / G;
  const long long es = prec == DPL_D ? 8 : 4;
  const long long nblk = (kf + QP_B - 1) / QP_B;
  char* b = (char*)ws;
  void* part1 = b;
  b += qp_align(es * 2 * 256 * 2 * QP_B);
  void* part2 = b;
  b += qp_align(es * 256LL * QP_B * nc);
  void* Yg = b;
  b += qp_align(es * QP_B * nc);
  void* Xc = b;
  b += qp_align(es * nblk * QP_B * kf);
  int* cnt = (int*)b;
  hipMemsetAsync(cnt, 0, sizeof(int), st);
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_qr_panel_persist<double>), dim3(G), dim3(256), 0, st, (double*)P, ldp, M, nc, kf, R,
                       (double*)V, ldv, (double*)Tm, ldt, (double*)part1, (double*)part2, (double*)Yg, (double*)Xc,
                       cnt, info);
  else
    hipLaunchKernelGGL((k_qr_panel_persist<float>), dim3(G), dim3(256), 0, st, (float*)P, ldp, M, nc, kf, R,
                       (float*)V, ldv, (float*)Tm, ldt, (float*)part1, (float*)part2, (float*)Yg, (float*)Xc, cnt,
                       info);
  return (int)hipGetLastError();
}
