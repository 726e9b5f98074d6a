// Dataflow Cholesky of one diagonal tile over ceil(n/32) cooperating workgroups: the shared body of
// k_potrf_rb / k_potrf_trsm_rb (potrf_rb.hip, where the algorithm is described) and of the
// device task runtime's POTRF tasks (dtr.hip).  LDS is passed in so a persistent kernel can
// overlay it with its other task bodies.
#pragma once
#include "common.h"
#include "grid_sync.h"

namespace rbk {
constexpr int RB = 32;            // row-block height
constexpr int MAXB = 16;          // at most 16 row blocks (n <= 512)
constexpr int BLK = RB * RB;      // doubles per block
constexpr int PSTRIDE = 32;       // ints between flags (one 128-B line each)
constexpr int NSLOT = 8;          // workspaces, one per stream that launches the kernel (get_ws)
#ifndef RB_PRIO
#define RB_PRIO 3                 // wave priority of the critical-path kernels (0..3)
#endif

struct RbWork {
  double* M;    // [MAXB][BLK]        M_k, column-major: inv(L(k,k)) = diag(S_k) M_k
  double* S;    // [MAXB][RB]         S_k
  double* Lp;   // [MAXB][MAXB][BLK]  L(i,k), T-layout
  int* prog;    // [MAXB * PSTRIDE]   epoch * 64 + number of published steps
  unsigned* ticket;  // workgroup start tickets (monotonic over the slot's launches)
  unsigned tbase;    // value of *ticket when this launch's first workgroup starts
};

// logical workgroup id = order of start (one atomic per workgroup); see the header comment
__device__ inline int wg_ticket(const RbWork& ws) {
  __shared__ int sid;
  if (threadIdx.x == 0) sid = (int)(atomicAdd(ws.ticket, 1u) - ws.tbase);
  __syncthreads();
  return sid;
}
// caller-visible copy of (M, S) for the panel TRSM (dpl_trsm_rb): MAXB * (BLK + RB) doubles
constexpr int ZBUF = MAXB * (BLK + RB);

__device__ inline int tl_index(int rho, int gam) {  // T-layout index of element (rho, gam) of a block
  const int q = ((rho >> 4) << 1) | (gam >> 4), g = gam & 15;
  return ((q * 4 + (g >> 2)) * 64) + (rho & 15) + 16 * (g & 3);
}

__device__ inline double readlane_d(double v, int lane) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, lane);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline double rcp_d(double d) {  // 1/d to full precision (hardware estimate + 2 Newton steps)
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  return r;
}

__device__ inline double rsqrt_d(double d) {  // 1/sqrt(d) (hardware estimate + 2 Newton steps)
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}

// Bounded spin on an epoch-tagged flag; once any spin of the launch has timed out (info = -1000)
// every later spin returns at once, so a broken schedule drains instead of hanging.
__device__ inline void spin_until(const int* flag, int target, int* info) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_sc1(flag) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (info && ld_sc1(info) == -1000) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ULL) {  // 100 MHz clock: 2 s
      if (info) atomicExch(info, -1000);
      return;
    }
  }
}

__device__ inline void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// two 8-byte agent-scope stores (sc1, write-through); drained by drain_stores().  Compiler-generated on purpose:
// the former inline-asm global_store_dwordx4 was invisible to the compiler's hazard recognizer, which then let the
// next VALU rewrite the store's address VGPRs in the following instruction -- with two workgroups per CU (two waves
// per SIMD interleaving) the published M_k came out wrong in a few % of DTR runs while everything the workgroup kept
// for itself was right (profiles/r6_dtr_coresidency_rootcause.txt: post-mortem of the published blocks).
__device__ inline void st_sc1_x2(double* p, double a, double b) {
  __hip_atomic_store(p, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// acc += sum_u Y(u) X(u): A operand Y, B operand X (T-layout chunks)
template <int NU>
__device__ inline d4_t mfma_chunks(const double* y, const double* x, d4_t acc) {
#pragma unroll
  for (int u = 0; u < NU; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(y[u], x[u], acc, 0, 0, 0);
  return acc;
}

// T-layout offset of (row half h, k-chunk u) for this lane
__device__ inline int qoff(int h, int u, int l) { return ((h * 2 + (u >> 2)) * 4 + (u & 3)) * 64 + l; }

// optional phase timestamps (s_memrealtime, 100 MHz): trace[64 * wg + slot]
#define RB_TRACE(slot)                                                                  \
  do {                                                                                  \
    if (trace && l == 0) trace[64 * i + (slot)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)

// Tb, Xb: LDS, BLK doubles each -- Tb: C(i,k) fully updated (input of step k's TRSM), finally C(i,i);
// Xb: L(i,k) of the current step
template <bool LOWER>
__device__ inline void rb_tile_body(double* __restrict__ A, int n, int lda, int* __restrict__ info, int info_base,
                                    const RbWork& ws, int epoch, unsigned long long* __restrict__ trace, const int i,
                                    double* __restrict__ Tb, double* __restrict__ Xb) {
  // critical path: win the SIMD's issue arbitration against co-resident trailing-update GEMM waves
  // (priority, then age -- MI355X_MICROARCH.md "Two waves per SIMD"); a scalar, wave-uniform op
  __builtin_amdgcn_s_setprio(RB_PRIO);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int a = w >> 1, b = w & 1;                       // this wave's quadrant of off-diagonal blocks
  const int qa_d = (w == 0) ? 0 : 1, qb_d = (w == 2) ? 1 : 0;  // diagonal quadrant of waves 0..2
  const long long si = LOWER ? 1 : lda, sj = LOWER ? lda : 1;
  const int base = epoch * 64;
  auto gidx = [&](int rho, int gam) -> long long { return (long long)rho * si + (long long)gam * sj; };
  auto ldA = [&](int rho, int gam) -> double {
    return (rho < n && gam < n) ? A[gidx(rho, gam)] : (rho == gam ? 1.0 : 0.0);
  };
  const int rho_a = RB * i + 16 * a + (l & 15);  // global row of this lane in off-diagonal quadrants
  if (w == 0) RB_TRACE(0);

  // ---- initial state: diagonal quadrants in registers, C(i,0) staged for the first TRSM
  d4_t dg = {0, 0, 0, 0};
  if (w < 3) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      dg[r] = ldA(RB * i + 16 * qa_d + (l & 15), RB * i + 16 * qb_d + (l >> 4) + 4 * r);
  }
  if (i > 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) Tb[(w * 4 + r) * 64 + l] = ldA(rho_a, 16 * b + (l >> 4) + 4 * r);
  }

  for (int k = 0; k < i; ++k) {
    // ---- wait for Z_k = inv(L(k,k))
    if (tid == 0) spin_until(ws.prog + k * PSTRIDE, base + k + 1, info);
    __syncthreads();
    if (w == 0) RB_TRACE(1 + 3 * k);
    // ---- L(i,k) = C(i,k) Z_k^T,  Z_k = diag(S_k) M_k  (M lower: chunks u < 4(b+1))
    d4_t acc = {0, 0, 0, 0};
    {
      const double* Mk = ws.M + (size_t)k * BLK;
      double y[8], x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        y[u] = (u < 4 * (b + 1)) ? ld_sc1(Mk + (4 * u + (l >> 4)) * RB + 16 * b + (l & 15)) : 0.0;
        x[u] = Tb[qoff(a, u, l)];
      }
      if (b == 0) acc = mfma_chunks<4>(y, x, acc);
      else acc = mfma_chunks<8>(y, x, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] *= ld_sc1(ws.S + (size_t)k * RB + 16 * b + (l >> 4) + 4 * r);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Xb[(w * 4 + r) * 64 + l] = acc[r];
      if (rho_a < n) A[gidx(rho_a, RB * k + 16 * b + (l >> 4) + 4 * r)] = acc[r];  // final L(i,k)
    }
    __syncthreads();  // L(i,k) complete in LDS; Tb free
    if (w == 0) RB_TRACE(2 + 3 * k);
    // ---- wave 3 publishes L(i,k) for the workgroups below (write-through, drained, flagged);
    // L(i,i-1) is published later, beside the diagonal factorisation
    if (w == 3 && k + 1 < i) {
      double* dst = ws.Lp + ((size_t)i * MAXB + k) * BLK;
#pragma unroll
      for (int e = 0; e < 16; ++e) st_sc1(dst + e * 64 + l, Xb[e * 64 + l]);
      drain_stores();
      if (l == 0) st_sc1(ws.prog + i * PSTRIDE, base + k + 1);
      drain_stores();
    }
    double xm[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xm[u] = -Xb[qoff(a, u, l)];
    // ---- off-diagonal updates C(i,j) -= L(i,k) L(j,k)^T, j = k+1..i-1 (software-pipelined fetches)
    if (k + 1 < i) {
      if (l == 0)
        for (int j = k + 1; j < i; ++j) spin_until(ws.prog + j * PSTRIDE, base + k + 1, info);
      __builtin_amdgcn_wave_barrier();
      double y0[8], y1[8];
      d4_t c0, c1;
      auto fetch = [&](int jj, double* y, d4_t& c) {
        const double* Yp = ws.Lp + ((size_t)jj * MAXB + k) * BLK;
#pragma unroll
        for (int u = 0; u < 8; ++u) y[u] = ld_sc1(Yp + qoff(b, u, l));
#pragma unroll
        for (int r = 0; r < 4; ++r)
          c[r] = (rho_a < n) ? ld_sc1(A + gidx(rho_a, RB * jj + 16 * b + (l >> 4) + 4 * r)) : 0.0;
      };
      auto finish = [&](int jj, const double* y, d4_t c) {
        c = mfma_chunks<8>(y, xm, c);
        if (jj == k + 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) Tb[(w * 4 + r) * 64 + l] = c[r];
        } else if (rho_a < n) {
#pragma unroll
          for (int r = 0; r < 4; ++r) A[gidx(rho_a, RB * jj + 16 * b + (l >> 4) + 4 * r)] = c[r];
        }
      };
      int j = k + 1;
      fetch(j, y0, c0);
      while (true) {
        if (j + 1 < i) fetch(j + 1, y1, c1);
        finish(j, y0, c0);
        if (++j >= i) break;
        if (j + 1 < i) fetch(j + 1, y0, c0);
        finish(j, y1, c1);
        if (++j >= i) break;
      }
      drain_stores();  // this wave re-reads these quadrants next step
    }
    // ---- diagonal block (registers of waves 0..2): C(i,i) -= L(i,k) L(i,k)^T
    if (w < 3) {
      double xd[8], yd[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xd[u] = -Xb[qoff(qa_d, u, l)];
        yd[u] = Xb[qoff(qb_d, u, l)];
      }
      dg = mfma_chunks<8>(yd, xd, dg);
    }
    if (w == 0) RB_TRACE(3 + 3 * k);
    // the next step starts with a workgroup barrier (after its Z poll)
  }
  __syncthreads();
  if (w < 3) {
#pragma unroll
    for (int r = 0; r < 4; ++r) Tb[((qa_d * 2 + qb_d) * 4 + r) * 64 + l] = dg[r];
  }
  __syncthreads();

  if (w == 3 && i > 0) {  // publish L(i,i-1) while wave 0 factors the diagonal block
    double* dst = ws.Lp + ((size_t)i * MAXB + (i - 1)) * BLK;
#pragma unroll
    for (int e = 0; e < 16; ++e) st_sc1(dst + e * 64 + l, Xb[e * 64 + l]);
    drain_stores();
    if (l == 0) st_sc1(ws.prog + i * PSTRIDE, base + i);
    drain_stores();
  }
  // ---- step i: Cholesky + inverse of the 32x32 diagonal block on wave 0.
  // Lanes 0..31 hold the columns of the symmetric block, lanes 32..63 the columns of M (initially
  // I).  Step c: the pivot d_c and column c are broadcast from lane c (readlane); every A column
  // j > c and every M column receives  col[t] -= A(t,c) * (col[c] / d_c),  t > c  -- the same
  // instruction for both halves, so the row operations that reduce A also build M with
  // M A M^T = D; then L = M^{-1} D^{1/2} (read off the reduced columns) and inv(L) = D^{-1/2} M
  // come out of one pass with no separate substitution.  M (exact zeros above the diagonal) and
  // S = D^{-1/2} are published as they are; consumers scale their products by S.
  const int j = l & 31;
  const bool mhalf = l >= RB;
  double col[RB];
  double s = 0.0;
  if (w == 0) {
    RB_TRACE(49);
#pragma unroll
    for (int p = 0; p < RB; ++p)
      col[p] = mhalf ? ((p == j) ? 1.0 : 0.0) : ((p >= j) ? Tb[tl_index(p, j)] : Tb[tl_index(j, p)]);
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      const double d = readlane_d(col[c], c);
      double akc[RB];
#pragma unroll
      for (int p = c + 1; p < RB; ++p) akc[p] = readlane_d(col[p], c);
      const double t = col[c] * rcp_d(d);
      if (l > c) {
#pragma unroll
        for (int p = c + 1; p < RB; ++p) col[p] = fma(-akc[p], t, col[p]);
      }
    }
    // lane j < 32: pivot d_j = col[j] (frozen since step j); L(p, j) = col[p] / sqrt(d_j), p >= j
    double dj = 1.0;
#pragma unroll
    for (int p = 0; p < RB; ++p)
      if (p == j) dj = col[p];
    const bool bad = !mhalf && !(dj > 0.0);
    const unsigned long long bm = __ballot(bad ? 1 : 0);
    if (bm != 0 && l == 0 && info) {
      const int c = __ffsll((long long)bm);  // first failing column + 1
      if (RB * i + c - 1 < n) atomicCAS(info, 0, info_base + RB * i + c);
    }
    RB_TRACE(50);
    s = rsqrt_d(dj);
    if (mhalf) {
      double* Mi = ws.M + (size_t)i * BLK + j * RB;
#pragma unroll
      for (int p = 0; p < RB; p += 2) st_sc1_x2(Mi + p, col[p], col[p + 1]);
    } else {
      st_sc1(ws.S + (size_t)i * RB + j, s);
    }
    drain_stores();
  }
  __syncthreads();  // wave 0 (M, S) and wave 3 (L(i,i-1)) drained
  if (tid == 0) st_sc1(ws.prog + i * PSTRIDE, base + i + 1);
  if (w == 0) {
    RB_TRACE(51);
    if (!mhalf) {
#pragma unroll
      for (int p = 0; p < RB; ++p) {
        const int rho = RB * i + p;
        if (p >= j && rho < n) A[gidx(rho, RB * i + j)] = col[p] * s;  // final L(i,i)
      }
    }
  }
}

}  // namespace rbk
