// Dataflow Cholesky of one diagonal tile over several workgroups (fp64, n <= 512).
//
// Reference role: the potrf_zpotrf task body (src/zpotrf_L.jdf:93-188; its GPU incarnation calls
// cusolverDnZpotrf, its CPU one CORE_zpotrf -> LAPACKE_zpotrf_work, src/cores/core_zpotrf.c:68-74)
// with the reference's info convention *INFO = k*mb + iinfo (src/zpotrf_L.jdf:180-182).
//
// Why a new kernel: the single-workgroup left-looking k_potrf_ll (potrf_trsm.hip) re-streams the
// whole left panel through ONE CU for every 16-column step (~n^3/6 doubles through one CU's L1/L2
// port) and is latency-bound at ~625 us for a 512 tile.  This kernel spreads the tile over
// ceil(n/32) workgroups, one 32-row block each, with the block row RESIDENT IN LDS for the whole
// factorisation (block 15 of a 512 tile = 16 x 8 KB), and runs a right-looking dataflow schedule:
//
//   WG i, step k < i:  wait Z_k = inv(L(k,k)) (published by WG k)
//                      L(i,k) = A(i,k) Z_k^T              (MFMA, 4 waves = 4 16x16 quadrants)
//                      publish L(i,k) (one wave, write-through stores + flag)
//                      A(i,j) -= L(i,k) L(j,k)^T, j = k+1..i  (L(j,k) from WG j's publication)
//   WG i, step i:      Cholesky + inverse of the 32x32 diagonal block on one wave, publish Z_i.
//
// Only 15 hand-offs sit on the critical path (Z_k -> WG k+1), each followed by one 32x32 TRSM,
// one SYRK and one 32x32 factorisation.  Workgroups only ever wait on workgroups with a SMALLER
// index, so the schedule cannot deadlock even if the grid is not co-resident (in-order dispatch);
// every spin is bounded anyway (info = -1000 after ~2 s).
//
// Data layout ("T-layout"): a 32x32 block is stored as 4 quadrants x 4 registers x 64 lanes;
// lane l, register r of quadrant q = (rh, ch) holds element
//     (16 rh + (l & 15), 16 ch + (l >> 4) + 4 r).
// It is simultaneously (a) the accumulator layout of v_mfma_f64_16x16x4 when the product is formed
// as D = Y X^T-transposed (A operand = Y, B operand = X), and (b) the A/B operand layout of the same
// instruction for k-chunk u = 4 ch + r.  Every LDS and workspace access is therefore one
// lane-contiguous 8-byte access (conflict-free, coalesced), and MFMA results are stored without
// any shuffle.
//
// Hand-off protocol (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility",
// first row of the sc1 table): payload stored with agent-scope relaxed atomics (sc1, write-through),
// s_waitcnt vmcnt(0) in every storing wave, one lane's sc1 flag store; consumers poll the flag with
// sc1 loads and read every handed-off byte with sc1 loads.  Flags carry a per-launch epoch, so no
// reset is needed between launches.
#include <mutex>

#include "common.h"
#include "grid_sync.h"

namespace {
constexpr int RB = 32;            // row-block height
constexpr int MAXB = 16;          // at most 16 row blocks (n <= 512)
constexpr int BLK = RB * RB;      // doubles per block
constexpr int PSTRIDE = 32;       // ints between flags (one 128-B line each)
constexpr int NSLOT = 8;          // workspaces (concurrent launches on different streams)

struct RbWork {
  double* Z;    // [MAXB][BLK]        inv(L(k,k)), T-layout
  double* Lp;   // [MAXB][MAXB][BLK]  L(i,k), T-layout
  int* prog;    // [MAXB * PSTRIDE]   epoch * 64 + number of published steps
};

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

// acc += sum_u Y(u) X(u): A operand Y, B operand X (T-layout chunks)
template <int NU>
__device__ inline d4_t mfma_chunks(const double* y, const double* x, d4_t acc) {
#pragma unroll
  for (int u = 0; u < NU; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(y[u], x[u], acc, 0, 0, 0);
  return acc;
}

// T-layout offset of (row half h, k-chunk u) for this lane
__device__ inline int qoff(int h, int u, int l) { return ((h * 2 + (u >> 2)) * 4 + (u & 3)) * 64 + l; }
// column-major 32x32 scratch with an XOR swizzle (conflict-free column writes by 32 lanes)
__device__ inline int sidx(int row, int col) { return col * RB + (row ^ col); }

template <bool LOWER>
__global__ __launch_bounds__(256) void k_potrf_rb(double* __restrict__ A, int n, int lda, int* __restrict__ info,
                                                  int info_base, RbWork ws, int epoch) {
  __shared__ double Tb[BLK];  // C(i,k) fully updated: input of step k's TRSM
  __shared__ double Xb[BLK];  // L(i,k) of the current step; later the diagonal block
  __shared__ double Sc[BLK];  // 32x32 scratch of the diagonal factorisation (sidx layout)
  const int i = blockIdx.x;
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
    // ---- L(i,k) = C(i,k) Z_k^T (Z lower: chunks u < 4(b+1))
    d4_t acc = {0, 0, 0, 0};
    {
      const double* Zk = ws.Z + (size_t)k * BLK;
      double y[8], x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        y[u] = (u < 4 * (b + 1)) ? ld_sc1(Zk + qoff(b, u, l)) : 0.0;
        x[u] = Tb[qoff(a, u, l)];
      }
      if (b == 0) acc = mfma_chunks<4>(y, x, acc);
      else acc = mfma_chunks<8>(y, x, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Xb[(w * 4 + r) * 64 + l] = acc[r];
      if (rho_a < n) A[gidx(rho_a, RB * k + 16 * b + (l >> 4) + 4 * r)] = acc[r];  // final L(i,k)
    }
    __syncthreads();  // L(i,k) complete in LDS; Tb free
    // ---- wave 3 publishes L(i,k) for the workgroups below (write-through, drained, flagged)
    if (w == 3) {
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
    // the next step starts with a workgroup barrier (after its Z poll)
  }
  __syncthreads();
  if (w < 3) {
#pragma unroll
    for (int r = 0; r < 4; ++r) Xb[((qa_d * 2 + qb_d) * 4 + r) * 64 + l] = dg[r];
  }
  __syncthreads();

  // ---- step i: Cholesky + inverse of the 32x32 diagonal block on wave 0.
  // Lanes 0..31 hold the columns of the symmetric block, lanes 32..63 the columns of M (initially
  // I).  Step c: the pivot d_c and column c are broadcast from lane c (readlane); every A column
  // j > c and every M column receives  col[t] -= A(t,c) * (col[c] / d_c),  t > c  -- the same
  // instruction for both halves, so the row operations that reduce A also build M with
  // M A M^T = D; then L = M^{-1} D^{1/2} (read off the reduced columns) and inv(L) = D^{-1/2} M
  // come out of one pass with no separate substitution.
  if (w != 0) return;
  const int j = l & 31;
  const bool mhalf = l >= RB;
  double col[RB];
#pragma unroll
  for (int p = 0; p < RB; ++p)
    col[p] = mhalf ? ((p == j) ? 1.0 : 0.0) : ((p >= j) ? Xb[tl_index(p, j)] : Xb[tl_index(j, p)]);
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
  const double s = rsqrt_d(dj);
  if (!mhalf) {
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int rho = RB * i + p;
      if (p >= j && rho < n) A[gidx(rho, RB * i + j)] = col[p] * s;  // final L(i,i)
    }
  } else {
    // inv(L)(p, j) = M(p, j) / sqrt(d_p)
#pragma unroll
    for (int p = 0; p < RB; ++p) Sc[sidx(p, j)] = (p >= j) ? col[p] * readlane_d(s, p) : 0.0;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  // publish Z_i in T-layout (write-through), drain, flag
  double* Zi = ws.Z + (size_t)i * BLK;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rho = 16 * (q >> 1) + (l & 15), gam = 16 * (q & 1) + (l >> 4) + 4 * r;
      st_sc1(Zi + (q * 4 + r) * 64 + l, Sc[sidx(rho, gam)]);
    }
  drain_stores();
  if (l == 0) st_sc1(ws.prog + i * PSTRIDE, base + i + 1);
}

std::mutex g_mu;
RbWork g_ws[64][NSLOT];
bool g_have[64] = {};
unsigned int g_launch = 0;

int get_ws(RbWork* out, int* epoch, hipStream_t st) {
  int dev = 0;
  HIP_CHECK_RET(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return -4;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_have[dev]) {
    for (int s = 0; s < NSLOT; ++s) {
      RbWork& w = g_ws[dev][s];
      HIP_CHECK_RET(hipMalloc((void**)&w.Z, sizeof(double) * MAXB * BLK));
      HIP_CHECK_RET(hipMalloc((void**)&w.Lp, sizeof(double) * MAXB * MAXB * BLK));
      HIP_CHECK_RET(hipMalloc((void**)&w.prog, sizeof(int) * MAXB * PSTRIDE));
      HIP_CHECK_RET(hipMemset(w.prog, 0, sizeof(int) * MAXB * PSTRIDE));
    }
    g_have[dev] = true;
  }
  ++g_launch;
  if ((g_launch & 0x1ffffff) == 0) {  // epoch wrap (every 2^25 launches): reset every flag
    HIP_CHECK_RET(hipDeviceSynchronize());
    for (int s = 0; s < NSLOT; ++s) HIP_CHECK_RET(hipMemset(g_ws[dev][s].prog, 0, sizeof(int) * MAXB * PSTRIDE));
    ++g_launch;
  }
  *out = g_ws[dev][g_launch % NSLOT];
  *epoch = (int)(g_launch & 0x1ffffff);
  return 0;
}
}  // namespace

// Cholesky of one n x n fp64 tile (n <= 512) in place; returns -3 when the shape is not supported.
DPL_API int dpl_potrf_tile_rb(int uplo, int n, double* A, int lda, int* info, int info_base, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > RB * MAXB) return -3;
  RbWork ws;
  int epoch = 0;
  const int rc = get_ws(&ws, &epoch, st);
  if (rc) return rc;
  const int nblk = cdiv(n, RB);
  if (uplo == DPL_LOWER)
    hipLaunchKernelGGL((k_potrf_rb<true>), dim3(nblk), dim3(256), 0, st, A, n, lda, info, info_base, ws, epoch);
  else
    hipLaunchKernelGGL((k_potrf_rb<false>), dim3(nblk), dim3(256), 0, st, A, n, lda, info, info_base, ws, epoch);
  return (int)hipGetLastError();
}
