// Distributed partial-pivoting panel: the process column picks every pivot on the GPUs.
//
// Reference roles: GETRF_MAX (per-process |max| of the column, src/zgetrf_ptgpanel.jdf:206),
// GETRF_RDC / GETRF_SVM (reduction of the P candidates, :379-520) and GETRF_SND (the Bruck
// exchange of the winner, :522-590) -- one round of tasks and messages per panel column.
//
// MI355X design.  Every rank of the panel's process column keeps, in one column-major buffer,
//   rows [0, tr)      T: a replica of the diagonal tile rows (every pivot destination is one of them),
//   rows [tr, m)      its own panel rows (panel-relative positions in lrel[]),
// and factors it with the persistent block kernel of lu_piv.hip (rows LDS-resident, one grid barrier
// per column), extended by ONE cross-process hand-off per column:
//   1. local grid barrier (agent scope): the local winner (|v| desc, position asc) is known to every WG;
//   2. the WG that owns it writes {|v|, position, the whole kbw-wide row} into slot [parity][me] of
//      every peer's exchange buffer (IPC-mapped device memory, system-scope stores over xGMI), then
//      a system-scope release and the slot's epoch flag;
//   3. every WG waits for the P flags of this column (system-scope polls of its own buffer), reduces
//      the P headers to the global winner and applies the interchange to FULL rows: row j := the
//      winner's row (from the slot), the displaced row j goes to the winner's position -- on every rank
//      when that position is a T row (replicated), else only on the rank that nominated it.
// Because rows move whole (every panel column at once), the recursion's laswp steps disappear and
// the displaced row never needs a second message: T is replicated, so its owner-side copy is local.
// Slots are double-buffered by column parity: a rank can only run one column ahead of a peer.
// Waits are bounded (20 s): a missing peer flags info = -1000 and the kernel drains.
#include "common.h"
#include "grid_sync.h"
#include <cstring>

#define DLR 256   // threads per workgroup, <= one row each
#define DBW 64    // block width

// slot layout (bytes): [0] int flag (epoch), [4] int position, [8] double |v|, [64..) row[kbw]
__device__ inline char* xslot(unsigned long long base, int par, int P, int q, int slot_bytes) {
  return (char*)base + ((long long)par * P + q) * slot_bytes;
}

template <typename T> __device__ inline void st_sys(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T> __device__ inline T ld_sys(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void wave_argmax_d(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
}

// (|v|, key) argmax over the 256 threads of a workgroup, returned to every thread: the four waves' winners
// meet in sv[0..3] / si[0..3] behind ONE barrier and every thread reduces them itself.  The caller must pass
// a barrier before the next call reuses the slots (every call site below is separated by one).
__device__ inline void block_argmax(double& v, int& i, double* sv, int* si) {
  const int tid = threadIdx.x;
  wave_argmax_d(v, i);
  if ((tid & 63) == 0) { sv[tid >> 6] = v; si[tid >> 6] = i; }
  __syncthreads();
  v = sv[0];
  i = si[0];
#pragma unroll
  for (int q = 1; q < DLR / 64; ++q) {
    const double v2 = sv[q];
    const int i2 = si[q];
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
}

template <typename T>
__global__ __launch_bounds__(DLR) void k_lu_block_dist(T* __restrict__ A, int ld, int m, int c0, int cend, int R,
                                                       int kbw, int tr, int diag, const int* __restrict__ lrel,
                                                       int* __restrict__ ipiv, double* __restrict__ pval, int* __restrict__ pidx,
                                                       T* __restrict__ oldrow, int* __restrict__ cnt,
                                                       const unsigned long long* __restrict__ peers, int P, int me,
                                                       int slot_bytes, int epoch0, int* __restrict__ info,
                                                       int info_base) {
  __shared__ T tile[DBW * DLR];      // column-major: tile[c * R + r]
  __shared__ T prow[DBW];
  __shared__ double sv[DLR];
  __shared__ int si[DLR];
  __shared__ int s_win[4];
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
  __builtin_amdgcn_s_setprio(3);   // critical-path panel: VALU issue priority over co-resident update waves
  const int BW = cend - c0;
  const int rbase = c0 + w * R;
  const int nr = max(0, min(R, m - rbase));
  const unsigned long long mybase = peers[me];
  for (int e = tid; e < BW * R; e += DLR) {
    const int c = e / R, r = e % R;
    if (r < nr) tile[c * R + r] = A[(rbase + r) + (long long)(c0 + c) * ld];
  }
  __syncthreads();
  const int r = tid, g = rbase + tid;
  const bool own = r < nr;
  for (int cj = 0; cj < BW; ++cj) {
    const int j = c0 + cj;
    const int epoch = epoch0 + cj;
    const int par = epoch & 1;
    // ---- 1. apply column cj-1 (its pivot row is in prow) to every row below the pivot (T replica too)
    if (cj > 0 && own && g >= j) {
      const T d = prow[cj - 1];
      T l = tile[(cj - 1) * R + r];
      if (!is_zero(d)) l = divv(l, d);
      tile[(cj - 1) * R + r] = l;
      for (int c = cj; c < BW; ++c) tile[c * R + r] = sub(tile[c * R + r], mul(l, prow[c]));
    }
    // ---- 2. local candidate: T rows only on the diagonal owner (the replicas must not nominate); the search
    //         reads only the thread's own row, and block_argmax's barrier orders the update before the row
    //         reads of the publication below
    const bool elig = own && g >= j && (g >= tr || diag);
    double cv = elig ? piv_mag((double)abs1(tile[cj * R + r])) : -1.0;
    int ci = elig ? g : 0x7fffffff;
    block_argmax(cv, ci, sv, si);
    if (tid == 0) {
      st_sc1(&pval[par * G + w], cv);
      st_sc1(&pidx[par * G + w], ci);
    }
    // the owner of row j publishes the FULL old row j (block part from LDS, the rest from memory)
    if (j >= rbase && j < rbase + nr) {
      for (int c = tid; c < kbw; c += DLR) {
        const T v = (c >= c0 && c < cend) ? tile[(c - c0) * R + (j - rbase)] : A[j + (long long)c * ld];
        st_sc1(&oldrow[(long long)par * kbw + c], v);
      }
    }
    grid_sync_counter(cnt, (cj + 1) * G, info);
    // ---- 3. local winner (same answer in every WG and every thread): local row index, key = local row
    double lval = -1.0;
    int lw = 0x7fffffff;                        // local row of the local winner (or 0x7fffffff)
    for (int b = tid; b < G; b += DLR) {
      const double v = ld_sc1(&pval[par * G + b]);
      const int i = ld_sc1(&pidx[par * G + b]);
      if (v > lval || (v == lval && i < lw)) { lval = v; lw = i; }
    }
    block_argmax(lval, lw, sv, si);
    const bool have = lw != 0x7fffffff;
    const int sender = have ? (lw - c0) / R : 0;
    // ---- 4. the sender publishes {|v|, position, row} into slot [par][me] of every rank
    if (w == sender) {
      int lpos = 0x7fffffff;
      if (have) lpos = lw < tr ? lw : lrel[lw - tr];
      for (int q = 0; q < P; ++q) {
        char* s = xslot(peers[q], par, P, me, slot_bytes);
        T* row = (T*)(s + 64);
        if (have) {
          for (int c = tid; c < kbw; c += DLR) {
            const T v = (c >= c0 && c < cend) ? tile[(c - c0) * R + (lw - rbase)] : A[lw + (long long)c * ld];
            st_sys(row + c, v);
          }
        }
        if (tid == 0) {
          st_sys((int*)(s + 4), lpos);
          st_sys((double*)(s + 8), have ? lval : -1.0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        for (int q = 0; q < P; ++q)
          __hip_atomic_store((int*)xslot(peers[q], par, P, me, slot_bytes), epoch, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // ---- 5. wait for the P candidates of this column, reduce them (|v| desc, position asc)
    if (tid == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (int q = 0; q < P; ++q) {
        const int* f = (const int*)xslot(mybase, par, P, q, slot_bytes);
        while (ld_sys(f) < epoch) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ULL) {   // 100 MHz: 20 s
            if (info) atomicExch(info, -1000);
            break;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      double best = -1.0;
      int bp = 0x7fffffff, bq = 0;
      for (int q = 0; q < P; ++q) {
        const char* s = xslot(mybase, par, P, q, slot_bytes);
        const double v = ld_sys((const double*)(s + 8));
        const int p = ld_sys((const int*)(s + 4));
        if (v > best || (v == best && p < bp)) { best = v; bp = p; bq = q; }
      }
      s_win[0] = bp;
      s_win[1] = bq;
      s_win[2] = best == 0.0;
    }
    __syncthreads();
    const int pw = s_win[0], qw = s_win[1];
    const T* wrow = (const T*)(xslot(mybase, par, P, qw, slot_bytes) + 64);
    // destination of the displaced row j: a T row (every rank holds it) or the winner's own row
    const int dest = pw < tr ? pw : (qw == me ? lw : -1);
    if (tid < BW) prow[tid] = ld_sys(wrow + c0 + tid);
    __syncthreads();
    if (dest != j) {
      if (j >= rbase && j < rbase + nr) {
        for (int c = tid; c < kbw; c += DLR) {
          if (c >= c0 && c < cend) tile[(c - c0) * R + (j - rbase)] = prow[c - c0];
          else A[j + (long long)c * ld] = ld_sys(wrow + c);
        }
      }
      if (dest >= 0 && dest >= rbase && dest < rbase + nr) {
        for (int c = tid; c < kbw; c += DLR) {
          const T v = ld_sc1(&oldrow[(long long)par * kbw + c]);
          if (c >= c0 && c < cend) tile[(c - c0) * R + (dest - rbase)] = v;
          else A[dest + (long long)c * ld] = v;
        }
      }
    }
    if (w == 0 && tid == 0) {
      ipiv[j] = pw;
      if (s_win[2] && info) atomicCAS(info, 0, info_base + j + 1);
    }
    __syncthreads();
  }
  // ---- last column: scale below the diagonal
  if (own && g >= cend) {
    const T d = prow[BW - 1];
    T l = tile[(BW - 1) * R + r];
    if (!is_zero(d)) l = divv(l, d);
    tile[(BW - 1) * R + r] = l;
  }
  __syncthreads();
  for (int e = tid; e < BW * R; e += DLR) {
    const int c = e / R, rr = e % R;
    if (rr < nr) A[(rbase + rr) + (long long)(c0 + c) * ld] = tile[c * R + rr];
  }
}

static int g_cus = 0;
static int g_maxwg = 0;   // > 0: at most this many workgroups per launch (a rank confined to a CU-masked stream)

// Cap the persistent panel's grid (0: one workgroup per CU of the device).  A launch on a CU-masked stream must not
// exceed the CUs of its mask: its grid barrier needs every workgroup co-resident (tools/gpu/lu_xlat_probe.py runs two
// emulated ranks on the two halves of one GPU).
DPL_API int dpl_lu_dist_set_maxwg(int n) {
  g_maxwg = n > 0 ? n : 0;
  return 0;
}

DPL_API int dpl_lu_dist_ws_bytes(int kbw) {
  // pval [2 x 256] doubles, pidx [2 x 256] ints, old row j [2 x kbw] (<= 16 B elements)
  return 16 * 2 * 256 + 64 + 2 * kbw * 16 + 64;
}

DPL_API int dpl_lu_dist_slot_bytes(int prec, int kbw) {
  const int es = (prec == DPL_S) ? 4 : 8;
  return ((64 + kbw * es) + 63) / 64 * 64;
}

// Factor block columns [c0, cend) (<= 64) of the local panel (m rows, ld) in one launch; rows above c0
// are final.  epoch0 = the exchange epoch of column c0 (the caller advances it by cend - c0).
DPL_API int dpl_lu_block_dist(int prec, void* A, int ld, int m, int c0, int cend, int kbw, int tr, int diag,
                              const int* lrel, int* ipiv, void* ws, int* cnt, const unsigned long long* peers, int P,
                              int me, int slot_bytes, int epoch0, int* info, int info_base, hipStream_t st) {
  if (cend - c0 > DBW || c0 >= cend || m <= c0 || cend > tr || cend > kbw) return -3;
  if (prec != DPL_D && prec != DPL_S) return -2;
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 1;
  }
  const int rows = m - c0;
  int gmax = g_cus < 256 ? g_cus : 256;
  if (g_maxwg > 0 && g_maxwg < gmax) gmax = g_maxwg;
  int G = (rows + DLR - 1) / DLR;
  if (G > gmax) G = gmax;
  if (G < 1) G = 1;
  const int R = (rows + G - 1) / G;
  if (R > DLR) return -4;   // more local rows than one per thread on every CU
  char* b = (char*)ws;
  double* pval = (double*)b;
  int* pidx = (int*)(b + 8LL * 2 * 256);
  char* old = b + 16LL * 2 * 256 + 64;
  (void)hipMemsetAsync(cnt, 0, sizeof(int), st);
  if (prec == DPL_D)
    hipLaunchKernelGGL((k_lu_block_dist<double>), dim3(G), dim3(DLR), 0, st, (double*)A, ld, m, c0, cend, R, kbw, tr,
                       diag, lrel, ipiv, pval, pidx, (double*)old, cnt, peers, P, me, slot_bytes,
                       epoch0, info, info_base);
  else
    hipLaunchKernelGGL((k_lu_block_dist<float>), dim3(G), dim3(DLR), 0, st, (float*)A, ld, m, c0, cend, R, kbw, tr,
                       diag, lrel, ipiv, pval, pidx, (float*)old, cnt, peers, P, me, slot_bytes,
                       epoch0, info, info_base);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- exchange buffers (IPC)
// Uncached device memory (every access goes to HBM: a peer's xGMI stores are never hidden behind a
// stale L2 line of the owner), zero-filled, exported as a 64-byte IPC handle.
DPL_API int dpl_xchg_alloc(long long bytes, void** ptr, void* handle) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipMalloc(&p, (size_t)bytes);
    if (e != hipSuccess) return (int)e;
  }
  e = dpl_zero_sync(p, (size_t)bytes);  // landed before any peer or stream reads it
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  std::memcpy(handle, &h, sizeof(h));
  *ptr = p;
  return 0;
}

// Zero-filled device memory exported as an IPC handle: cached (hipMalloc: data a peer stores into with
// system-scope stores and this process reads with plain loads after a system acquire -- the distributed
// DTR's receive buffers and W) or uncached (flags and counters polled across processes).
DPL_API int dpl_ipc_alloc(long long bytes, int cached, void** ptr, void* handle) {
  if (!cached) return dpl_xchg_alloc(bytes, ptr, handle);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = dpl_zero_sync(p, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  std::memcpy(handle, &h, sizeof(h));
  *ptr = p;
  return 0;
}

// clear device memory and return once the zeros have landed (value: the byte)
// device-to-device copy, completed on return (used on IPC-mapped buffers before a cross-process barrier)
DPL_API int dpl_memcpy_sync(void* dst, const void* src, long long bytes) {
  if (bytes <= 0) return 0;
  if (hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice) != hipSuccess) return -1;
  return (int)hipDeviceSynchronize();
}

// (value: any byte -- 0xFF fills doubles with NaN: the poisoned receive slots of bench.py's engine race)
DPL_API int dpl_memset_sync(void* ptr, int value, long long bytes) {
  if (value < 0 || value > 255) return -2;
  if (bytes <= 0) return 0;
  return (int)dpl_fill_sync(ptr, value, (size_t)bytes);
}

DPL_API int dpl_xchg_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

DPL_API int dpl_xchg_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

DPL_API int dpl_xchg_free(void* ptr) { return (int)hipFree(ptr); }

DPL_API int dpl_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }
