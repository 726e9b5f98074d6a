// Grid-wide hand-off helpers shared by the persistent (one workgroup per CU) kernels:
// lu_piv.hip (pivoting LU panel) and qr_panel.hip (Householder QR panel).
#pragma once
#include <hip/hip_runtime.h>

// Bounded spin: if the grid is not co-resident (e.g. several processes share the device) the
// barrier gives up after ~2 s, flags info = -1000 and lets the kernel drain instead of hanging.
// Every byte handed across the barrier is written and read with agent-scope relaxed atomics
// (sc1: coherent past the per-XCD L2s) and drained (vmcnt(0)) before the arrival, so the
// barrier itself needs no cache-maintenance fences (MI355X_MICROARCH.md handoff rows).
__device__ inline void grid_sync_counter(int* cnt, int target, int* info) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ULL) {  // 100 MHz clock: 2 s
        if (info) atomicExch(info, -1000);
        break;
      }
    }
  }
  __syncthreads();
}

template <typename T> __device__ inline void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T> __device__ inline T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- tagged granules: one 8-byte {32-bit payload (high half), 32-bit tag} word per sc1 store; a reader polls the
// word itself until the tag matches (no drain, flag or counter; lu_piv.hip k_lu_block_tag, lu_dist.hip)
__device__ inline bool tag_poll(const unsigned long long* p, unsigned tag, unsigned long long& x, int* info) {
  x = ld_sc1(p);
  if ((unsigned)x == tag) return true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  do {
    __builtin_amdgcn_s_sleep(1);
    x = ld_sc1(p);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ULL) {  // 100 MHz clock: 2 s (grid not co-resident)
      if (info) atomicExch(info, -1000);
      return false;
    }
  } while ((unsigned)x != tag);
  return true;
}

// one element as NW tagged words (payload in the high half) / back, polling stale words
template <typename T> __device__ inline void tag_put(unsigned long long* p, T x, unsigned tag) {
  constexpr int NW = sizeof(T) / 4;
  unsigned u[NW];
  __builtin_memcpy(u, &x, sizeof(T));
#pragma unroll
  for (int q = 0; q < NW; ++q) st_sc1(&p[q], ((unsigned long long)u[q] << 32) | tag);
}
template <typename T> __device__ inline T tag_get(const unsigned long long* p, unsigned tag, int* info) {
  constexpr int NW = sizeof(T) / 4;
  unsigned long long x[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) x[q] = ld_sc1(&p[q]);
  unsigned u[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    if ((unsigned)x[q] != tag) tag_poll(&p[q], tag, x[q], info);
    u[q] = (unsigned)(x[q] >> 32);
  }
  T v;
  __builtin_memcpy(&v, u, sizeof(T));
  return v;
}
