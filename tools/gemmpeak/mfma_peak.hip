// MI355X fp64/fp32 matrix-core and vector peak microbenchmark (the tools/gemmpeak analogue:
// reference tools/gemmpeak/{cu-gemmpeak.cpp,sgemmN.cu} measures the attainable SGEMM rate of
// the card; here we measure the attainable per-instruction rates that bound our tile kernels).
//
//   mfma_peak [waves_per_simd]
//
// Each wave runs a long unrolled chain over NACC independent accumulators (no memory traffic),
// so the measured rate is the issue-limited MFMA (or VALU FMA) throughput at the clock the
// card sustains under that load.  Modes: f64 MFMA 16x16x4, f32 MFMA 16x16x4, f64 VALU FMA,
// and f64 MFMA + f64 VALU FMA in separate waves of the same CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NA = 8;

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

template <int NACC>
__global__ __launch_bounds__(512) void k_mfma_f64(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-9, b = seed - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(512) void k_mfma_f32(float* out, int iters, float seed) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = seed + threadIdx.x * 1e-6f, b = seed - threadIdx.x * 1e-6f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(512) void k_valu_f64(double* out, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = seed * i;
  const double a = 1.0000001, b = 1e-9 * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.678) out[threadIdx.x] = s;
}

template <typename F>
static double time_ms(F f) {
  hipEvent_t s, e;
  CHECK(hipEventCreate(&s));
  CHECK(hipEventCreate(&e));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(s));
  f();
  CHECK(hipEventRecord(e));
  CHECK(hipEventSynchronize(e));
  float ms;
  CHECK(hipEventElapsedTime(&ms, s, e));
  return ms;
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, dev));
  const int cus = p.multiProcessorCount;
  printf("device %s, %d CUs, clock %d MHz\n", p.gcnArchName, cus, p.clockRate / 1000);
  double* out;
  CHECK(hipMalloc(&out, 1 << 20));
  const int iters = 20000;
  for (int wps : {1, 2}) {
    const int threads = 256 * wps;  // 4 waves per SIMD-set per block -> wps waves per SIMD
    const int blocks = cus;
    double ms = time_ms([&] { hipLaunchKernelGGL((k_mfma_f64<NA>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0); });
    double flops = (double)blocks * (threads / 64) * iters * NA * (16.0 * 16 * 4 * 2);
    printf("f64 MFMA 16x16x4  waves/SIMD=%d : %8.2f TF/s\n", wps, flops / ms / 1e9);
    ms = time_ms([&] { hipLaunchKernelGGL((k_mfma_f32<NA>), dim3(blocks), dim3(threads), 0, 0, (float*)out, iters, 1.0f); });
    printf("f32 MFMA 16x16x4  waves/SIMD=%d : %8.2f TF/s\n", wps, flops / ms / 1e9);
    ms = time_ms([&] { hipLaunchKernelGGL((k_valu_f64<16>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0); });
    flops = (double)blocks * threads * iters * 16 * 2.0;
    printf("f64 VALU FMA      waves/SIMD=%d : %8.2f TF/s\n", wps, flops / ms / 1e9);
  }
  // MFMA and VALU on separate streams at once (different waves share the CUs)
  hipStream_t s1, s2;
  CHECK(hipStreamCreate(&s1));
  CHECK(hipStreamCreate(&s2));
  double ms = time_ms([&] {
    hipLaunchKernelGGL((k_mfma_f64<NA>), dim3(cus), dim3(256), 0, s1, out, iters, 1.0);
    hipLaunchKernelGGL((k_valu_f64<16>), dim3(cus), dim3(256), 0, s2, out + 4096, iters, 1.0);
    CHECK(hipStreamSynchronize(s1));
    CHECK(hipStreamSynchronize(s2));
  });
  double fl = (double)cus * 4 * iters * NA * 2048.0 + (double)cus * 256 * iters * 16 * 2.0;
  printf("f64 MFMA || VALU FMA concurrently : %8.2f TF/s combined\n", fl / ms / 1e9);
  CHECK(hipFree(out));
  return 0;
}
