// Shared device-side helpers for the dplasma_amd CDNA4 (gfx950) kernel library.
//
// Every kernel in this library works on *tile items*: small POD records that
// carry element offsets into a base allocation (the local tile storage of a
// block-cyclic descriptor, or a contiguous panel buffer) plus the tile's
// effective extent.  The host (Python side, dplasma_amd/ops/gpu.py) builds
// item lists once per taskpool ("ENQ" phase, excluded from timing as in the
// reference's tests/common.h:252-277) so that a whole step of the algorithm is
// ONE launch instead of one launch per tile (SURVEY.md §7.1 "batching is
// mandatory").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_complex.h>
#include <stdint.h>

#define DPL_API extern "C" __attribute__((visibility("default")))

// precision codes (match dplasma constants.h: RealFloat=2 .. ComplexDouble=5)
enum { DPL_S = 2, DPL_D = 3, DPL_C = 4, DPL_Z = 5 };
// BLAS enums (same numeric values as dplasma constants.h)
enum { DPL_NOTRANS = 111, DPL_TRANS = 112, DPL_CONJTRANS = 113,
       DPL_UPPER = 121, DPL_LOWER = 122, DPL_UPPERLOWER = 123,
       DPL_NONUNIT = 131, DPL_UNIT = 132, DPL_LEFT = 141, DPL_RIGHT = 142 };

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- scalar traits
template <typename T> struct ST;
template <> struct ST<float> {
  typedef float real;
  static __device__ __host__ inline float zero() { return 0.f; }
  static __device__ __host__ inline float one() { return 1.f; }
};
template <> struct ST<double> {
  typedef double real;
  static __device__ __host__ inline double zero() { return 0.; }
  static __device__ __host__ inline double one() { return 1.; }
};
template <> struct ST<hipFloatComplex> {
  typedef float real;
  static __device__ __host__ inline hipFloatComplex zero() { return make_hipFloatComplex(0.f, 0.f); }
  static __device__ __host__ inline hipFloatComplex one() { return make_hipFloatComplex(1.f, 0.f); }
};
template <> struct ST<hipDoubleComplex> {
  typedef double real;
  static __device__ __host__ inline hipDoubleComplex zero() { return make_hipDoubleComplex(0., 0.); }
  static __device__ __host__ inline hipDoubleComplex one() { return make_hipDoubleComplex(1., 0.); }
};

// uniform arithmetic helpers so templates read like the math
__device__ __host__ inline float mul(float a, float b) { return a * b; }
__device__ __host__ inline double mul(double a, double b) { return a * b; }
__device__ __host__ inline hipFloatComplex mul(hipFloatComplex a, hipFloatComplex b) { return hipCmulf(a, b); }
__device__ __host__ inline hipDoubleComplex mul(hipDoubleComplex a, hipDoubleComplex b) { return hipCmul(a, b); }
__device__ __host__ inline float add(float a, float b) { return a + b; }
__device__ __host__ inline double add(double a, double b) { return a + b; }
__device__ __host__ inline hipFloatComplex add(hipFloatComplex a, hipFloatComplex b) { return hipCaddf(a, b); }
__device__ __host__ inline hipDoubleComplex add(hipDoubleComplex a, hipDoubleComplex b) { return hipCadd(a, b); }
__device__ __host__ inline float sub(float a, float b) { return a - b; }
__device__ __host__ inline double sub(double a, double b) { return a - b; }
__device__ __host__ inline hipFloatComplex sub(hipFloatComplex a, hipFloatComplex b) { return hipCsubf(a, b); }
__device__ __host__ inline hipDoubleComplex sub(hipDoubleComplex a, hipDoubleComplex b) { return hipCsub(a, b); }
// fused a + b*c
__device__ inline float fma_(float b, float c, float a) { return fmaf(b, c, a); }
__device__ inline double fma_(double b, double c, double a) { return fma(b, c, a); }
__device__ inline hipFloatComplex fma_(hipFloatComplex b, hipFloatComplex c, hipFloatComplex a) {
  return make_hipFloatComplex(fmaf(-b.y, c.y, fmaf(b.x, c.x, a.x)), fmaf(b.y, c.x, fmaf(b.x, c.y, a.y)));
}
__device__ inline hipDoubleComplex fma_(hipDoubleComplex b, hipDoubleComplex c, hipDoubleComplex a) {
  return make_hipDoubleComplex(fma(-b.y, c.y, fma(b.x, c.x, a.x)), fma(b.y, c.x, fma(b.x, c.y, a.y)));
}
__device__ __host__ inline float conj_(float a) { return a; }
__device__ __host__ inline double conj_(double a) { return a; }
__device__ __host__ inline hipFloatComplex conj_(hipFloatComplex a) { return hipConjf(a); }
__device__ __host__ inline hipDoubleComplex conj_(hipDoubleComplex a) { return hipConj(a); }
__device__ inline float absv(float a) { return fabsf(a); }
__device__ inline double absv(double a) { return fabs(a); }
__device__ inline float absv(hipFloatComplex a) { return hypotf(a.x, a.y); }
__device__ inline double absv(hipDoubleComplex a) { return hypot(a.x, a.y); }
// LAPACK i?amax magnitude: |re| + |im| for complex (cabs1)
__device__ inline float abs1(float a) { return fabsf(a); }
__device__ inline double abs1(double a) { return fabs(a); }
__device__ inline float abs1(hipFloatComplex a) { return fabsf(a.x) + fabsf(a.y); }
__device__ inline double abs1(hipDoubleComplex a) { return fabs(a.x) + fabs(a.y); }
__device__ inline float realv(float a) { return a; }
__device__ inline double realv(double a) { return a; }
__device__ inline float realv(hipFloatComplex a) { return a.x; }
__device__ inline double realv(hipDoubleComplex a) { return a.x; }
__device__ inline float imagv(float) { return 0.f; }
__device__ inline double imagv(double) { return 0.; }
__device__ inline float imagv(hipFloatComplex a) { return a.y; }
__device__ inline double imagv(hipDoubleComplex a) { return a.y; }
template <typename T> __device__ inline T from_real(typename ST<T>::real r);
template <> __device__ inline float from_real<float>(float r) { return r; }
template <> __device__ inline double from_real<double>(double r) { return r; }
template <> __device__ inline hipFloatComplex from_real<hipFloatComplex>(float r) { return make_hipFloatComplex(r, 0.f); }
template <> __device__ inline hipDoubleComplex from_real<hipDoubleComplex>(double r) { return make_hipDoubleComplex(r, 0.); }
// scalar from (re, im); the imaginary part is dropped for real types
template <typename T> __device__ inline T make_sc(typename ST<T>::real re, typename ST<T>::real im);
template <> __device__ inline float make_sc<float>(float re, float) { return re; }
template <> __device__ inline double make_sc<double>(double re, double) { return re; }
template <> __device__ inline hipFloatComplex make_sc<hipFloatComplex>(float re, float im) { return make_hipFloatComplex(re, im); }
template <> __device__ inline hipDoubleComplex make_sc<hipDoubleComplex>(double re, double im) { return make_hipDoubleComplex(re, im); }
__device__ inline float divv(float a, float b) { return a / b; }
__device__ inline double divv(double a, double b) { return a / b; }
__device__ inline hipFloatComplex divv(hipFloatComplex a, hipFloatComplex b) { return hipCdivf(a, b); }
__device__ inline hipDoubleComplex divv(hipDoubleComplex a, hipDoubleComplex b) { return hipCdiv(a, b); }
__device__ inline bool is_zero(float a) { return a == 0.f; }
__device__ inline bool is_zero(double a) { return a == 0.; }
__device__ inline bool is_zero(hipFloatComplex a) { return a.x == 0.f && a.y == 0.f; }
__device__ inline bool is_zero(hipDoubleComplex a) { return a.x == 0. && a.y == 0.; }

// ---------------------------------------------------------------- XCD mapping
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md §Workgroup
// dispatch).  Remap so that consecutive *logical* block ids share an XCD (and
// therefore its 4 MiB L2): the sub-tiles of one output tile, and neighbouring
// tiles of one tile-row, then re-use the same A/B panel strips from L2.
// Bijective for any nwg (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ inline int xcd_remap(int bid, int nwg) {
  const int NX = 8;
  int q = nwg / NX, r = nwg % NX;
  int xcd = bid % NX, loc = bid / NX;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

// ---------------------------------------------------------------- item records
// One output tile of a batched GEMM-like launch.
struct GemmItem {
  long long c_off, a_off, b_off;  // element offsets from the launch's C/A/B base pointers
  int m, n, k;                    // effective op(A) m×k, op(B) k×n, C m×n
  int flags;                      // bits 0-1: C write mask 0=full 1=lower(r>=c) 2=upper(r<=c)
};
// One tile of a unary / binary map launch (laset, lacpy, geadd, generators, norms).
struct TileItem {
  long long a_off, b_off;  // element offsets (b_off unused by unary ops)
  int m, n;                // tile extent
  int gi, gj;              // global element coordinates of the tile's (0,0)
};

// ---------------------------------------------------------------- misc
__device__ inline int lane_id() { return threadIdx.x & 63; }
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

#define HIP_CHECK_RET(x)                              \
  do {                                                \
    hipError_t e__ = (x);                             \
    if (e__ != hipSuccess) return (int)e__;           \
  } while (0)

// Zero device memory and return only once the zeros have landed, through a private non-blocking
// stream and hipStreamSynchronize -- not hipMemset on the null stream + hipDeviceSynchronize, which
// a rocprofv3 trace showed completing after a later kernel on a non-blocking stream had started
// (profiles/r4_potrf_rb_race.txt).
static inline hipError_t dpl_fill_sync(void* p, int byte, size_t bytes) {
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(p, byte & 255, bytes, s);
  const hipError_t e2 = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  return e != hipSuccess ? e : e2;
}
static inline hipError_t dpl_zero_sync(void* p, size_t bytes) { return dpl_fill_sync(p, 0, bytes); }

// Pivot-search magnitude: |x| with NaN mapped to 0, so an eligible row always beats the "no candidate" marker
// (-1) and a NaN column still yields an in-range pivot (the row j itself) instead of the sentinel index.
template <typename R> __device__ inline R piv_mag(R v) { return v >= R(0) ? v : R(0); }
