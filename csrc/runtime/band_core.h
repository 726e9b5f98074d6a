// Native core of the band -> tridiagonal bulge chasing (no Python dependency: the pybind11
// module band.cpp and the sanitizer test driver tests/native/test_runtime_core.cpp both use it).
// Hermitian band -> real symmetric tridiagonal reduction by Householder bulge
// chasing (native host stage of the eigenvalue / singular value pipelines).
//
// Reference: src/zhbrdt.jdf + CORE_zhbtype{1,2,3}cb (PLASMA bulge-chasing
// kernels driven by PaRSEC), used by dplasma_zheev_New (src/zheev_wrapper.c:
// herbt -> diag_band_to_rect -> hbrdt -> dsterf on rank 0).
//
// After the GPU two-sided tile reduction (models/eigen.py: herbt, ge2gb) the
// band has only (nb+1) x N entries; chasing it down to tridiagonal is a
// memory-latency-bound O(N^2 nb) sweep that does not pay to run on the GPU at
// the sizes where the tile stage dominates, so it runs here, on the host.
//
// Algorithm (sweep j annihilates column j below the subdiagonal):
//   reflector H = I - tau v v^H on rows S = [st, ed] (|S| <= b) built from
//   A(S, col); A := H^H A H restricted to the band:
//     (a) columns c < st   : A(S, c)  := H^H A(S, c)
//     (b) diagonal block   : A(S, S)  := H^H A(S, S) H   (symmetric rank-2 form)
//     (c) rows r > ed      : A(r, S)  := A(r, S) H       (creates the bulge)
//   then the bulge's first column is annihilated by the next reflector
//   (col = st, S = [ed+1, ed+b]) until it falls off the matrix.  Fill stays
//   within r - c <= 2b - 1, so the working band keeps 2b+1 diagonals.
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <limits>
#include <stdexcept>
#include <thread>
#include <vector>

namespace dpl_band {


template <typename T> struct real_of { using type = T; };
template <typename R> struct real_of<std::complex<R>> { using type = R; };

template <typename T> inline T cj(T x) { return x; }
template <typename R> inline std::complex<R> cj(std::complex<R> x) { return std::conj(x); }
template <typename T> inline typename real_of<T>::type re(T x) { return x; }
template <typename R> inline R re(std::complex<R> x) { return x.real(); }
template <typename T> inline typename real_of<T>::type abs2(T x) { return x * x; }
template <typename R> inline R abs2(std::complex<R> x) { return std::norm(x); }

template <typename T> struct WorkBand {
  std::vector<T> w;
  int64_t ld, n;
  WorkBand(int64_t n_, int64_t ld_) : w(static_cast<size_t>(n_ * ld_), T(0)), ld(ld_), n(n_) {}
  // lower storage: r >= c, r - c < ld
  inline T get(int64_t r, int64_t c) const {
    if (r >= c) return (r - c < ld) ? w[(r - c) + c * ld] : T(0);
    return (c - r < ld) ? cj(w[(c - r) + r * ld]) : T(0);
  }
  inline void set_lower(int64_t r, int64_t c, T v) {
    if (r - c < ld) w[(r - c) + c * ld] = v;
  }
};

// LAPACK xLARFG convention: H^H [alpha; x] = [beta; 0], H = I - tau v v^H, v[0] = 1, beta real.
template <typename T> void larfg(int64_t len, T* x, T& tau, typename real_of<T>::type& beta) {
  using R = typename real_of<T>::type;
  R xn = 0;
  for (int64_t i = 1; i < len; ++i) xn += abs2(x[i]);
  T alpha = x[0];
  R ai = std::sqrt(std::max<R>(abs2(alpha) - re(alpha) * re(alpha), R(0)));
  if (xn == R(0) && ai == R(0)) {
    tau = T(0);
    beta = re(alpha);
    x[0] = T(1);
    return;
  }
  R nrm = std::sqrt(abs2(alpha) + xn);
  beta = (re(alpha) >= 0) ? -nrm : nrm;
  tau = (T(beta) - alpha) / T(beta);
  T scal = T(1) / (alpha - T(beta));
  for (int64_t i = 1; i < len; ++i) x[i] *= scal;
  x[0] = T(1);
}

template <typename T> struct Work {
  std::vector<T> v, p, wv, s;
  explicit Work(int64_t b) : v(b + 1), p(b + 1), wv(b + 1), s(3 * b + 2) {}
};

// One reflector step: annihilate A(st+1:ed, col) and apply H two-sided within the band.
template <typename T>
void chase_step(WorkBand<T>& A, int64_t b, int64_t col, int64_t st, int64_t ed, Work<T>& W) {
  // Column c of the lower band is contiguous: A(r, c) = P(c)[r - c] for 0 <= r - c < ld.
  const int64_t n = A.n, ld = A.ld;
  T* const w = A.w.data();
  auto P = [&](int64_t c) { return w + c * ld; };
  T *v = W.v.data(), *p = W.p.data(), *wv = W.wv.data(), *s = W.s.data();
  const int64_t len = ed - st + 1;
  T* pc = P(col) + (st - col);
  for (int64_t i = 0; i < len; ++i) v[i] = (st - col + i < ld) ? pc[i] : T(0);
  T tau;
  typename real_of<T>::type beta;
  larfg(len, v, tau, beta);
  pc[0] = T(beta);
  for (int64_t i = 1; i < len && st - col + i < ld; ++i) pc[i] = T(0);
  if (tau == T(0)) return;
  const T ctau = cj(tau);
  // (a) columns c < st (other than col): A(S, c) := H^H A(S, c)
  for (int64_t c = std::max<int64_t>(0, st - 2 * b); c < st; ++c) {
    if (c == col) continue;
    T* a = P(c) + (st - c);
    const int64_t m = std::min(len, ld - (st - c));
    if (m <= 0) continue;
    T t = 0;
    for (int64_t i = 0; i < m; ++i) t += cj(v[i]) * a[i];
    if (t == T(0)) continue;
    t *= ctau;
    for (int64_t i = 0; i < m; ++i) a[i] -= v[i] * t;
  }
  // (b) diagonal block: B := B - v w^H - w v^H, w = tau p - |tau|^2 (v^H p) / 2 v, p = B v
  for (int64_t i = 0; i < len; ++i) p[i] = T(0);
  for (int64_t k = 0; k < len; ++k) {
    const T* a = P(st + k);  // a[r - k] = B(r, k), r >= k
    T acc = a[0] * v[k];
    for (int64_t r = k + 1; r < len; ++r) {
      p[r] += a[r - k] * v[k];
      acc += cj(a[r - k]) * v[r];
    }
    p[k] += acc;
  }
  T vp = 0;
  for (int64_t i = 0; i < len; ++i) vp += cj(v[i]) * p[i];
  const T half = T(abs2(tau) * re(vp) / 2);
  for (int64_t i = 0; i < len; ++i) wv[i] = tau * p[i] - half * v[i];
  for (int64_t c = 0; c < len; ++c) {
    T* a = P(st + c);
    const T cw = cj(wv[c]), cv = cj(v[c]);
    for (int64_t r = c; r < len; ++r) a[r - c] -= v[r] * cw + wv[r] * cv;
  }
  // (c) rows r in (ed, rmax]: A(r, S) := A(r, S) H  (column-oriented: s_r = sum_k A(r, st+k) v_k)
  const int64_t r0 = ed + 1, rmax = std::min(n - 1, ed + 2 * b);
  if (r0 > rmax) return;
  const int64_t nr = rmax - r0 + 1;
  for (int64_t i = 0; i < nr; ++i) s[i] = T(0);
  for (int64_t k = 0; k < len; ++k) {
    const int64_t off = r0 - (st + k);
    const int64_t m = std::min(nr, ld - off);
    const T* a = P(st + k) + off;
    for (int64_t i = 0; i < m; ++i) s[i] += a[i] * v[k];
  }
  for (int64_t i = 0; i < nr; ++i) s[i] *= tau;
  for (int64_t k = 0; k < len; ++k) {
    const int64_t off = r0 - (st + k);
    const int64_t m = std::min(nr, ld - off);
    T* a = P(st + k) + off;
    const T cv = cj(v[k]);
    for (int64_t i = 0; i < m; ++i) a[i] -= s[i] * cv;
  }
}

// Sweeps run on a thread pool, sweep j on thread j % nthreads.  Block t of sweep j
// (st = j + 1 + t b, ed = st + b - 1) touches lower entries with rows in
// [st, ed + 2b] and columns in [st - 2b, ed]; block t' of sweep j-1 has rows >= j + t' b
// and columns >= j + (t' - 2) b, so both ranges are disjoint once t' >= t + 4 = t + LAG:
// block t may start when sweep j-1 has finished blocks 0..t+3 (or is done).  The
// result equals the sequential order bit for bit.
template <typename T>
void chase(WorkBand<T>& A, int64_t b, int nthreads) {
  const int64_t n = A.n;
  const int64_t nsw = std::max<int64_t>(n - 2, 0);
  if (nsw == 0) return;
  constexpr int64_t LAG = 4;
  constexpr int64_t DONE = std::numeric_limits<int64_t>::max();
  struct alignas(64) Counter { std::atomic<int64_t> v{0}; };
  std::vector<Counter> progv(static_cast<size_t>(nsw));
  auto prog = [&](int64_t j) -> std::atomic<int64_t>& { return progv[static_cast<size_t>(j)].v; };
  nthreads = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(nthreads, nsw)));
  auto worker = [&](int tid) {
    Work<T> W(b);
    for (int64_t j = tid; j < nsw; j += nthreads) {
      int64_t col = j, st = j + 1, ed = std::min(j + b, n - 1), t = 0;
      while (st < n && ed > st) {
        if (j > 0) {
          int spins = 0;
          while (prog(j - 1).load(std::memory_order_acquire) < t + LAG)
            if (++spins > 4096) std::this_thread::yield();
            else __builtin_ia32_pause();
        }
        chase_step(A, b, col, st, ed, W);
        prog(j).store(++t, std::memory_order_release);
        col = st;
        st = ed + 1;
        ed = std::min(ed + b, n - 1);
      }
      prog(j).store(DONE, std::memory_order_release);
    }
  };
  if (nthreads == 1) {
    worker(0);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nthreads; ++t) pool.emplace_back(worker, t);
  for (auto& th : pool) th.join();
}

// ab: LAPACK lower band storage (ldab >= b + 1, column-major, n columns); d[n], e[n-1] receive the
// diagonal and |subdiagonal| of the tridiagonal form.
template <typename T>
void hbrdt_core(const T* ab, int64_t ldab, int64_t n, int64_t b, int nthreads, typename real_of<T>::type* d,
                typename real_of<T>::type* e) {
  if (b < 0 || ldab < b + 1) throw std::invalid_argument("hbrdt: ldab must be >= b + 1");
  WorkBand<T> W(n, 2 * std::max<int64_t>(b, 1) + 1);
  for (int64_t c = 0; c < n; ++c)
    for (int64_t dd = 0; dd <= b && c + dd < n; ++dd) W.w[dd + c * W.ld] = ab[dd + c * ldab];
  if (b > 1) chase(W, b, nthreads);
  for (int64_t i = 0; i < n; ++i) d[i] = re(W.w[i * W.ld]);
  for (int64_t i = 0; i + 1 < n; ++i) e[i] = std::sqrt(abs2(W.w[1 + i * W.ld]));
}

}  // namespace dpl_band
