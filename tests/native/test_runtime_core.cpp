// Sanitizer driver of the native runtime cores (csrc/runtime/dag_core.h, band_core.h): built with
// -fsanitize=address,undefined and with -fsanitize=thread by tools/build.py --sanitize and run by
// tests/test_sanitizers.py (the reference's debug / sanitizer build modes, configure:81-90).
// Plain C++: no Python, no GPU.  Exits non-zero on a failed check; the sanitizers abort on a bug.
#include <cmath>
#include <complex>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "band_core.h"
#include "dag_core.h"

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

// program-order tile Cholesky (lower): POTRF(k), TRSM(m,k), SYRK(m,k), GEMM(m,n,k); 3 roles per task
static void chol_dag(int nt, std::vector<int64_t>& ops, std::vector<uint8_t>& modes, std::vector<int>& kind) {
  auto key = [&](int m, int n) { return (int64_t)m * 1000 + n; };
  auto add = [&](int k, int64_t a, uint8_t ma, int64_t b, uint8_t mb, int64_t c, uint8_t mc) {
    ops.insert(ops.end(), {a, b, c});
    modes.insert(modes.end(), {ma, mb, mc});
    kind.push_back(k);
  };
  for (int k = 0; k < nt; ++k) {
    add(0, key(k, k), 3, 0, 0, 0, 0);
    for (int m = k + 1; m < nt; ++m) add(1, key(m, k), 3, key(k, k), 1, 0, 0);
    for (int m = k + 1; m < nt; ++m) {
      add(2, key(m, m), 3, key(m, k), 1, 0, 0);
      for (int n = k + 1; n < m; ++n) add(3, key(m, n), 3, key(m, k), 1, key(n, k), 1);
    }
  }
}

static void test_dag() {
  const int nt = 7;
  std::vector<int64_t> ops;
  std::vector<uint8_t> modes;
  std::vector<int> kind;
  chol_dag(nt, ops, modes, kind);
  const int64_t n = (int64_t)kind.size(), R = 3;
  std::vector<int32_t> lv(n), ver(n * R);
  dpl_dag::levels(ops.data(), modes.data(), n, R, lv.data());
  dpl_dag::versions(ops.data(), modes.data(), n, R, ver.data());
  const dpl_dag::Schedule S = dpl_dag::schedule(ops.data(), modes.data(), n, R);
  // POTRF(k) sits at level 3k: potrf -> trsm -> update -> next potrf
  int k = 0;
  for (int64_t t = 0; t < n; ++t)
    if (kind[t] == 0) {
      CHECK(lv[t] == 3 * k);
      CHECK(S.level[t] == lv[t]);
      CHECK(ver[t * R] == k);  // the diagonal tile was written by k SYRKs before POTRF(k)
      ++k;
    }
  CHECK(k == nt);
  // every edge goes forward in program order and in level; levels agree with the edge relation
  for (size_t e = 0; e < S.esrc.size(); ++e) {
    CHECK(S.esrc[e] < S.edst[e]);
    CHECK(S.level[S.edst[e]] > S.level[S.esrc[e]]);
    CHECK(S.blevel[S.esrc[e]] > S.blevel[S.edst[e]]);
  }
  CHECK(S.blevel[0] == 3 * (nt - 1));  // critical path POTRF(0) ... POTRF(nt-1)
}

template <typename T> T rnd(std::mt19937_64& g);
template <> double rnd<double>(std::mt19937_64& g) { return std::uniform_real_distribution<double>(-1, 1)(g); }
template <> std::complex<double> rnd<std::complex<double>>(std::mt19937_64& g) {
  std::uniform_real_distribution<double> u(-1, 1);
  return {u(g), u(g)};
}

template <typename T> void test_band(int64_t n, int64_t b) {
  std::mt19937_64 g(1234 + n + b);
  const int64_t ldab = b + 1;
  std::vector<T> ab(ldab * n, T(0));
  double tr = 0, fro2 = 0;
  for (int64_t c = 0; c < n; ++c)
    for (int64_t d = 0; d <= b && c + d < n; ++d) {
      T v = rnd<T>(g);
      if (d == 0) v = T(std::real(v) + 4.0);
      ab[d + c * ldab] = v;
      if (d == 0) {
        tr += std::real(v);
        fro2 += std::norm(v);
      } else {
        fro2 += 2 * std::norm(v);
      }
    }
  std::vector<double> d1(n), e1(n - 1), d4(n), e4(n - 1);
  dpl_band::hbrdt_core<T>(ab.data(), ldab, n, b, 1, d1.data(), e1.data());
  dpl_band::hbrdt_core<T>(ab.data(), ldab, n, b, 4, d4.data(), e4.data());
  double s = 0, f = 0;
  for (int64_t i = 0; i < n; ++i) s += d1[i], f += d1[i] * d1[i];
  for (int64_t i = 0; i + 1 < n; ++i) f += 2 * e1[i] * e1[i];
  CHECK(std::fabs(s - tr) < 1e-9 * std::max(1.0, std::fabs(tr)));   // similarity keeps the trace
  CHECK(std::fabs(f - fro2) < 1e-9 * fro2);                          // ... and the Frobenius norm
  for (int64_t i = 0; i < n; ++i) CHECK(d1[i] == d4[i]);             // threaded chase: same bits
  for (int64_t i = 0; i + 1 < n; ++i) CHECK(e1[i] == e4[i]);
}

// list scheduler: every policy gives a topological order of the Cholesky DAG's edges
static void test_list_schedule() {
  const int nt = 6;
  std::vector<int64_t> ops;
  std::vector<uint8_t> modes;
  std::vector<int> kind;
  chol_dag(nt, ops, modes, kind);
  const int64_t n = (int64_t)kind.size(), R = 3;
  const dpl_dag::Schedule S = dpl_dag::schedule(ops.data(), modes.data(), n, R);
  std::vector<int64_t> ptr(n + 1, 0), idx(S.edst.size());
  for (int64_t d : S.edst) ++ptr[d + 1];
  for (int64_t t = 0; t < n; ++t) ptr[t + 1] += ptr[t];
  std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
  for (size_t e = 0; e < S.esrc.size(); ++e) idx[fill[S.edst[e]]++] = S.esrc[e];
  std::vector<int32_t> prio(n);
  for (int64_t t = 0; t < n; ++t) prio[t] = S.blevel[t];
  for (int pol = 0; pol < 6; ++pol) {
    const std::vector<int64_t> order = dpl_dag::list_schedule(n, ptr.data(), idx.data(), prio.data(), pol, 7);
    CHECK((int64_t)order.size() == n);
    std::vector<int64_t> pos(n, -1);
    for (int64_t i = 0; i < (int64_t)order.size(); ++i) pos[order[i]] = i;
    for (size_t e = 0; e < S.esrc.size(); ++e) CHECK(pos[S.esrc[e]] < pos[S.edst[e]]);
  }
}

int main() {
  test_dag();
  test_list_schedule();
  test_band<double>(257, 8);
  test_band<std::complex<double>>(200, 5);
  // concurrent independent reductions (thread-safety of the core under TSan)
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t) th.emplace_back([t] { test_band<double>(150 + 7 * t, 4 + t); });
  for (auto& x : th) x.join();
  std::printf("%s (%d failures)\n", g_fail ? "NATIVE FAIL" : "NATIVE OK", g_fail);
  return g_fail ? 1 : 0;
}
