// Composition of LU row interchanges for the deferred left-column pass of getrf_1d (DPLASMA_LU_DEFER_LEFT): for
// every factored tile column n, the permutation that all later steps' interchanges apply to its rows [(n+1) nb, m).
// Backward over the LAPACK pivot sequence with the map and its inverse, one O(1) update per swap -- O(K + m kt) in
// total, where applying the swaps per column would be O(K kt).  Reference role: the swpback(k, n) tasks of
// src/zgetrf_1d.jdf:360-409 (step k's interchanges applied to left column n, off the critical path).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

// ipiv: K 1-based pivots (row i swapped with ipiv[i] - 1, ipiv[i] - 1 >= i), m rows, nb tile rows, kt panels.
// Returns (src, off): for column n < kt - 1, src[off[n] : off[n] + m - (n+1) nb] are the source rows of rows
// (n+1) nb .. m-1 (row r takes former row src[...]); off has kt entries (off[kt-1] = len(src)).
py::tuple piv_compose_left(py::array_t<int32_t, py::array::c_style | py::array::forcecast> ipiv, int64_t m,
                           int64_t nb, int64_t kt) {
  const int64_t K = ipiv.size();
  if (m <= 0 || nb <= 0 || kt <= 0 || K > m) throw std::invalid_argument("piv_compose_left: bad sizes");
  const int32_t* p = ipiv.data();
  std::vector<int64_t> off(kt, 0);
  int64_t tot = 0;
  for (int64_t n = 0; n < kt; ++n) {
    off[n] = tot;
    if (n + 1 < kt) tot += std::max<int64_t>(0, m - (n + 1) * nb);
  }
  py::array_t<int32_t> src_out(tot);
  py::array_t<int64_t> off_out(kt);
  int32_t* so = src_out.mutable_data();
  std::copy(off.begin(), off.end(), off_out.mutable_data());
  {
    py::gil_scoped_release nogil;
    std::vector<int32_t> src(m), inv(m);
    for (int64_t r = 0; r < m; ++r) src[r] = inv[r] = (int32_t)r;
    // snapshot for column n is taken right after applying swap s_n = (n+1) nb (swaps s_n .. K-1 composed)
    int64_t n = kt - 2;
    for (int64_t i = K - 1; i >= 0 && n >= 0; --i) {
      const int32_t q = p[i] - 1;
      if (q < i || q >= m) throw std::invalid_argument("piv_compose_left: pivot out of range");
      if (q != i) {   // src := tau_i o src: the values i and q trade places
        const int32_t a = inv[i], b = inv[q];
        src[a] = q;
        src[b] = (int32_t)i;
        inv[q] = a;
        inv[i] = b;
      }
      while (n >= 0 && i == (n + 1) * nb) {
        std::copy(src.begin() + (n + 1) * nb, src.end(), so + off[n]);
        --n;
      }
    }
    for (; n >= 0; --n) {   // columns whose row range starts past the last pivot: identity
      const int64_t s = (n + 1) * nb;
      for (int64_t r = s; r < m; ++r) so[off[n] + (r - s)] = (int32_t)r;
    }
  }
  return py::make_tuple(src_out, off_out);
}

}  // namespace

void register_perm(py::module_& m) {
  m.def("piv_compose_left", &piv_compose_left, py::arg("ipiv"), py::arg("m"), py::arg("nb"), py::arg("kt"),
        "Per factored tile column n < kt - 1: the source rows of rows (n+1) nb .. m-1 under all later LU "
        "interchanges (1-based LAPACK pivots); returns (src int32, off int64[kt]).");
}
