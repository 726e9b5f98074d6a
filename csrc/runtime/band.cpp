// Hermitian band -> real symmetric tridiagonal reduction: pybind11 binding of band_core.h
// (native host stage of the eigenvalue / singular value pipelines; reference src/zhbrdt.jdf).
#include <pybind11/complex.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "band_core.h"

namespace py = pybind11;

namespace {
using dpl_band::real_of;

template <typename T>
py::tuple hbrdt_impl(py::array ab_in, int64_t b, int nthreads) {
  using R = typename real_of<T>::type;
  auto ab = py::array_t<T, py::array::f_style>::ensure(ab_in);
  if (!ab || ab.ndim() != 2) throw std::invalid_argument("hbrdt: band must be a 2-D (ldab x n) array");
  const int64_t ldab = ab.shape(0), n = ab.shape(1);
  py::array_t<R> d(n), e(std::max<int64_t>(n - 1, 0));
  const T* src = ab.data();
  R* dp = d.mutable_data();
  R* ep = e.mutable_data();
  {
    py::gil_scoped_release nogil;
    dpl_band::hbrdt_core<T>(src, ldab, n, b, nthreads, dp, ep);
  }
  return py::make_tuple(d, e);
}

py::tuple hbrdt(py::array ab, int64_t b, int nthreads) {
  if (nthreads <= 0) {
    const char* e = std::getenv("OMP_NUM_THREADS");
    nthreads = e ? std::atoi(e) : static_cast<int>(std::thread::hardware_concurrency());
    nthreads = std::max(1, std::min(nthreads, 16));
  }
  auto dt = ab.dtype();
  if (dt.is(py::dtype::of<double>())) return hbrdt_impl<double>(ab, b, nthreads);
  if (dt.is(py::dtype::of<float>())) return hbrdt_impl<float>(ab, b, nthreads);
  if (dt.is(py::dtype::of<std::complex<double>>())) return hbrdt_impl<std::complex<double>>(ab, b, nthreads);
  if (dt.is(py::dtype::of<std::complex<float>>())) return hbrdt_impl<std::complex<float>>(ab, b, nthreads);
  throw std::invalid_argument("hbrdt: unsupported dtype");
}

}  // namespace

void register_band(py::module_& m) {
  m.def("hbrdt", &hbrdt, py::arg("ab"), py::arg("b"), py::arg("nthreads") = 0,
        "Reduce a Hermitian band matrix (LAPACK lower band storage, ldab >= b+1) to real symmetric tridiagonal "
        "form by Householder bulge chasing; returns (d, e) with e = |subdiagonal|.");
}
