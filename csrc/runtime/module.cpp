// pybind11 entry point of the native runtime module ``dplasma_amd.lib._dplasma_rt``.
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_dag(py::module_& m);
void register_band(py::module_& m);
void register_perm(py::module_& m);

PYBIND11_MODULE(_dplasma_rt, m) {
  m.doc() = "dplasma_amd native runtime: tile-DAG analysis, band reductions, pivot compositions";
  register_dag(m);
  register_band(m);
  register_perm(m);
}
