// Native tile-DAG analysis for the level-synchronous executor
// (dplasma_amd/runtime/dag.py).
//
// The reference builds its task graphs with PaRSEC's PTG compiler (JDF files,
// e.g. src/zgeqrf.jdf) or the DTD insert-task interface and discovers ready
// tasks dynamically.  On MI355X a single tile task (one 256x256 tile update) is
// far too small to fill 256 CUs, so dplasma_amd executes a DAG as a sequence of
// *levels*: every task of a level is independent of the others and all tasks
// of one kind within a level become ONE batched kernel launch.  This file
// computes those levels from the program-order task list (DTD semantics:
// read-after-write, write-after-read and write-after-write hazards on tile
// keys), plus the per-level remote-tile traffic of a distributed execution.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

#include "dag_core.h"

namespace {

using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

void check_shapes(const I64& ops, const U8& modes, const char* who) {
  if (ops.ndim() != 2 || modes.ndim() != 2 || ops.shape(0) != modes.shape(0) || ops.shape(1) != modes.shape(1))
    throw std::invalid_argument(std::string(who) + ": ops and modes must be (ntasks, nroles) arrays of equal shape");
}

py::array_t<int32_t> dag_levels(I64 ops, U8 modes) {
  check_shapes(ops, modes, "dag_levels");
  const int64_t n = ops.shape(0), R = ops.shape(1);
  py::array_t<int32_t> out(n);
  const int64_t* o = ops.data();
  const uint8_t* m = modes.data();
  int32_t* lv = out.mutable_data();
  {
    py::gil_scoped_release rel;
    dpl_dag::levels(o, m, n, R, lv);
  }
  return out;
}

py::array_t<int32_t> dag_versions(I64 ops, U8 modes) {
  check_shapes(ops, modes, "dag_versions");
  const int64_t n = ops.shape(0), R = ops.shape(1);
  py::array_t<int32_t> out({n, R});
  const int64_t* o = ops.data();
  const uint8_t* m = modes.data();
  int32_t* v = out.mutable_data();
  {
    py::gil_scoped_release rel;
    dpl_dag::versions(o, m, n, R, v);
  }
  return out;
}

py::tuple dag_schedule(I64 ops, U8 modes) {
  check_shapes(ops, modes, "dag_schedule");
  const int64_t n = ops.shape(0), R = ops.shape(1);
  dpl_dag::Schedule S;
  const int64_t* o = ops.data();
  const uint8_t* m = modes.data();
  {
    py::gil_scoped_release rel;
    S = dpl_dag::schedule(o, m, n, R);
  }
  py::array_t<int32_t> lv(n), bl(n);
  py::array_t<int64_t> es(static_cast<int64_t>(S.esrc.size())), ed(static_cast<int64_t>(S.edst.size()));
  std::copy(S.level.begin(), S.level.end(), lv.mutable_data());
  std::copy(S.blevel.begin(), S.blevel.end(), bl.mutable_data());
  std::copy(S.esrc.begin(), S.esrc.end(), es.mutable_data());
  std::copy(S.edst.begin(), S.edst.end(), ed.mutable_data());
  return py::make_tuple(lv, bl, es, ed);
}

py::array_t<int64_t> dag_list_schedule(I64 pred_ptr, I64 pred_idx, py::array_t<int32_t, py::array::c_style |
                                        py::array::forcecast> prio, int policy, uint64_t seed) {
  const int64_t n = prio.shape(0);
  if (pred_ptr.ndim() != 1 || pred_ptr.shape(0) != n + 1)
    throw std::invalid_argument("dag_list_schedule: pred_ptr must have ntasks + 1 entries");
  const int64_t* pp = pred_ptr.data();
  const int64_t* pi = pred_idx.data();
  if (pp[0] != 0 || pp[n] != pred_idx.shape(0))
    throw std::invalid_argument("dag_list_schedule: pred_ptr does not describe pred_idx");
  for (int64_t e = 0; e < pred_idx.shape(0); ++e)
    if (pi[e] < 0 || pi[e] >= n) throw std::invalid_argument("dag_list_schedule: predecessor out of range");
  std::vector<int64_t> order;
  {
    py::gil_scoped_release rel;
    order = dpl_dag::list_schedule(n, pp, pi, prio.data(), policy, seed);
  }
  if (static_cast<int64_t>(order.size()) != n) throw std::invalid_argument("dag_list_schedule: the graph has a cycle");
  py::array_t<int64_t> out(n);
  std::copy(order.begin(), order.end(), out.mutable_data());
  return out;
}

// Bottom level (longest weighted path to a sink, the task's own weight included) of a DAG given by successor
// lists (CSR): Kahn's order, then one backward pass.  The device task runtime's push scheduler ranks its ready
// rings by it (models/potrf_dtr.py queue_classes).
py::array_t<double> dag_bottom_level(py::array_t<int32_t, py::array::c_style | py::array::forcecast> succ_off,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> succ,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> w) {
  const int64_t n = w.shape(0);
  if (succ_off.ndim() != 1 || succ_off.shape(0) != n + 1)
    throw std::invalid_argument("dag_bottom_level: succ_off must have n + 1 entries");
  const int32_t* so = succ_off.data();
  const int32_t* sc = succ.data();
  const double* wt = w.data();
  for (int64_t e = 0; e < so[n]; ++e)
    if (sc[e] < 0 || sc[e] >= n) throw std::invalid_argument("dag_bottom_level: successor out of range");
  py::array_t<double> out(n);
  double* bl = out.mutable_data();
  bool cyc = false;
  {
    py::gil_scoped_release rel;
    std::vector<int32_t> indeg(n, 0), order;
    order.reserve(n);
    for (int64_t e = 0; e < so[n]; ++e) ++indeg[sc[e]];
    for (int64_t t = 0; t < n; ++t)
      if (!indeg[t]) order.push_back((int32_t)t);
    for (size_t h = 0; h < order.size(); ++h)
      for (int32_t e = so[order[h]]; e < so[order[h] + 1]; ++e)
        if (--indeg[sc[e]] == 0) order.push_back(sc[e]);
    cyc = (int64_t)order.size() != n;
    if (!cyc)
      for (int64_t h = n - 1; h >= 0; --h) {
        const int32_t t = order[h];
        double m = 0;
        for (int32_t e = so[t]; e < so[t + 1]; ++e) m = std::max(m, bl[sc[e]]);
        bl[t] = wt[t] + m;
      }
  }
  if (cyc) throw std::invalid_argument("dag_bottom_level: the graph has a cycle");
  return out;
}

}  // namespace

void register_dag(py::module_& m) {
  m.def("dag_bottom_level", &dag_bottom_level, py::arg("succ_off"), py::arg("succ"), py::arg("w"),
        "Longest weighted path from each task to a sink (its own weight included)");
  m.def("dag_list_schedule", &dag_list_schedule, py::arg("pred_ptr"), py::arg("pred_idx"), py::arg("prio"),
        py::arg("policy"), py::arg("seed") = 0,
        "Issue order of a task graph under a ready-queue policy (0 program, 1 priority, 2 inverse "
        "priority, 3 FIFO, 4 LIFO, 5 random)");
  m.def("dag_schedule", &dag_schedule, py::arg("ops"), py::arg("modes"),
        "(level, bottom level, edge sources, edge destinations) of a program-order tile DAG");
  m.def("dag_levels", &dag_levels, py::arg("ops"), py::arg("modes"),
        "Level (0-based) of every task of a program-order tile DAG under RAW/WAR/WAW hazards");
  m.def("dag_versions", &dag_versions, py::arg("ops"), py::arg("modes"),
        "Version of each tile access (number of prior writes of that tile)");
}
