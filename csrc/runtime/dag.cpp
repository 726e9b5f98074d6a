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
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

struct TileState {
  int32_t last_write = -1;  // level of the last writer
  int32_t max_read = -1;    // max level of readers since that write
};

// modes: 0 = unused slot, 1 = read, 2 = write, 3 = read+write
py::array_t<int32_t> dag_levels(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ops,
                                py::array_t<uint8_t, py::array::c_style | py::array::forcecast> modes) {
  if (ops.ndim() != 2 || modes.ndim() != 2 || ops.shape(0) != modes.shape(0) || ops.shape(1) != modes.shape(1))
    throw std::invalid_argument("dag_levels: ops and modes must be (ntasks, nroles) arrays of equal shape");
  const int64_t n = ops.shape(0), R = ops.shape(1);
  auto o = ops.unchecked<2>();
  auto md = modes.unchecked<2>();
  py::array_t<int32_t> out(n);
  auto lv = out.mutable_unchecked<1>();
  std::unordered_map<int64_t, TileState> st;
  st.reserve(static_cast<size_t>(std::min<int64_t>(n * 2 + 16, 1 << 24)));
  {
    py::gil_scoped_release rel;
    for (int64_t t = 0; t < n; ++t) {
      int32_t L = 0;
      for (int64_t r = 0; r < R; ++r) {
        const uint8_t m = md(t, r);
        if (!m) continue;
        auto it = st.find(o(t, r));
        if (it == st.end()) continue;
        const TileState& s = it->second;
        if (s.last_write >= L) L = s.last_write + 1;        // RAW / WAW
        if ((m & 2) && s.max_read >= L) L = s.max_read + 1;  // WAR
      }
      lv(t) = L;
      for (int64_t r = 0; r < R; ++r) {
        const uint8_t m = md(t, r);
        if (!m) continue;
        TileState& s = st[o(t, r)];
        if (m & 2) {
          s.last_write = L;
          s.max_read = -1;
        } else if (L > s.max_read) {
          s.max_read = L;
        }
      }
    }
  }
  return out;
}

// Versioned tile accesses for the distributed plan.  For every (task, role)
// access returns the version of the tile it touches (0 = initial data, v = the
// state after the v-th writing task).  Readers see the current version; a
// writing access also reports the version it reads (it produces version+1).
py::array_t<int32_t> dag_versions(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ops,
                                  py::array_t<uint8_t, py::array::c_style | py::array::forcecast> modes) {
  const int64_t n = ops.shape(0), R = ops.shape(1);
  auto o = ops.unchecked<2>();
  auto md = modes.unchecked<2>();
  py::array_t<int32_t> out({n, R});
  auto v = out.mutable_unchecked<2>();
  std::unordered_map<int64_t, int32_t> ver;
  {
    py::gil_scoped_release rel;
    for (int64_t t = 0; t < n; ++t) {
      for (int64_t r = 0; r < R; ++r) {
        v(t, r) = -1;
        if (!md(t, r)) continue;
        auto it = ver.find(o(t, r));
        v(t, r) = it == ver.end() ? 0 : it->second;
      }
      for (int64_t r = 0; r < R; ++r)
        if (md(t, r) & 2) ver[o(t, r)] += 1;
    }
  }
  return out;
}

// Full schedule analysis: levels, bottom levels (longest path to a sink) and
// the deduplicated dependency edges.  Edges always point from an earlier to a
// later task in program order, so the reverse program order is a reverse
// topological order for the bottom-level pass.
py::tuple dag_schedule(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ops,
                       py::array_t<uint8_t, py::array::c_style | py::array::forcecast> modes) {
  if (ops.ndim() != 2 || modes.ndim() != 2 || ops.shape(0) != modes.shape(0) || ops.shape(1) != modes.shape(1))
    throw std::invalid_argument("dag_schedule: ops and modes must be (ntasks, nroles) arrays of equal shape");
  const int64_t n = ops.shape(0), R = ops.shape(1);
  auto o = ops.unchecked<2>();
  auto md = modes.unchecked<2>();
  struct St {
    int64_t writer = -1;           // last writing task
    std::vector<int64_t> readers;  // readers since that write
  };
  std::vector<int32_t> level(n, 0), blevel(n, 0);
  std::vector<int64_t> esrc, edst;
  {
    py::gil_scoped_release rel;
    std::unordered_map<int64_t, St> st;
    st.reserve(static_cast<size_t>(std::min<int64_t>(n * 2 + 16, 1 << 24)));
    std::vector<int64_t> preds;
    esrc.reserve(n * 3);
    edst.reserve(n * 3);
    for (int64_t t = 0; t < n; ++t) {
      preds.clear();
      for (int64_t r = 0; r < R; ++r) {
        const uint8_t m = md(t, r);
        if (!m) continue;
        auto it = st.find(o(t, r));
        if (it == st.end()) continue;
        if (it->second.writer >= 0) preds.push_back(it->second.writer);
        if (m & 2)
          for (int64_t q : it->second.readers) preds.push_back(q);
      }
      std::sort(preds.begin(), preds.end());
      preds.erase(std::unique(preds.begin(), preds.end()), preds.end());
      int32_t L = 0;
      for (int64_t p : preds) {
        if (p == t) continue;
        L = std::max(L, level[p] + 1);
        esrc.push_back(p);
        edst.push_back(t);
      }
      level[t] = L;
      for (int64_t r = 0; r < R; ++r) {
        const uint8_t m = md(t, r);
        if (!m) continue;
        St& s = st[o(t, r)];
        if (m & 2) {
          s.writer = t;
          s.readers.clear();
        } else {
          s.readers.push_back(t);
        }
      }
    }
    // bottom levels: iterate edges in reverse destination order
    std::vector<int64_t> order(esrc.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<int64_t>(i);
    // edges were appended grouped by increasing destination: walking them backwards is reverse-topological
    for (int64_t i = static_cast<int64_t>(esrc.size()) - 1; i >= 0; --i) {
      const int64_t s = esrc[i], d = edst[i];
      blevel[s] = std::max(blevel[s], blevel[d] + 1);
    }
  }
  py::array_t<int32_t> lv(n), bl(n);
  py::array_t<int64_t> es(static_cast<int64_t>(esrc.size())), ed(static_cast<int64_t>(edst.size()));
  std::copy(level.begin(), level.end(), lv.mutable_data());
  std::copy(blevel.begin(), blevel.end(), bl.mutable_data());
  std::copy(esrc.begin(), esrc.end(), es.mutable_data());
  std::copy(edst.begin(), edst.end(), ed.mutable_data());
  return py::make_tuple(lv, bl, es, ed);
}

}  // namespace

void register_dag(py::module_& m) {
  m.def("dag_schedule", &dag_schedule, py::arg("ops"), py::arg("modes"),
        "(level, bottom level, edge sources, edge destinations) of a program-order tile DAG");
  m.def("dag_levels", &dag_levels, py::arg("ops"), py::arg("modes"),
        "Level (0-based) of every task of a program-order tile DAG under RAW/WAR/WAW hazards");
  m.def("dag_versions", &dag_versions, py::arg("ops"), py::arg("modes"),
        "Version of each tile access (number of prior writes of that tile)");
}
