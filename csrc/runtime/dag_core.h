// Native core of the tile-DAG analysis (no Python dependency: used by the pybind11 module dag.cpp
// and by the sanitizer test driver tests/native/test_runtime_core.cpp).  See dag.cpp for the role.
#pragma once
#include <algorithm>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace dpl_dag {

struct TileState {
  int32_t last_write = -1;  // level of the last writer
  int32_t max_read = -1;    // max level of readers since that write
};

// ops/modes: row-major (n, R); modes 0 = unused slot, 1 = read, 2 = write, 3 = read+write.
// lv[n] receives the level (0-based) of every task under RAW / WAR / WAW hazards.
inline void levels(const int64_t* ops, const uint8_t* modes, int64_t n, int64_t R, int32_t* lv) {
  std::unordered_map<int64_t, TileState> st;
  st.reserve(static_cast<size_t>(std::min<int64_t>(n * 2 + 16, 1 << 24)));
  for (int64_t t = 0; t < n; ++t) {
    int32_t L = 0;
    for (int64_t r = 0; r < R; ++r) {
      const uint8_t m = modes[t * R + r];
      if (!m) continue;
      auto it = st.find(ops[t * R + r]);
      if (it == st.end()) continue;
      const TileState& s = it->second;
      if (s.last_write >= L) L = s.last_write + 1;        // RAW / WAW
      if ((m & 2) && s.max_read >= L) L = s.max_read + 1;  // WAR
    }
    lv[t] = L;
    for (int64_t r = 0; r < R; ++r) {
      const uint8_t m = modes[t * R + r];
      if (!m) continue;
      TileState& s = st[ops[t * R + r]];
      if (m & 2) {
        s.last_write = L;
        s.max_read = -1;
      } else if (L > s.max_read) {
        s.max_read = L;
      }
    }
  }
}

// v[n * R]: version of the tile each access touches (0 = initial data, v = after the v-th write)
inline void versions(const int64_t* ops, const uint8_t* modes, int64_t n, int64_t R, int32_t* v) {
  std::unordered_map<int64_t, int32_t> ver;
  for (int64_t t = 0; t < n; ++t) {
    for (int64_t r = 0; r < R; ++r) {
      v[t * R + r] = -1;
      if (!modes[t * R + r]) continue;
      auto it = ver.find(ops[t * R + r]);
      v[t * R + r] = it == ver.end() ? 0 : it->second;
    }
    for (int64_t r = 0; r < R; ++r)
      if (modes[t * R + r] & 2) ver[ops[t * R + r]] += 1;
  }
}

struct Schedule {
  std::vector<int32_t> level, blevel;  // level, bottom level (longest path to a sink)
  std::vector<int64_t> esrc, edst;     // deduplicated dependency edges (program order)
};

// Full schedule analysis.  Edges always point from an earlier to a later task in program order,
// so walking them backwards is a reverse topological order for the bottom-level pass.
inline Schedule schedule(const int64_t* ops, const uint8_t* modes, int64_t n, int64_t R) {
  struct St {
    int64_t writer = -1;           // last writing task
    std::vector<int64_t> readers;  // readers since that write
  };
  Schedule S;
  S.level.assign(n, 0);
  S.blevel.assign(n, 0);
  std::unordered_map<int64_t, St> st;
  st.reserve(static_cast<size_t>(std::min<int64_t>(n * 2 + 16, 1 << 24)));
  std::vector<int64_t> preds;
  S.esrc.reserve(n * 3);
  S.edst.reserve(n * 3);
  for (int64_t t = 0; t < n; ++t) {
    preds.clear();
    for (int64_t r = 0; r < R; ++r) {
      const uint8_t m = modes[t * R + r];
      if (!m) continue;
      auto it = st.find(ops[t * R + r]);
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
      L = std::max(L, S.level[p] + 1);
      S.esrc.push_back(p);
      S.edst.push_back(t);
    }
    S.level[t] = L;
    for (int64_t r = 0; r < R; ++r) {
      const uint8_t m = modes[t * R + r];
      if (!m) continue;
      St& s = st[ops[t * R + r]];
      if (m & 2) {
        s.writer = t;
        s.readers.clear();
      } else {
        s.readers.push_back(t);
      }
    }
  }
  for (int64_t i = static_cast<int64_t>(S.esrc.size()) - 1; i >= 0; --i) {
    const int64_t s = S.esrc[i], d = S.edst[i];
    S.blevel[s] = std::max(S.blevel[s], S.blevel[d] + 1);
  }
  return S;
}

// ---------------------------------------------------------------- ready-queue list scheduler
// The issue order of a task graph under one of the reference's scheduler policies (PaRSEC's
// "-o" choice, tests/common.c): tasks become ready when all predecessors are issued and are taken
// from the ready set by the policy's key.  pred_ptr / pred_idx: CSR predecessor lists (any order).
enum Policy : int {
  POL_PROGRAM = 0,  // program order (default)
  POL_PRIO = 1,     // highest priority first, ties in program order (lfq, ltq, pbq, lhq, spq, ap)
  POL_INVPRIO = 2,  // lowest priority first (ip)
  POL_FIFO = 3,     // breadth first: in order of readiness (gd, global dequeue)
  POL_LIFO = 4,     // depth first: most recently readied first (ll, local LIFO)
  POL_RANDOM = 5    // uniformly random among ready tasks (rnd), seeded
};

inline std::vector<int64_t> list_schedule(int64_t n, const int64_t* pred_ptr, const int64_t* pred_idx,
                                          const int32_t* prio, int policy, uint64_t seed) {
  std::vector<int64_t> order;
  order.reserve(static_cast<size_t>(n));
  std::vector<int64_t> npred(static_cast<size_t>(n)), succ_ptr(static_cast<size_t>(n) + 1, 0);
  for (int64_t t = 0; t < n; ++t) {
    npred[t] = pred_ptr[t + 1] - pred_ptr[t];
    for (int64_t e = pred_ptr[t]; e < pred_ptr[t + 1]; ++e) ++succ_ptr[pred_idx[e] + 1];
  }
  for (int64_t t = 0; t < n; ++t) succ_ptr[t + 1] += succ_ptr[t];
  std::vector<int64_t> succ(static_cast<size_t>(succ_ptr[n])), fill(succ_ptr.begin(), succ_ptr.end() - 1);
  for (int64_t t = 0; t < n; ++t)
    for (int64_t e = pred_ptr[t]; e < pred_ptr[t + 1]; ++e) succ[fill[pred_idx[e]]++] = t;
  // ready set: a max-heap on (key, -tid) -- the key encodes the policy
  uint64_t rng = seed * 6364136223846793005ULL + 1442695040888963407ULL;
  int64_t stamp = 0;
  struct Item {
    int64_t k1, k2, tid;
    bool operator<(const Item& o) const {
      if (k1 != o.k1) return k1 < o.k1;
      if (k2 != o.k2) return k2 < o.k2;
      return tid > o.tid;  // smaller tid wins ties
    }
  };
  std::vector<Item> heap;
  auto push = [&](int64_t t) {
    Item it{0, 0, t};
    switch (policy) {
      case POL_PRIO: it.k1 = prio[t]; break;
      case POL_INVPRIO: it.k1 = -static_cast<int64_t>(prio[t]); break;
      case POL_FIFO: it.k1 = -(stamp++); break;
      case POL_LIFO: it.k1 = stamp++; break;
      case POL_RANDOM:
        rng = rng * 6364136223846793005ULL + 1442695040888963407ULL;
        it.k1 = static_cast<int64_t>(rng >> 17);
        break;
      default: it.k1 = -t; break;
    }
    heap.push_back(it);
    std::push_heap(heap.begin(), heap.end());
  };
  for (int64_t t = 0; t < n; ++t)
    if (npred[t] == 0) push(t);
  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end());
    const int64_t t = heap.back().tid;
    heap.pop_back();
    order.push_back(t);
    for (int64_t e = succ_ptr[t]; e < succ_ptr[t + 1]; ++e)
      if (--npred[succ[e]] == 0) push(succ[e]);
  }
  return order;  // shorter than n only if the graph has a cycle
}

}  // namespace dpl_dag
