// Reduction trees of the hierarchical tile QR / LQ for the interpreter-free engine: the query interface of
// dplasma_qrtree_t (getnbgeqrf, getm, geti, gettype, currpiv, nextpiv, prevpiv) answered in C++ with the same
// semantics as models/qrtree.py (itself pinned to the reference's src/dplasma_hqr.c / dplasma_systolic_qr.c by
// tests/test_qrtree_parity.py), plus the per-panel elimination plan the native tile engine executes.
#pragma once
#include <memory>
#include <string>
#include <vector>

namespace nq {

enum { FLAT = 0, GREEDY = 1, FIBONACCI = 2, BINARY = 3, GREEDY1P = 4 };
enum { KILLED_BY_TS = 0, KILLED_BY_LOCALTREE = 1, KILLED_BY_DOMINO = 2, KILLED_BY_DISTTREE = 3 };

struct Kill {
  int piv, m, type;
};

// one of the two reduction levels of the hierarchical tree (models/qrtree.py _Sub and subclasses)
struct Sub {
  int ldd, a, p, min_mn;
  bool domino;
  Sub(int ldd_, int a_, int p_, bool dom, int mn) : ldd(ldd_), a(a_), p(p_), min_mn(mn), domino(dom) {}
  virtual ~Sub() {}
  int k_a(int k, int row) const { return domino ? k / a : (k + p - 1 - row % p) / p / a; }
  virtual int currpiv(int k, int m) const = 0;
  virtual int nextpiv(int k, int piv, int s) const = 0;
  virtual int prevpiv(int k, int piv, int s) const = 0;
};

class Tree {
 public:
  int mt = 0, nt = 0, a = 1, p = 1;
  std::string name;
  virtual ~Tree() {}
  virtual int getnbgeqrf(int k) const = 0;
  virtual int getm(int k, int i) const = 0;
  virtual int gettype(int k, int m) const = 0;
  virtual int currpiv(int k, int m) const = 0;
  virtual int nextpiv(int k, int piv, int start) const = 0;
  virtual int prevpiv(int k, int piv, int start) const = 0;
  // index of m among panel k's GEQRT rows (-1 if it is not one)
  int geti(int k, int m) const;
  // panel k's GEQRT rows (getm order) and its kills in post-order of the elimination tree: every
  // annihilator's kills in its nextpiv order, every row's own kills before the kill that eliminates it
  void plan(int k, std::vector<int>& heads, std::vector<Kill>& kills) const;
  // 0 if every panel's plan is a valid elimination (models/qrtree.py QRTree.check), else 1 with err set
  int check(std::string& err) const;
  std::string print_type() const;
  std::string print_pivot() const;
  std::string print_nbgeqrt() const;
  std::string dot(int k) const;
};

// dplasma_hqr_init semantics (a = -1: 4; domino < 0: automatic from the aspect ratio)
Tree* make_hqr(int mt, int nt, int llvl, int hlvl, int a, int p, int domino, int tsrr);
Tree* make_systolic(int mt, int nt, int p, int q);
Tree* make_svd(int mt, int nt, int hlvl, int p, int nbcores_per_node, int ratio, int nodes);

}  // namespace nq
