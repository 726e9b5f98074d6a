// Reduction trees of the hierarchical tile QR in C++ (see native_qrtree.h).  Every formula follows
// models/qrtree.py line by line (the Python module documents each one and cites its reference source:
// HQR src/dplasma_hqr.c:182-322 / 1241-1640 / 1790-1945, systolic src/dplasma_systolic_qr.c, the adaptive
// SVD tree src/dplasma_hqr.c:1975-2700); tests/test_qrtree_native.py checks this port against the
// reference-oracle digests of tests/fixtures/qrtree_ref.json, tree by tree.
#include "native_qrtree.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <set>
#include <utility>

namespace nq {
namespace {

// C remainder of the reference formulas (C++ % already truncates)
inline int nbextra1(int k, int pa, int p) { return (k % pa) > (pa - p) ? (-k) % pa + pa : 0; }
inline int ilog2_floor(int x) { return x > 0 ? (int)(std::log((double)x) / std::log(2.0)) : -1; }
inline int ceil_div(int x, int y) { return (x + y - 1) / y; }   // x >= 0, y > 0

// ---------------------------------------------------------------------------- low-level trees
struct LowFlat : Sub {
  using Sub::Sub;
  int currpiv(int k, int m) const override { return k_a(k, m); }
  int nextpiv(int k, int pv, int s) const override {
    const int ka = k_a(k, pv), ppa = (pv / p) / a;
    if (s <= ppa) return ldd;
    if (ppa == ka && ldd - ka > 1) {
      if (s == ldd) return ppa + 1;
      if (s < ldd) return s + 1;
    }
    return ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    const int ka = k_a(k, pv), ppa = (pv / p) / a;
    if (ppa == ka && ldd - ka > 1) {
      if (s == ppa) return ldd - 1;
      if (s > ppa + 1) return s - 1;
    }
    return ldd;
  }
};

struct LowBinary : Sub {
  using Sub::Sub;
  int currpiv(int k, int m) const override {
    const int ka = k_a(k, m), mpa = (m / p) / a, d = mpa - ka;
    return d == 0 ? 0 : mpa - (d & -d);
  }
  int nextpiv(int k, int pv, int s) const override {
    const int ka = k_a(k, pv), ppa = (pv / p) / a;
    if (s <= ppa) return ldd;
    const int off = ppa - ka;
    int bit = 0;
    if (s != ldd) {
      while (bit < 30 && ((s - ka) & (1 << bit)) == 0) ++bit;
      ++bit;
    }
    const int t = off | (1 << bit);
    return (t != off && t + ka < ldd) ? t + ka : ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    const int ka = k_a(k, pv), ppa = (pv / p) / a, off = ppa - ka;
    if (s == ppa && off % 2 == 0) {
      int bit = 0;
      if (off == 0) {
        bit = ilog2_floor(ldd - ka);
      } else {
        while (bit < 30 && (off & (1 << bit)) == 0) ++bit;
      }
      for (int i = bit; i >= 0; --i) {
        const int t = off | (1 << i);
        if (off != t && t + ka < ldd) return t + ka;
      }
      return ldd;
    }
    if (s - ppa > 1) return ppa + ((s - ppa) >> 1);
    return ldd;
  }
};

// trees given by a pivot table: nextpiv scans down from start - 1, prevpiv up from start + 1
struct LowTable : Sub {
  using Sub::Sub;
  virtual const std::vector<int>& col(int k, int row) const = 0;
  virtual int ppa_of(int pv) const { return (pv / p) / a; }
  int currpiv(int k, int m) const override { return col(k, m)[(m / p) / a]; }
  int nextpiv(int k, int pv, int s) const override {
    const std::vector<int>& c = col(k, pv);
    const int ka = k_a(k, pv), ppa = ppa_of(pv);
    for (int i = s - 1; i > ka; --i)
      if (c[i] == ppa) return i;
    return ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    const std::vector<int>& c = col(k, pv);
    const int ppa = (pv / p) / a;
    for (int i = s + 1; i < ldd; ++i)
      if (c[i] == ppa) return i;
    return ldd;
  }
};

struct LowFib : LowTable {
  std::vector<std::vector<int>> tab;
  LowFib(int ldd_, int a_, int p_, bool dom, int mn) : LowTable(ldd_, a_, p_, dom, mn) {
    const int mt = ldd;
    tab.assign(std::max(1, min_mn), std::vector<int>(std::max(1, mt), 0));
    int f1 = 1, m = 1;
    while (m < mt) {
      int kk = 0;
      while (kk < f1 && m < mt) {
        tab[0][m] = m - f1;
        ++kk;
        ++m;
      }
      ++f1;
    }
    for (int k = 1; k < min_mn; ++k)
      for (int m2 = k + 1; m2 < mt; ++m2) tab[k][m2] = tab[k - 1][m2 - 1] + 1;
  }
  const std::vector<int>& col(int k, int row) const override { return tab[k_a(k, row)]; }
};

struct LowGreedy : LowTable {
  std::vector<std::vector<std::vector<int>>> tab;   // [section][k][domain]
  LowGreedy(int ldd_, int a_, int p_, bool dom, int mn, bool init = true) : LowTable(ldd_, a_, p_, dom, mn) {
    if (init) build();
  }
  void build() {
    const int mt = ldd, pa = p * a;
    if (domino) {
      min_mn = std::min(min_mn, mt * a);
      const int mn = min_mn;
      std::vector<std::vector<int>> t(mn, std::vector<int>(mt, 0));
      std::vector<int> nT(mn, 0), nZ(mn, 0);
      nT[0] = mt;
      int k = 0, first = 0;
      while (!(nT[mn - 1] == mt - (mn - 1) / a && nZ[mn - 1] + 1 == nT[mn - 1]) && first < mn) {
        const int h = (nT[k] - nZ[k]) / 2;
        if (h == 0) {
          while (first < mn && nT[first] == mt - first / a && nZ[first] + 1 == nT[first]) {
            if (first % a != a - 1 && first < mn - 1) nT[first + 1] += 1;
            ++first;
          }
          k = first;
          continue;
        }
        if (k < mn - 1) nT[k + 1] += h;
        const int top = mt - nZ[k] - 1;
        nZ[k] += h;
        for (int j = top; j > top - h; --j) t[k][j] = j - h;
        ++k;
        if (k > mn - 1) k = first;
      }
      tab.push_back(std::move(t));
      return;
    }
    const int mn = min_mn;
    for (int r = 0; r < p; ++r) {
      std::vector<std::vector<int>> t(mn, std::vector<int>(mt, 0));
      int lmn = mn;
      std::vector<int> todo(mn, 0);
      for (int k = 0; k < mn; ++k) {
        todo[k] = std::max(mt - (k + p - 1 - r) / pa, 0);
        if (todo[k] == 0) {
          lmn = k;
          break;
        }
      }
      std::vector<int> nT(mn, 0), nZ(mn, 0);
      nT[0] = mt;
      int k = 0, first = 0;
      while (lmn > 0 && !(nT[lmn - 1] == todo[lmn - 1] && nZ[lmn - 1] + 1 == nT[lmn - 1]) && first < lmn) {
        const int h = (nT[k] - nZ[k]) / 2;
        if (h == 0) {
          while (first < lmn && nT[first] == todo[first] && nZ[first] + 1 == nT[first]) {
            if (first < lmn - 1 && first % pa != (a - 1) * p + r) nT[first + 1] += 1;
            ++first;
          }
          k = first;
          continue;
        }
        if (k < lmn - 1) nT[k + 1] += h;
        const int top = mt - nZ[k] - 1;
        nZ[k] += h;
        for (int j = top; j > top - h; --j) t[k][j] = j - h;
        ++k;
        if (k > lmn - 1) k = first;
      }
      tab.push_back(std::move(t));
    }
  }
  const std::vector<int>& col(int k, int row) const override { return tab[domino ? 0 : row % p][k]; }
  int ppa_of(int pv) const override { return pv / (p * a); }
};

struct LowGreedy1p : LowGreedy {
  LowGreedy1p(int ldd_, int a_, int p_, bool dom, int mn) : LowGreedy(ldd_, a_, p_, dom, mn, false) {
    const int mt = ldd, pa = p * a;
    auto halve = [&](std::vector<int>& c, int nTv) {
      int nZ = 0;
      while (nZ < nTv - 1) {
        const int h = (nTv - nZ) / 2;
        const int top = mt - nZ - 1;
        nZ += h;
        for (int j = top; j > top - h; --j) c[j] = j - h;
      }
    };
    if (domino) {
      min_mn = std::min(mn, mt * a);
      std::vector<std::vector<int>> t(min_mn, std::vector<int>(mt, 0));
      for (int k = 0; k < min_mn; ++k) halve(t[k], std::max(mt - k / a, 0));
      tab.push_back(std::move(t));
    } else {
      for (int r = 0; r < p; ++r) {
        std::vector<std::vector<int>> t(mn, std::vector<int>(mt, 0));
        for (int k = 0; k < mn; ++k) {
          const int nTv = std::max(mt - (k + p - 1 - r) / pa, 0);
          if (nTv == 0) break;
          halve(t[k], nTv);
        }
        tab.push_back(std::move(t));
      }
    }
  }
};

// ---------------------------------------------------------------------------- high-level (distributed band) trees
struct HighFlat : Sub {
  using Sub::Sub;
  int currpiv(int k, int) const override { return k; }
  int nextpiv(int k, int pv, int s) const override {
    if (pv == k && ldd > 1) {
      if (s == ldd) return pv + 1;
      if (s < ldd && s - k < p - 1) return s + 1;
    }
    return ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    if (pv == k && ldd > 1) {
      if (s == pv && pv != ldd - 1) return std::min(pv + p - 1, ldd - 1);
      if (s > pv + 1 && s - k < p) return s - 1;
    }
    return ldd;
  }
};

struct HighBinary : Sub {
  using Sub::Sub;
  int currpiv(int k, int m) const override {
    const int d = m - k;
    return d == 0 ? 0 : m - (d & -d);
  }
  int nextpiv(int k, int pv, int s) const override {
    if (s <= pv) return ldd;
    const int off = pv - k;
    int bit = 0;
    if (s != ldd) {
      while (bit < 30 && ((s - k) & (1 << bit)) == 0) ++bit;
      ++bit;
    }
    const int t = off | (1 << bit);
    return (t != off && t < p && t + k < ldd) ? t + k : ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    const int off = pv - k;
    if (s == pv && off % 2 == 0) {
      int bit = 0;
      if (off == 0) {
        bit = ilog2_floor(std::min(p, ldd - k));
      } else {
        while (bit < 30 && (off & (1 << bit)) == 0) ++bit;
      }
      for (int i = bit; i >= 0; --i) {
        const int t = off | (1 << i);
        if (off != t && t < p && t + k < ldd) return t + k;
      }
      return ldd;
    }
    if (s - pv > 1) return pv + ((s - pv) >> 1);
    return ldd;
  }
};

struct HighFib : Sub {
  std::vector<int> tab;
  HighFib(int ldd_, int a_, int p_, bool dom, int mn, bool greedy1p) : Sub(ldd_, a_, p_, dom, mn) {
    tab.assign(std::max(1, p), 0);
    if (greedy1p) {
      const int mt = ldd;
      const int nT = mt;
      int nZ = std::max(mt - p, 0);
      while (!(nT == mt && nZ + 1 == nT)) {
        const int h = (nT - nZ) / 2;
        if (h == 0) break;
        const int top = mt - nZ - 1;
        nZ += h;
        for (int j = top; j > top - h; --j) tab[j] = j - h;
      }
    } else {
      int f1 = 1, m = 1;
      while (m < p) {
        int kk = 0;
        while (kk < f1 && m < p) {
          tab[m] = m - f1;
          ++kk;
          ++m;
        }
        ++f1;
      }
    }
  }
  int currpiv(int k, int m) const override { return tab[m - k] + k; }
  int nextpiv(int k, int pv, int s) const override {
    for (int i = std::min(s - k - 1, p - 1); i > 0; --i)
      if (tab[i] == pv - k) return i + k;
    return ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    const int lp = pv - k, end = std::min(ldd - k, p);
    for (int i = s - k + 1; i < end; ++i)
      if (tab[i] == lp) return i + k;
    return ldd;
  }
};

struct HighGreedy : Sub {
  std::vector<std::vector<int>> tab;
  HighGreedy(int ldd_, int a_, int p_, bool dom, int mn) : Sub(ldd_, a_, p_, dom, mn) {
    const int mt = ldd;
    tab.assign(std::max(1, mn), std::vector<int>(std::max(1, p), 0));
    if (mn <= 0) return;
    std::vector<int> nT(mn, 0), nZ(mn, 0);
    nT[0] = mt;
    nZ[0] = std::max(mt - p, 0);
    for (int k = 1; k < mn; ++k) nT[k] = nZ[k] = std::max(mt - k - p, 0);
    int k = 0, first = 0;
    while (!(nT[mn - 1] == mt - (mn - 1) && nZ[mn - 1] + 1 == nT[mn - 1]) && first < mn) {
      const int h = (nT[k] - nZ[k]) / 2;
      if (h == 0) {
        while (first < mn && nT[first] == mt - first && nZ[first] + 1 == nT[first]) ++first;
        k = first;
        continue;
      }
      const int top = mt - nZ[k] - 1;
      nZ[k] += h;
      if (k < mn - 1) nT[k + 1] = nZ[k];
      for (int j = top; j > top - h; --j) tab[k][j - k] = j - h;
      ++k;
      if (k > mn - 1) k = first;
    }
  }
  int currpiv(int k, int m) const override { return tab[k][m - k]; }
  int nextpiv(int k, int pv, int s) const override {
    for (int i = std::min(s - 1, k + p - 1); i > k; --i)
      if (tab[k][i - k] == pv) return i;
    return ldd;
  }
  int prevpiv(int k, int pv, int s) const override {
    for (int i = s - k + 1; i < p; ++i)
      if (tab[k][i] == pv) return k + i;
    return ldd;
  }
};

Sub* low_tree(int kind, int ldd, int a, int p, bool domino, int mn) {
  switch (kind) {
    case FLAT: return new LowFlat(ldd, a, p, domino, mn);
    case FIBONACCI: return new LowFib(ldd, a, p, domino, mn);
    case BINARY: return new LowBinary(ldd, a, p, domino, mn);
    case GREEDY1P: return new LowGreedy1p(ldd, a, p, domino, mn);
    default: return new LowGreedy(ldd, a, p, domino, mn);
  }
}

Sub* high_tree(int kind, int mt, int a, int p, bool domino, int mn, bool default_flat) {
  if (kind == FLAT) return new HighFlat(mt, a, p, domino, mn);
  if (kind == GREEDY) return new HighGreedy(mt, a, p, domino, mn);
  if (kind == GREEDY1P) return new HighFib(mt, a, p, domino, mn, true);
  if (kind == BINARY) return new HighBinary(mt, a, p, domino, mn);
  if (kind == FIBONACCI || !default_flat) return new HighFib(mt, a, p, domino, mn, false);
  return new HighFlat(mt, a, p, domino, mn);
}

// ---------------------------------------------------------------------------- HQR
class HqrTree : public Tree {
 public:
  int llvl, hlvl;
  bool domino, tsrr;
  std::unique_ptr<Sub> low, high;
  std::vector<std::vector<int>> perm;
  std::vector<std::map<int, int>> inv;

  HqrTree(int mt_, int nt_, int llvl_, int hlvl_, int a_, int p_, int domino_, int tsrr_) : llvl(llvl_), hlvl(hlvl_) {
    int aa = a_ == -1 ? 4 : std::max(a_, 1);
    const int pp = std::max(p_, 1);
    const double ratio = mt_ ? (double)nt_ / mt_ : 1.0;
    domino = domino_ >= 0 ? domino_ != 0 : ratio < 0.5;
    tsrr = tsrr_ != 0;
    aa = std::min(aa, mt_);
    mt = mt_;
    nt = nt_;
    a = std::max(aa, 1);
    p = pp;
    name = "hqr";
    const int min_mn = std::min(mt, nt);
    const int low_mt = (mt + p * a - 1) / (p * a);
    low.reset(low_tree(llvl, low_mt, a, p, domino, min_mn));
    if (p > 1) high.reset(high_tree(hlvl, mt, a, p, domino, min_mn, ratio >= 0.5));
    genperm();
  }

  void genperm() {
    const int m = mt, n = nt, pa = p * a;
    const int endpa = m - m % pa;
    for (int k = 0; k < std::min(m, n); ++k) {
      std::vector<int> pm(m + 1, -1);
      if (!tsrr) {
        for (int i = 0; i <= m; ++i) pm[i] = i;
      } else {
        int end2 = p + (domino ? k * p : k + nbextra1(k, pa, p));
        end2 = std::min(ceil_div(end2, pa) * pa, m);
        for (int i = k; i < end2; ++i) pm[i] = i;
        int i = std::max(end2, k);
        while (i < endpa) {
          for (int j = 0; j < pa; ++j) pm[i + j] = i + (j + p * (k % a)) % pa;
          i += pa;
        }
        for (; i < m; ++i) pm[i] = i;
        pm[m] = m;
      }
      std::map<int, int> iv;
      for (int i = 0; i <= m; ++i)
        if (pm[i] >= 0) iv[pm[i]] = i;
      perm.push_back(std::move(pm));
      inv.push_back(std::move(iv));
    }
  }

  int invperm(int k, int m) const {
    if (a == 1) return m;
    auto it = inv[k].find(m);
    return it == inv[k].end() ? m : it->second;
  }

  int getnbgeqrf(int k) const override {
    const int pa = p * a, gmt = mt;
    int nb2, nb11;
    if (domino) {
      nb2 = k * (p - 1);
      nb11 = ceil_div(p * (k + 1), pa) * pa;
    } else {
      nb2 = nbextra1(k, pa, p);
      nb11 = ceil_div(k + p, pa) * pa;
    }
    const int nb12 = (gmt / pa) * pa;
    const int nb1 = (nb12 - nb11) / a + std::min(p, gmt - nb12);   // C truncation, as the reference
    return std::min(nb1 + nb2 + p, gmt - k);
  }

  int getm(int k, int i) const override {
    const int pa = p * a;
    const int nb23 = p + (domino ? k * (p - 1) : nbextra1(k, pa, p));
    if (i < nb23) return k + i;
    const int j = i - nb23;
    const int pos1 = ceil_div(domino ? p * (k + 1) : p + k, pa) * pa;
    return perm[k][pos1 + (j / p) * pa + j % p];
  }

  int gettype(int k, int m) const override {
    const int lm = invperm(k, m);
    if (lm < k + p) return KILLED_BY_DISTTREE;
    if (domino && lm < p * (k + 1)) return KILLED_BY_DOMINO;
    return (lm / p) % a == 0 ? KILLED_BY_LOCALTREE : KILLED_BY_TS;
  }

  int currpiv(int k, int m) const override {
    const int gmt = mt;
    const int pm = invperm(k, m);
    const int lm = pm / p, rank = pm % p;
    const std::vector<int>& pr = perm[k];
    const int t = gettype(k, m);
    if (domino) {
      if (t == KILLED_BY_TS) {
        const int tmp = lm / a;
        return tmp == k / a ? pr[k * p + rank] : pr[tmp * a * p + rank];
      }
      if (t == KILLED_BY_LOCALTREE) {
        const int tmp = low->currpiv(k, pm);
        return pr[tmp == k / a ? k * p + rank : tmp * a * p + rank];
      }
      if (t == KILLED_BY_DOMINO) return m - p;
      return high ? high->currpiv(k, pm) : gmt;
    }
    const int tmpk = k / (p * a);
    if (t == KILLED_BY_TS) {
      const int tmp = lm / a;
      return pr[tmp == tmpk ? k + (pm - k) % p : tmp * a * p + rank];
    }
    if (t == KILLED_BY_LOCALTREE) {
      const int tmp = low->currpiv(k, pm);
      return pr[tmp == tmpk ? k + (pm - k) % p : tmp * a * p + rank];
    }
    if (t == KILLED_BY_DOMINO) return pr[pm - p];
    return high ? pr[high->currpiv(k, pm)] : gmt;
  }

  int nextpiv(int k, int opivot, int ostart) const override {
    const int gmt = mt;
    int start = ostart != gmt ? invperm(k, ostart) : gmt;
    const int pivot = invperm(k, opivot);
    const int lpivot = pivot / p, rpivot = pivot % p;
    int lstart = start == gmt ? low->ldd * a : start / p;
    const std::vector<int>& pr = perm[k];
    const int ls = start < gmt ? gettype(k, ostart) : -1;
    const int lp = gettype(k, opivot);
    int stage = ls;
    if (stage == -1) {
      if (lp == KILLED_BY_TS) return gmt;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      if (!(domino && lpivot < k)) {
        const int nextp = start == gmt ? pivot + p : start + p;
        if (nextp < gmt && nextp < pivot + a * p && (nextp / p) % a != 0) return pr[nextp];
        start = gmt;
        lstart = low->ldd * a;
        stage = KILLED_BY_LOCALTREE;
      } else {
        stage = KILLED_BY_DOMINO;
        start = gmt;
        lstart = low->ldd * a;
      }
    }
    if (stage == KILLED_BY_LOCALTREE) {
      if (!(domino && lpivot < k)) {
        int tmp = low->nextpiv(k, pivot, lstart / a);
        if (tmp * a * p + rpivot >= gmt && tmp == low->ldd - 1) tmp = low->nextpiv(k, pivot, tmp);
        if (tmp != low->ldd) return pr[tmp * a * p + rpivot];
      }
      start = gmt;
      lstart = low->ldd * a;
      stage = KILLED_BY_DOMINO;
    }
    if (stage == KILLED_BY_DOMINO) {
      if (lp < KILLED_BY_DOMINO) return gmt;
      if (domino && start == gmt && lpivot < k && pivot + p < gmt) return pr[pivot + p];
      start = gmt;
      lstart = low->ldd * a;
      stage = KILLED_BY_DISTTREE;
    }
    (void)lstart;
    if (stage == KILLED_BY_DISTTREE) {
      if (lp < KILLED_BY_DISTTREE) return gmt;
      if (high) {
        const int tmp = high->nextpiv(k, pivot, start);
        if (tmp != gmt) return pr[tmp];
      }
    }
    return gmt;
  }

  int prevpiv(int k, int opivot, int ostart) const override {
    const int gmt = mt;
    int start = invperm(k, ostart);
    const int pivot = invperm(k, opivot);
    const int lpivot = pivot / p, rpivot = pivot % p;
    int lstart = start / p;
    const std::vector<int>& pr = perm[k];
    const int ls = gettype(k, ostart), lp = gettype(k, opivot);
    if (lp == KILLED_BY_TS) return gmt;
    int stage = ls;
    if (stage == KILLED_BY_DISTTREE) {
      if (high) {
        const int tmp = high->prevpiv(k, pivot, start);
        if (tmp != gmt) return pr[tmp];
      }
      start = pivot;
      lstart = pivot / p;
      stage = KILLED_BY_DOMINO;
    }
    if (stage == KILLED_BY_DOMINO) {
      if (domino && lpivot < k) {
        if (start == pivot && start + p < gmt) return pr[start + p];
        if (lp > KILLED_BY_LOCALTREE) return gmt;
      }
      start = pivot;
      lstart = pivot / p;
      stage = KILLED_BY_LOCALTREE;
    }
    if (stage == KILLED_BY_LOCALTREE) {
      if (domino && lpivot < k) return gmt;
      int tmp = low->prevpiv(k, pivot, lstart / a);
      if (tmp * a * p + rpivot >= gmt && tmp == low->ldd - 1) tmp = low->prevpiv(k, pivot, tmp);
      if (tmp != low->ldd) return pr[tmp * a * p + rpivot];
      start = pivot;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      int nextp;
      if (start == pivot) {
        const int tmp = lpivot + a - 1 - lpivot % a;
        nextp = tmp * p + rpivot;
        while (pivot < nextp && nextp >= gmt) nextp -= p;
      } else {
        nextp = start - p;
      }
      if (pivot < nextp) return pr[nextp];
    }
    return gmt;
  }
};

// ---------------------------------------------------------------------------- systolic
class SystolicTree : public Tree {
 public:
  SystolicTree(int mt_, int nt_, int p_, int q_) {
    mt = mt_;
    nt = nt_;
    a = std::max(1, q_);
    p = std::max(1, p_);
    name = "systolic";
  }
  int getnbgeqrf(int k) const override { return std::min(p * a, mt - k); }
  int getm(int k, int i) const override { return k + i; }
  int gettype(int k, int m) const override {
    const int pq = p * a;
    if (m >= k + pq) return KILLED_BY_TS;
    return m >= k + p ? KILLED_BY_LOCALTREE : KILLED_BY_DISTTREE;
  }
  int currpiv(int k, int m) const override {
    const int pq = p * a, t = gettype(k, m);
    if (t == KILLED_BY_TS) return (m - k) % pq + k;
    if (t == KILLED_BY_LOCALTREE) return (m - k) % p + k;
    return k;
  }
  int nextpiv(int k, int pivot, int start) const override {
    const int q = a, pq = p * q;
    const int ls = start < mt ? gettype(k, start) : -1, lp = gettype(k, pivot);
    int stage = ls;
    if (stage == -1) {
      if (lp == KILLED_BY_TS) return mt;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      const int nextp = start == mt ? pivot + pq : start + pq;
      if (nextp < mt) return nextp;
      start = mt;
      stage = KILLED_BY_LOCALTREE;
    }
    if (stage == KILLED_BY_LOCALTREE) {
      if (lp < KILLED_BY_DISTTREE) return mt;
      const int nextp = start == mt ? pivot + p : start + p;
      if (k + p <= nextp && nextp < std::min(k + pq, mt)) return nextp;
      start = mt;
      stage = KILLED_BY_DISTTREE;
    }
    if (stage == KILLED_BY_DISTTREE) {
      if (pivot > k) return mt;
      const int nextp = start == mt ? pivot + 1 : start + 1;
      if (nextp < k + p) return nextp;
    }
    return mt;
  }
  int prevpiv(int k, int pivot, int start) const override {
    const int q = a, pq = p * q, rpivot = pivot % pq;
    const int ls = gettype(k, start), lp = gettype(k, pivot);
    if (lp == KILLED_BY_TS) return mt;
    int stage = ls;
    if (stage == KILLED_BY_DISTTREE) {
      if (pivot == k) {
        int nextp;
        if (start == pivot) {
          nextp = start + p - 1;
          while (pivot < nextp && nextp >= mt) nextp -= 1;
        } else {
          nextp = start - 1;
        }
        if (pivot < nextp && nextp < k + p) return nextp;
      }
      start = pivot;
      stage = KILLED_BY_LOCALTREE;
    }
    if (stage == KILLED_BY_LOCALTREE) {
      if (lp > KILLED_BY_LOCALTREE) {
        int nextp;
        if (start == pivot) {
          nextp = start + (q - 1) * p;
          while (pivot < nextp && nextp >= mt) nextp -= p;
        } else {
          nextp = start - p;
        }
        if (pivot < nextp && nextp < k + pq) return nextp;
      }
      start = pivot;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      if (lp > KILLED_BY_TS) {
        int nextp;
        if (start == pivot) {
          nextp = mt - (mt - rpivot - 1) % pq - 1;
          while (pivot < nextp && nextp >= mt) nextp -= pq;
        } else {
          nextp = start - pq;
        }
        if (pivot < nextp) return nextp;
      }
    }
    return mt;
  }
};

// ---------------------------------------------------------------------------- adaptive SVD tree
class SvdTree : public Tree {
 public:
  int hlvl;
  std::vector<int> sa, sldd;                            // per panel: domain size, number of domains
  std::vector<std::vector<std::vector<int>>> lowtab;    // [rank][k] -> greedy pivot column
  std::unique_ptr<Sub> high;

  SvdTree(int mt_, int nt_, int hlvl_, int p_, int nbcores_per_node, int ratio, int nodes) : hlvl(hlvl_) {
    const int pp = std::max(p_, 1);
    mt = mt_;
    nt = nt_;
    a = -1;
    p = pp;
    name = "svd";
    if (nodes <= 0) nodes = pp;
    const int cores = std::max(1, nbcores_per_node) * std::max(1, nodes / pp);
    ratio = std::max(1, ratio);
    const int min_mn = std::min(mt, nt);
    for (int k = 0; k < min_mn; ++k) {
      const int height = ceil_div(mt - k, p);
      int aa = std::max(height * (nt - k) / (ratio * cores), 1);
      const int j = ceil_div(height, aa);
      aa = ceil_div(mt - k, j);
      sa.push_back(aa);
      sldd.push_back(ceil_div(mt, p * aa));
    }
    for (int r = 0; r < p; ++r) {
      std::vector<std::vector<int>> cols;
      for (int k = 0; k < min_mn; ++k) {
        const int aa = sa[k], ldd = sldd[k];
        std::vector<int> c(std::max(ldd, 1), 0);
        const int nT = std::max(ldd - (k + p - 1 - r) / (p * aa), 0);
        int nZ = 0;
        while (nZ < nT - 1) {
          const int h = (nT - nZ) / 2;
          const int top = ldd - nZ - 1;
          nZ += h;
          for (int jj = top; jj > top - h; --jj) c[jj] = jj - h;
        }
        cols.push_back(std::move(c));
      }
      lowtab.push_back(std::move(cols));
    }
    if (p > 1) high.reset(high_tree(hlvl, mt, -1, p, false, min_mn, false));
  }

  int ka(int k, int row) const { return (k + p - 1 - row % p) / p / sa[k]; }

  int getnbgeqrf(int k) const override {
    const int aa = sa[k], pa = p * aa, gmt = mt;
    const int nb2 = nbextra1(k, pa, p);
    const int nb11 = ceil_div(k + p, pa) * pa;
    const int nb12 = (gmt / pa) * pa;
    const int nb1 = (nb12 - nb11) / aa + std::min(p, gmt - nb12);
    return std::min(nb1 + nb2 + p, gmt - k);
  }
  int getm(int k, int i) const override {
    const int aa = sa[k], pa = p * aa;
    const int nb23 = p + nbextra1(k, pa, p);
    if (i < nb23) return k + i;
    const int j = i - nb23;
    const int pos1 = ceil_div(p + k, pa) * pa;
    return pos1 + (j / p) * pa + j % p;
  }
  int gettype(int k, int m) const override {
    if (m < k + p) return KILLED_BY_DISTTREE;
    return (m / p) % sa[k] == 0 ? KILLED_BY_LOCALTREE : KILLED_BY_TS;
  }
  int low_currpiv(int k, int m) const { return lowtab[m % p][k][(m / p) / sa[k]]; }
  int low_nextpiv(int k, int piv, int s) const {
    const std::vector<int>& c = lowtab[piv % p][k];
    const int ppa = piv / (p * sa[k]), kk = ka(k, piv);
    for (int i = s - 1; i > kk; --i)
      if (c[i] == ppa) return i;
    return sldd[k];
  }
  int low_prevpiv(int k, int piv, int s) const {
    const std::vector<int>& c = lowtab[piv % p][k];
    const int ppa = piv / p / sa[k];
    for (int i = s + 1; i < sldd[k]; ++i)
      if (c[i] == ppa) return i;
    return sldd[k];
  }
  int currpiv(int k, int m) const override {
    const int aa = sa[k], gmt = mt;
    const int lm = m / p, rank = m % p, t = gettype(k, m), tmpk = k / (p * aa);
    if (t == KILLED_BY_TS) {
      const int tmp = lm / aa;
      return tmp == tmpk ? k + (m - k) % p : tmp * aa * p + rank;
    }
    if (t == KILLED_BY_LOCALTREE) {
      const int tmp = low_currpiv(k, m);
      return tmp == tmpk ? k + (m - k) % p : tmp * aa * p + rank;
    }
    return high ? high->currpiv(k, m) : gmt;
  }
  int nextpiv(int k, int pivot, int start) const override {
    const int gmt = mt, aa = sa[k], ldd = sldd[k], rpivot = pivot % p;
    int lstart = start == gmt ? ldd * aa : start / p;
    const int ls = start < gmt ? gettype(k, start) : -1, lp = gettype(k, pivot);
    int stage = ls;
    if (stage == -1) {
      if (lp == KILLED_BY_TS) return gmt;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      const int nextp = start == gmt ? pivot + p : start + p;
      if (nextp < gmt && nextp < pivot + aa * p && (nextp / p) % aa != 0) return nextp;
      start = gmt;
      lstart = ldd * aa;
      stage = KILLED_BY_LOCALTREE;
    }
    if (stage == KILLED_BY_LOCALTREE) {
      int tmp = low_nextpiv(k, pivot, lstart / aa);
      if (tmp * aa * p + rpivot >= gmt && tmp == ldd - 1) tmp = low_nextpiv(k, pivot, tmp);
      if (tmp != ldd) return tmp * aa * p + rpivot;
      start = gmt;
      stage = KILLED_BY_DISTTREE;
    }
    if (stage == KILLED_BY_DISTTREE) {
      if (lp < KILLED_BY_DISTTREE) return gmt;
      if (high) {
        const int tmp = high->nextpiv(k, pivot, start);
        if (tmp != gmt) return tmp;
      }
    }
    return gmt;
  }
  int prevpiv(int k, int pivot, int start) const override {
    const int gmt = mt, aa = sa[k], ldd = sldd[k];
    const int lpivot = pivot / p, rpivot = pivot % p;
    int lstart = start / p;
    const int ls = gettype(k, start), lp = gettype(k, pivot);
    if (lp == KILLED_BY_TS) return gmt;
    int stage = ls;
    if (stage == KILLED_BY_DISTTREE) {
      if (high) {
        const int tmp = high->prevpiv(k, pivot, start);
        if (tmp != gmt) return tmp;
      }
      start = pivot;
      lstart = pivot / p;
      stage = KILLED_BY_LOCALTREE;
    }
    if (stage == KILLED_BY_LOCALTREE) {
      int tmp = low_prevpiv(k, pivot, lstart / aa);
      if (tmp * aa * p + rpivot >= gmt && tmp == ldd - 1) tmp = low_prevpiv(k, pivot, tmp);
      if (tmp != ldd) return tmp * aa * p + rpivot;
      start = pivot;
      stage = KILLED_BY_TS;
    }
    if (stage == KILLED_BY_TS) {
      int nextp;
      if (start == pivot) {
        const int tmp = lpivot + aa - 1 - lpivot % aa;
        nextp = tmp * p + rpivot;
        while (pivot < nextp && nextp >= gmt) nextp -= p;
      } else {
        nextp = start - p;
      }
      if (pivot < nextp) return nextp;
    }
    return gmt;
  }
};

}  // namespace

// ---------------------------------------------------------------------------- plans and validation
int Tree::geti(int k, int m) const {
  const int n = getnbgeqrf(k);
  for (int i = 0; i < n; ++i)
    if (getm(k, i) == m) return i;
  return -1;
}

void Tree::plan(int k, std::vector<int>& heads, std::vector<Kill>& kills) const {
  heads.clear();
  kills.clear();
  const int n = getnbgeqrf(k);
  for (int i = 0; i < n; ++i) heads.push_back(getm(k, i));
  // post-order walk of the elimination tree rooted at the diagonal row (bounded: a malformed tree cannot spin)
  std::vector<std::pair<int, int>> stack{{k, nextpiv(k, k, mt)}};
  long guard = 0;
  const long limit = 8L * (mt + 1) * (mt + 1) + 64;
  while (!stack.empty() && ++guard < limit) {
    const int piv = stack.back().first, nxt = stack.back().second;
    if (nxt == mt) {
      stack.pop_back();
      if (!stack.empty()) {
        const int parent = stack.back().first;
        kills.push_back(Kill{parent, piv, gettype(k, piv)});
        stack.back().second = nextpiv(k, parent, piv);
      }
      continue;
    }
    stack.push_back({nxt, nextpiv(k, nxt, mt)});
  }
}

int Tree::check(std::string& err) const {
  char buf[160];
  for (int k = 0; k < std::min(mt, nt); ++k) {
    std::vector<int> hv;
    std::vector<Kill> kv;
    plan(k, hv, kv);
    const std::set<int> heads(hv.begin(), hv.end());
    if (!heads.count(k)) {
      std::snprintf(buf, sizeof buf, "panel %d: diagonal row is not a GEQRT head", k);
      err = buf;
      return 1;
    }
    std::set<int> killed;
    for (const Kill& x : kv) {
      const int pv = x.piv, m = x.m, t = x.type;
      const char* why = nullptr;
      if (!(k <= pv && pv < mt && k < m && m < mt)) why = "bad pair";
      else if (killed.count(m) || killed.count(pv)) why = "row used after being killed";
      else if (t == KILLED_BY_TS && heads.count(m)) why = "TS kill of a GEQRT row";
      else if (t != KILLED_BY_TS && (!heads.count(m) || !heads.count(pv))) why = "TT kill between non-triangular rows";
      else if (t == KILLED_BY_TS && !heads.count(pv)) why = "TS annihilator is not triangular";
      else if (currpiv(k, m) != pv) why = "currpiv disagrees with the plan";
      if (why) {
        std::snprintf(buf, sizeof buf, "panel %d: %s (%d, %d)", k, why, pv, m);
        err = buf;
        return 1;
      }
      killed.insert(m);
    }
    for (int m = k + 1; m < mt; ++m) {
      if (!killed.count(m)) {
        std::snprintf(buf, sizeof buf, "panel %d: row %d survives", k, m);
        err = buf;
        return 1;
      }
      if (!heads.count(m) && gettype(k, m) != KILLED_BY_TS) {
        std::snprintf(buf, sizeof buf, "panel %d: row %d neither GEQRT'ed nor TS-killed", k, m);
        err = buf;
        return 1;
      }
    }
  }
  return 0;
}

std::string Tree::print_type() const {
  std::string s;
  char b[16];
  for (int m = 0; m < mt; ++m) {
    for (int k = 0; k < std::min(mt, nt); ++k) {
      if (k) s += ' ';
      if (m >= k) std::snprintf(b, sizeof b, "%2d", gettype(k, m));
      else std::snprintf(b, sizeof b, " .");
      s += b;
    }
    s += '\n';
  }
  return s;
}

std::string Tree::print_pivot() const {
  std::string s;
  char b[16];
  for (int m = 0; m < mt; ++m) {
    for (int k = 0; k < std::min(mt, nt); ++k) {
      if (k) s += ' ';
      if (m > k) std::snprintf(b, sizeof b, "%3d", currpiv(k, m));
      else std::snprintf(b, sizeof b, "  .");
      s += b;
    }
    s += '\n';
  }
  return s;
}

std::string Tree::print_nbgeqrt() const {
  std::string s;
  for (int k = 0; k < std::min(mt, nt); ++k) {
    if (k) s += ' ';
    s += std::to_string(getnbgeqrf(k));
  }
  return s + "\n";
}

std::string Tree::dot(int k0) const {
  std::string s = "digraph qrtree {\n";
  for (int k = 0; k < std::min(mt, nt); ++k) {
    if (k0 >= 0 && k != k0) continue;
    std::vector<int> hv;
    std::vector<Kill> kv;
    plan(k, hv, kv);
    for (const Kill& x : kv) {
      char b[128];
      std::snprintf(b, sizeof b, "  \"k%d_%d\" -> \"k%d_%d\" [style=%s,label=\"%d\"];\n", k, x.m, k, x.piv,
                    x.type ? "solid" : "dashed", x.type);
      s += b;
    }
  }
  return s + "}\n";
}

Tree* make_hqr(int mt, int nt, int llvl, int hlvl, int a, int p, int domino, int tsrr) {
  return new HqrTree(mt, nt, llvl, hlvl, a, p, domino, tsrr);
}
Tree* make_systolic(int mt, int nt, int p, int q) { return new SystolicTree(mt, nt, p, q); }
Tree* make_svd(int mt, int nt, int hlvl, int p, int nbcores_per_node, int ratio, int nodes) {
  return new SvdTree(mt, nt, hlvl, p, nbcores_per_node, ratio, nodes);
}

}  // namespace nq

// ---------------------------------------------------------------------------- the C handle (qr_param.h)
// A native descriptor's tree: q->args holds the nq::Tree and the query pointers below answer from it
// (dplasma_capi.cpp's qt_* functions route here when the descriptor has no framework object).
#include <initializer_list>

#include "native_internal.h"

namespace {
nq::Tree* tree_of(const dplasma_qrtree_t* q) { return (nq::Tree*)q->args; }
int q_getnbgeqrf(const dplasma_qrtree_t* q, int k) { return tree_of(q)->getnbgeqrf(k); }
int q_getm(const dplasma_qrtree_t* q, int k, int i) { return tree_of(q)->getm(k, i); }
int q_geti(const dplasma_qrtree_t* q, int k, int m) { return tree_of(q)->geti(k, m); }
int q_gettype(const dplasma_qrtree_t* q, int k, int m) { return tree_of(q)->gettype(k, m); }
int q_currpiv(const dplasma_qrtree_t* q, int k, int m) { return tree_of(q)->currpiv(k, m); }
int q_nextpiv(const dplasma_qrtree_t* q, int k, int p, int m) { return tree_of(q)->nextpiv(k, p, m); }
int q_prevpiv(const dplasma_qrtree_t* q, int k, int p, int m) { return tree_of(q)->prevpiv(k, p, m); }
}  // namespace

bool nat_qrtree_is(const dplasma_qrtree_t* q) { return q && q->args && q->getnbgeqrf == q_getnbgeqrf; }
nq::Tree* nat_qrtree(const dplasma_qrtree_t* q) { return nat_qrtree_is(q) ? tree_of(q) : nullptr; }

int nat_qrtree_init(dplasma_qrtree_t* q, const char* kind, int trans, dplasma_desc_t* dA, std::initializer_list<int> ints) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!q || !A) {
    dpl_set_error("qrtree init: a descriptor of a native or framework context");
    return -1;
  }
  const bool notrans = trans == NOTRANS;
  const int mt = notrans ? A->mt : A->nt, nt = notrans ? A->nt : A->mt;
  std::vector<int> v(ints);
  nq::Tree* t = nullptr;
  const std::string k = kind;
  if (k == "hqr") {   // llvl, hlvl, a, p, domino, tsrr; p <= 0: the grid rows (QR) / columns (LQ)
    const int a = v[2] == -1 ? -1 : std::max(v[2], 1);
    const int p = v[3] > 0 ? v[3] : (notrans ? A->P : A->Q);
    t = nq::make_hqr(mt, nt, v[0], v[1], a, p, v[4], v[5]);
  } else if (k == "systolic") {
    t = nq::make_systolic(mt, nt, v[0], v[1]);
  } else if (k == "svd") {   // hlvl, p, cores per node, ratio; nodes = the descriptor's ranks
    t = nq::make_svd(mt, nt, v[0], v[1], v[2], v[3], A->P * A->Q);
  }
  if (!t) {
    dpl_set_error("qrtree init: unknown tree kind");
    return -1;
  }
  q->args = t;
  q->getnbgeqrf = q_getnbgeqrf;
  q->getm = q_getm;
  q->geti = q_geti;
  q->gettype = q_gettype;
  q->currpiv = q_currpiv;
  q->nextpiv = q_nextpiv;
  q->prevpiv = q_prevpiv;
  q->mt = t->mt;
  q->nt = t->nt;
  q->a = t->a;
  q->p = t->p;
  return 0;
}

void nat_qrtree_fini(dplasma_qrtree_t* q) {
  if (!nat_qrtree_is(q)) return;
  delete tree_of(q);
  q->args = nullptr;
}

int nat_qrtree_check(const dplasma_qrtree_t* q) {
  std::string err;
  const int rc = tree_of(q)->check(err);
  if (rc) dpl_set_error(err.c_str());
  return rc;
}

void nat_qrtree_print(const dplasma_qrtree_t* q, const char* what, int k, int* perm, const char* file) {
  const nq::Tree* t = tree_of(q);
  const std::string w = what;
  std::string out;
  if (w == "dag") {
    FILE* f = std::fopen(file && *file ? file : "qrtree.dot", "w");
    if (f) {
      const std::string s = t->dot(-1);
      std::fwrite(s.data(), 1, s.size(), f);
      std::fclose(f);
    }
    return;
  }
  if (w == "type") out = t->print_type();
  else if (w == "pivot") out = t->print_pivot();
  else if (w == "nbgeqrt") out = t->print_nbgeqrt();
  else if (w == "perm") {   // the order rows are killed in at each step (perm[k * mt + i])
    for (int kk = 0; kk < std::min(t->mt, t->nt); ++kk) {
      std::vector<int> hv;
      std::vector<nq::Kill> kv;
      t->plan(kk, hv, kv);
      std::vector<int> order{kk};
      for (auto it = kv.rbegin(); it != kv.rend(); ++it) order.push_back(it->m);
      for (size_t i = 0; i < order.size(); ++i) {
        if (perm) perm[(size_t)kk * t->mt + i] = order[i];
        out += (i ? " " : "") + std::to_string(order[i]);
      }
      out += "\n";
    }
  } else if (w == "next_k" || w == "prev_k") {
    char b[16];
    for (int p = k; p < t->mt; ++p) {
      for (int m = k; m <= t->mt; ++m) {
        std::snprintf(b, sizeof b, "%s%3d", m > k ? " " : "", w == "next_k" ? t->nextpiv(k, p, m) : t->prevpiv(k, p, m));
        out += b;
      }
      out += "\n";
    }
  } else if (w == "geqrt_k") {
    std::vector<int> hv;
    std::vector<nq::Kill> kv;
    t->plan(k, hv, kv);
    for (size_t i = 0; i < hv.size(); ++i) out += (i ? " " : "") + std::to_string(hv[i]);
    out += "\n";
  }
  std::fputs(out.c_str(), stdout);
  std::fflush(stdout);
}

// test hooks (tests/test_qrtree_native.py drives the C++ trees against the reference-oracle digests)
extern "C" {
// kind 0: hqr (llvl, hlvl, a, p, domino, tsrr); 1: systolic (p, q); 2: svd (hlvl, p, cores, ratio, nodes)
DPL_CAPI void* dpl_nq_create(int kind, int mt, int nt, const int* v) {
  if (kind == 0) return nq::make_hqr(mt, nt, v[0], v[1], v[2], v[3], v[4], v[5]);
  if (kind == 1) return nq::make_systolic(mt, nt, v[0], v[1]);
  if (kind == 2) return nq::make_svd(mt, nt, v[0], v[1], v[2], v[3], v[4]);
  return nullptr;
}
// fn 0 getnbgeqrf(k) 1 getm(k, x) 2 gettype(k, x) 3 currpiv(k, x) 4 nextpiv(k, x, y) 5 prevpiv(k, x, y) 6 check
DPL_CAPI int dpl_nq_query(void* h, int fn, int k, int x, int y) {
  const nq::Tree* t = (const nq::Tree*)h;
  switch (fn) {
    case 0: return t->getnbgeqrf(k);
    case 1: return t->getm(k, x);
    case 2: return t->gettype(k, x);
    case 3: return t->currpiv(k, x);
    case 4: return t->nextpiv(k, x, y);
    case 5: return t->prevpiv(k, x, y);
    case 6: {
      std::string err;
      return t->check(err);
    }
    default: return -1;
  }
}
DPL_CAPI void dpl_nq_free(void* h) { delete (nq::Tree*)h; }
}
