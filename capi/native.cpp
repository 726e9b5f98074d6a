// Interpreter-free single-GPU engine behind the C ABI (dplasma_init_native).
//
// The default C ABI (dplasma_capi.cpp) embeds CPython and forwards every call to dplasma_amd.  A
// native context never starts the interpreter: descriptors are LAPACK-layout device buffers, the
// algorithms below are compiled into stream programs here in C++ and their tasks launch the HIP
// kernels of libdplasma_kernels.so directly (the same kernels, batch records and schedules as the
// Python builders: models/potrf.py, models/gemm.py, models/blas3.py, models/aux.py).
//
// Runtime: a program is a list of tasks, each bound to one of the context's two HIP streams
// ("panel", high priority: the critical path; "update", low priority: bulk trailing updates)
// with explicit dependencies on earlier tasks; running it enqueues every task in order and
// inserts a HIP event wait only for cross-stream edges (the PaRSEC dataflow of the reference's
// JDF taskpools -- src/zpotrf_L.jdf:93-188 -- as stream order + events, no host round trips).
// Batch records (GemmItemK / KPair / TileItem / RbItem) are built and uploaded once, when the
// program is built (dplasma_<p><op>_New), so a run only launches kernels.
//
// Scope: one process, one GPU; s/d/c/z potrf, potrs, posv, gemm, trsm (all 8 side/uplo/trans
// variants), herk / syrk, the element-wise maps (geadd, tradd, lacpy, laset, lascal), the norms lange /
// lantr, plghe, plgsy, plrnt.
// Every other entry point returns an error on a native context.
#include <complex>
#include <limits>
#include <thread>
#include <map>
#include <set>

#include "native_comm.h"
#include "native_internal.h"
#include "native_qrtree.h"
#include "../csrc/runtime/band_core.h"


namespace {

// ----------------------------------------------------------------------------- batches

// ----------------------------------------------------------------------------- POTRF
// models/potrf.py on one process: blocks of D panels; per panel POTRF(k) and its panel TRSM on the
// panel stream, NEAR(k) (the rest of the block) right after; per block NEXT (the next block's
// columns, K = D*nb) and REST (everything beyond) on the update stream; the next block's first
// POTRF follows NEXT.  fp64 tiles <= 512: dataflow tile kernel + register-resident panel TRSM
// sharing the inverted 32-blocks (potrf_rb.hip); other precisions: tile POTRF + batched TRSM.
bool add_potrf(NatProgram& P, int uplo, NatDesc& A) {
  const int prec = A.prec, nt = A.nt;
  const bool lower = uplo == LOWER;
  const int D = std::max(1, env_int("DPLASMA_POTRF_DEFER", 4));
  const int min_tiles = env_int("DPLASMA_POTRF_DEFER_MIN_TILES", 24);
  const bool rb = prec == P_D && A.mb == A.nb && A.mb <= 512;
  const int zsz = rb ? dpl_potrf_zbuf_size() : 0;
  DevPtr zb;
  if (rb) {
    zb = dev_alloc((size_t)2 * zsz * sizeof(double), false);
    if (!zb) return false;
    P.keep.push_back(zb);
  }
  auto tc = [&](int i, int k) { return lower ? std::make_pair(i, k) : std::make_pair(k, i); };
  const int tri_mask = lower ? 1 : 2;
  const int tA = lower ? NOTRANS : CONJTRANS, tB = lower ? CONJTRANS : NOTRANS;
  const Scalar m_one(prec, -1.0), one(prec, 1.0);
  char* base = A.data;
  const int ld = A.lld, mbA = A.mb;
  int* info = (int*)P.info->p;

  auto update = [&](const std::vector<int>& ks, int n0, int n1) {
    auto g = std::make_shared<Gemm>();
    for (int n_ = n0; n_ < n1; ++n_)
      for (int m_ = n_; m_ < nt; ++m_) {
        const auto cc = lower ? std::make_pair(m_, n_) : std::make_pair(n_, m_);
        std::vector<KPair> kp;
        for (int k : ks) {
          const auto a = tc(cc.first, k), b = tc(cc.second, k);
          kp.push_back(KPair{A.off(a.first, a.second), A.off(b.first, b.second), A.rows(k), 0});
        }
        g->add(A.off(cc.first, cc.second), A.rows(cc.first), A.cols(cc.second), kp, m_ == n_ ? tri_mask : 0);
      }
    return g;
  };
  auto gemm_task = [&](std::shared_ptr<Gemm> g) {
    return [=](hipStream_t s) { return g->launch(prec, tA, tB, m_one, base, ld, base, ld, one, base, ld, s); };
  };

  std::vector<std::pair<int, int>> blocks;
  for (int c = 0; c < nt;) {
    const int d = nt - c >= min_tiles ? D : 1;
    blocks.emplace_back(c, std::min(nt, c + d));
    c += d;
  }
  int gate = -1, last_upd = -1;
  for (size_t b = 0; b < blocks.size(); ++b) {
    const int c0 = blocks[b].first, c1 = blocks[b].second;
    for (int k = c0; k < c1; ++k) {
      const int kb = A.rows(k);
      const long long dk = A.off(k, k);
      double* zk = rb ? (double*)zb->p + (size_t)(k % 2) * zsz : nullptr;
      int t_potrf;
      if (rb) {
        t_potrf = P.task(0, [=](hipStream_t s) {
          return dpl_potrf_tile_rbz(uplo, kb, (double*)base + dk, ld, info, k * mbA, zk, s);
        }, {gate});
      } else {
        // other precisions: nb-wide sub-steps (tile POTRF, batched TRSM, masked MFMA GEMM) as
        // ops.potrf_tile_blocked -- a single workgroup on a whole complex 512 tile is ~10 ms
        const int sb = 128;
        auto at = [&](int i, int j) { return dk + (lower ? (long long)i + (long long)j * ld : (long long)j + (long long)i * ld); };
        int prev = gate;
        for (int j0 = 0; j0 < kb; j0 += sb) {
          const int jb = std::min(sb, kb - j0);
          const long long dj = at(j0, j0);
          prev = P.task(0, [=](hipStream_t s) {
            return dpl_potrf_tile(prec, uplo, jb, base, dj, ld, info, k * mbA + j0, s);
          }, {prev});
          if (j0 + jb >= kb) break;
          auto tr = std::make_shared<Trsm1>();
          tr->tri = dj;
          auto g = std::make_shared<Gemm>();
          for (int i0 = j0 + jb; i0 < kb; i0 += sb) {
            const int ib = std::min(sb, kb - i0);
            if (lower) tr->add(at(i0, j0), ib, jb);
            else tr->add(at(i0, j0), jb, ib);
          }
          for (int c0_ = j0 + jb; c0_ < kb; c0_ += sb) {
            const int cbw = std::min(sb, kb - c0_);
            for (int r0 = c0_; r0 < kb; r0 += sb) {
              const int rbw = std::min(sb, kb - r0);
              const int mask = r0 == c0_ ? tri_mask : 0;
              if (lower)   // C(r, c) -= L(r, j) L(c, j)^H
                g->add(at(r0, c0_), rbw, cbw, {KPair{at(r0, j0), at(c0_, j0), jb, 0}}, mask);
              else         // C(c, r) -= U(j, c)^H U(j, r)
                g->add(at(r0, c0_), cbw, rbw, {KPair{at(c0_, j0), at(r0, j0), jb, 0}}, mask);
            }
          }
          const int side = lower ? RIGHT : LEFT;
          if (!tr->upload(P, prec, side) || !g->upload(P)) return false;
          prev = P.task(0, [=](hipStream_t s) {
            return tr->launch(prec, side, uplo, CONJTRANS, NONUNIT, one, base, ld, base, ld, s);
          }, {prev});
          prev = P.task(0, gemm_task(g), {prev});
        }
        t_potrf = prev;
      }
      int t_trsm = t_potrf;
      if (k + 1 < nt) {
        if (rb) {
          std::vector<RbItem> strips;
          for (int i = k + 1; i < nt; ++i) {
            const auto cc = tc(i, k);
            const int ext = lower ? A.rows(i) : A.cols(i);
            for (int r0 = 0; r0 < ext; r0 += 16)
              strips.push_back(RbItem{A.off(cc.first, cc.second) + (lower ? r0 : (long long)r0 * ld),
                                      std::min(16, ext - r0), 0});
          }
          DevPtr d = dev_upload(strips);
          if (!d) return false;
          P.keep.push_back(d);
          const int nrb = (int)strips.size();
          t_trsm = P.task(0, [=](hipStream_t s) {
            return dpl_trsm_rb(uplo, kb, (double*)base + dk, ld, zk, nrb, d->p, (double*)base, ld, s);
          }, {t_potrf, gate});
        } else {
          auto tr = std::make_shared<Trsm1>();
          tr->tri = dk;
          for (int i = k + 1; i < nt; ++i) {
            const auto cc = tc(i, k);
            tr->add(A.off(cc.first, cc.second), A.rows(cc.first), A.cols(cc.second));
          }
          const int side = lower ? RIGHT : LEFT;
          if (!tr->upload(P, prec, side)) return false;
          t_trsm = P.task(0, [=](hipStream_t s) {
            return tr->launch(prec, side, uplo, CONJTRANS, NONUNIT, one, base, ld, base, ld, s);
          }, {t_potrf, gate});
        }
      }
      if (k == nt - 1) break;
      auto near = update({k}, k + 1, c1);
      if (!near->empty()) {
        if (!near->upload(P)) return false;
        gate = P.task(0, gemm_task(near), {t_trsm, gate});
      } else {
        gate = t_trsm;
      }
    }
    if (c1 >= nt) break;
    std::vector<int> ks;
    for (int k = c0; k < c1; ++k) ks.push_back(k);
    const int n0 = blocks[b + 1].first, n1 = blocks[b + 1].second;
    auto nxt = update(ks, n0, n1), rest = update(ks, n1, nt);
    int t_next = -1;
    if (!nxt->empty()) {
      if (!nxt->upload(P)) return false;
      t_next = P.task(1, gemm_task(nxt), {gate, last_upd});
      last_upd = t_next;
    }
    if (!rest->empty()) {
      if (!rest->upload(P)) return false;
      last_upd = P.task(1, gemm_task(rest), {gate, last_upd});
    }
    if (t_next >= 0) gate = t_next;
  }
  return true;
}

// ----------------------------------------------------------------------------- TRSM
// op(A) X = alpha B (left) / X op(A) = alpha B (right), tile by tile (models/blas3.py): solve one
// block row (left) / column (right) of B against the diagonal tile, then update the blocks still
// to be solved with one GEMM launch (beta = alpha on the first step, 1 afterwards).
bool add_trsm(NatProgram& P, int side, int uplo, int trans, int diag, const Scalar& alpha, NatDesc& A, NatDesc& B,
              int stream, int first_dep = -1) {
  const int prec = B.prec;
  const bool left = side == LEFT, notrans = trans == NOTRANS;
  const int nk = left ? B.mt : B.nt;
  // effective lower (forward) for left: lower & notrans or upper & trans; right is the mirror
  const bool forward = left ? ((uplo == LOWER) == notrans) : ((uplo == UPPER) == notrans);
  std::vector<int> order;
  for (int i = 0; i < nk; ++i) order.push_back(forward ? i : nk - 1 - i);
  const Scalar one(prec, 1.0), m_one(prec, -1.0);
  char* a = A.data;
  char* bb = B.data;
  const int lda = A.lld, ldb = B.lld;
  int prev = first_dep;   // the first solve follows this task (e.g. the factorisation's last one)
  for (int s = 0; s < nk; ++s) {
    const int k = order[s];
    const Scalar ak = s == 0 ? alpha : one;
    auto tr = std::make_shared<Trsm1>();
    tr->tri = A.off(k, k);
    if (left)
      for (int n = 0; n < B.nt; ++n) tr->add(B.off(k, n), B.rows(k), B.cols(n));
    else
      for (int m = 0; m < B.mt; ++m) tr->add(B.off(m, k), B.rows(m), B.cols(k));
    if (!tr->upload(P, prec, side)) return false;
    prev = P.task(stream, [=](hipStream_t st) {
      return tr->launch(prec, side, uplo, trans, diag, ak, a, lda, bb, ldb, st);
    }, {prev});
    if (s + 1 == nk) break;
    auto g = std::make_shared<Gemm>();
    for (int r = s + 1; r < nk; ++r) {
      const int i = order[r];
      if (left) {   // B(i, n) = ak B(i, n) - op(A)(i, k) X(k, n)
        const long long ao = notrans ? A.off(i, k) : A.off(k, i);
        for (int n = 0; n < B.nt; ++n)
          g->add(B.off(i, n), B.rows(i), B.cols(n), {KPair{ao, B.off(k, n), B.rows(k), 0}}, 0);
      } else {      // B(m, i) = ak B(m, i) - X(m, k) op(A)(k, i)
        const long long ao = notrans ? A.off(k, i) : A.off(i, k);
        for (int m = 0; m < B.mt; ++m)
          g->add(B.off(m, i), B.rows(m), B.cols(i), {KPair{B.off(m, k), ao, B.cols(k), 0}}, 0);
      }
    }
    if (!g->upload(P)) return false;
    if (left)
      prev = P.task(stream, [=](hipStream_t st) {
        return g->launch(prec, notrans ? NOTRANS : trans, NOTRANS, m_one, a, lda, bb, ldb, ak, bb, ldb, st);
      }, {prev});
    else
      prev = P.task(stream, [=](hipStream_t st) {
        return g->launch(prec, NOTRANS, notrans ? NOTRANS : trans, m_one, bb, ldb, a, lda, ak, bb, ldb, st);
      }, {prev});
  }
  return true;
}

// first_dep: the task the solves must follow (posv: the factorisation's last panel-stream task; the
// solves run on the update stream, so stream order covers the factorisation's update-stream tasks)
bool add_potrs(NatProgram& P, int uplo, NatDesc& A, NatDesc& B, int first_dep = -1) {
  const Scalar one(B.prec, 1.0);
  if (uplo == LOWER)
    return add_trsm(P, LEFT, LOWER, NOTRANS, NONUNIT, one, A, B, 1, first_dep) &&
           add_trsm(P, LEFT, LOWER, CONJTRANS, NONUNIT, one, A, B, 1);
  return add_trsm(P, LEFT, UPPER, CONJTRANS, NONUNIT, one, A, B, 1, first_dep) &&
         add_trsm(P, LEFT, UPPER, NOTRANS, NONUNIT, one, A, B, 1);
}

// the grid version: two distributed solves appended after everything already in the program
bool add_potrs_dist(NatProgram& P, int uplo, NatDesc& A, NatDesc& B) {
  const Scalar one(B.prec, 1.0);
  if (uplo == LOWER)
    return nat_dist_trsm_into(P, LEFT, LOWER, NOTRANS, NONUNIT, one, A, B) &&
           nat_dist_trsm_into(P, LEFT, LOWER, CONJTRANS, NONUNIT, one, A, B);
  return nat_dist_trsm_into(P, LEFT, UPPER, CONJTRANS, NONUNIT, one, A, B) &&
         nat_dist_trsm_into(P, LEFT, UPPER, NOTRANS, NONUNIT, one, A, B);
}

// last task of a program on a stream (-1: none)
int last_on(const NatProgram& P, int stream) {
  for (int i = (int)P.tasks.size() - 1; i >= 0; --i)
    if (P.tasks[i].stream == stream) return i;
  return -1;
}

// descriptors of context c and precision prec; same_ctx also refuses multi-process contexts (the
// operations without a distributed builder), same_ctx_dist accepts them
bool same_ctx_dist(NatCtx* c, std::initializer_list<const NatDesc*> ds, int prec) {
  for (const NatDesc* d : ds)
    if (!d || d->ctx != c || d->prec != prec) return false;
  return true;
}
bool same_ctx(NatCtx* c, std::initializer_list<const NatDesc*> ds, int prec) {
  if (c && c->dist()) {
    nat_dist_refused = true;
    return false;
  }
  return same_ctx_dist(c, ds, prec);
}

}  // namespace

// ----------------------------------------------------------------------------- builders (capi_bridge.h)
NatProgram* nat_potrf(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return fail(nullptr, "potrf: descriptor of another context or precision");
  if (A->m != A->n || A->mb != A->nb || (uplo != LOWER && uplo != UPPER))
    return fail(nullptr, "potrf: square matrix with square tiles and uplo Lower/Upper required");
  if (c->dist()) return nat_dist_potrf(c, uplo, *A);
  NatProgram* P = new_program(c, "potrf", true);
  if (!P->info || !add_potrf(*P, uplo, *A)) return fail(P, "potrf: device allocation failed");
  return P;
}

NatProgram* nat_potrs(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec) || A->m != A->n || B->m != A->n || B->mb != A->nb)
    return fail(nullptr, "potrs: descriptors do not conform");
  NatProgram* P = new_program(c, "potrs", false);
  if (!(c->dist() ? add_potrs_dist(*P, uplo, *A, *B) : add_potrs(*P, uplo, *A, *B)))
    return fail(P, "potrs: device allocation failed");
  return P;
}

NatProgram* nat_posv(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatProgram* P = nat_potrf(ctx, prec, uplo, dA);
  if (!P) return nullptr;
  NatDesc *A = dA->nat, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {B}, prec) || B->m != A->n || B->mb != A->nb)
    return fail(P, "posv: right-hand side does not conform");
  P->gate = (int)P->tasks.size();   // B is left unchanged when A is not positive definite
  if (ctx->nat->dist())   // the solves follow the whole factorisation (every stream)
    return add_potrs_dist(*P, uplo, *A, *B) ? P : fail(P, "posv: device allocation failed");
  // the solves (update stream) start after the factorisation's last panel-stream task (POTRF / TRSM /
  // NEAR of the last tiles): without this edge they could read A(nt-1, nt-1) before it is factored
  if (!add_potrs(*P, uplo, *A, *B, last_on(*P, 0))) return fail(P, "posv: device allocation failed");
  return P;
}

// A := alpha x y^T + A (geru) or alpha x y^H + A (gerc): X is M x 1, Y is N x 1 -- a K = 1 GEMM on the same
// engine (reference: dplasma_zgeru / zgerc, src/zger.jdf); one process or a grid
NatProgram* nat_ger(dplasma_context_t* ctx, int prec, int conj, const void* alpha, dplasma_desc_t* dX,
                    dplasma_desc_t* dY, dplasma_desc_t* dA) {
  double one[2] = {1.0, 0.0};
  float onef[2] = {1.0f, 0.0f};
  const void* beta = (prec == P_D || prec == P_Z) ? (const void*)one : (const void*)onef;
  const bool cplx = prec == P_C || prec == P_Z;
  return nat_gemm(ctx, prec, NOTRANS, (conj && cplx) ? CONJTRANS : TRANS, alpha, dX, dY, beta, dA);
}

NatProgram* nat_gemm(dplasma_context_t* ctx, int prec, int tA, int tB, const void* alpha, dplasma_desc_t* dA,
                     dplasma_desc_t* dB, const void* beta, dplasma_desc_t* dC) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx_dist(c, {A, B, C}, prec)) return fail(nullptr, "gemm: descriptors of another context or precision");
  const int am = tA == NOTRANS ? A->m : A->n, ak = tA == NOTRANS ? A->n : A->m;
  const int bk = tB == NOTRANS ? B->m : B->n, bn = tB == NOTRANS ? B->n : B->m;
  const int akb = tA == NOTRANS ? A->nb : A->mb, bkb = tB == NOTRANS ? B->mb : B->nb;
  if (am != C->m || bn != C->n || ak != bk || akb != bkb || (tA == NOTRANS ? A->mb : A->nb) != C->mb ||
      (tB == NOTRANS ? B->nb : B->mb) != C->nb)
    return fail(nullptr, "gemm: operands do not conform");
  if (c->dist()) return nat_dist_gemm(c, prec, tA, tB, Scalar(prec, alpha), *A, *B, Scalar(prec, beta), *C);
  NatProgram* P = new_program(c, "gemm", false);
  auto g = std::make_shared<Gemm>();
  const int kt = (ak + akb - 1) / akb;
  for (int n = 0; n < C->nt; ++n)
    for (int m = 0; m < C->mt; ++m) {
      std::vector<KPair> kp;
      for (int k = 0; k < kt; ++k) {
        const long long ao = tA == NOTRANS ? A->off(m, k) : A->off(k, m);
        const long long bo = tB == NOTRANS ? B->off(k, n) : B->off(n, k);
        kp.push_back(KPair{ao, bo, tA == NOTRANS ? A->cols(k) : A->rows(k), 0});
      }
      g->add(C->off(m, n), C->rows(m), C->cols(n), kp, 0);
    }
  if (!g->upload(*P)) return fail(P, "gemm: device allocation failed");
  const Scalar al(prec, alpha), be(prec, beta);
  char *a = A->data, *b = B->data, *cc = C->data;
  const int lda = A->lld, ldb = B->lld, ldc = C->lld;
  P->task(1, [=](hipStream_t s) { return g->launch(prec, tA, tB, al, a, lda, b, ldb, be, cc, ldc, s); }, {});
  return P;
}

NatProgram* nat_trsm(dplasma_context_t* ctx, int prec, int side, int uplo, int trans, int diag, const void* alpha,
                     dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec)) return fail(nullptr, "trsm: descriptors of another context or precision");
  const int order = side == LEFT ? B->m : B->n;
  if (A->m != A->n || A->m != order || A->mb != A->nb || (side == LEFT ? B->mb : B->nb) != A->nb)
    return fail(nullptr, "trsm: operands do not conform");
  NatProgram* P = new_program(c, "trsm", false);
  if (c->dist())
    return nat_dist_trsm_into(*P, side, uplo, trans, diag, Scalar(prec, alpha), *A, *B)
               ? P : fail(P, "trsm: device allocation failed");
  if (!add_trsm(*P, side, uplo, trans, diag, Scalar(prec, alpha), *A, *B, 1))
    return fail(P, "trsm: device allocation failed");
  return P;
}

// ----------------------------------------------------------------------------- HERK / SYRK
// C = alpha op(A) op(A)^{H|T} + beta C on the uplo triangle (models/blas3.py): one launch of the MFMA
// GEMM engine over every tile of the triangle, k-runs over A's tile columns (rows for trans), the
// diagonal tiles masked to their triangle.
// C = alpha op(A) op(B)^{H|T} on C's uplo triangle tiles (beta on the first pass); rank-2k adds the
// swapped product in a second launch.  Tasks on stream 1 after `prev`; returns the last task (-2: failure).
static int add_rank_k(NatProgram& Pr, int prec, int uplo, int trans, const Scalar& alpha, const NatDesc* A,
                      const NatDesc* B, const Scalar& beta, NatDesc* C, bool herm, int prev, bool fixdiag = true) {
  NatProgram* P = &Pr;
  const bool nt = trans == NOTRANS;
  const int ak = nt ? A->n : A->m, akb = nt ? A->nb : A->mb;
  const int ct = herm ? CONJTRANS : TRANS;
  if (C->ctx->dist()) {   // the SUMMA GEMM over the grid, restricted to C's triangle
    if (!nat_dist_gemm_into(Pr, prec, nt ? NOTRANS : ct, nt ? ct : NOTRANS, alpha, *const_cast<NatDesc*>(A),
                            *const_cast<NatDesc*>(B), beta, *C, uplo))
      return -2;
    prev = (int)Pr.tasks.size() - 1;
  }
  auto g = std::make_shared<Gemm>();
  const int kt = (ak + akb - 1) / akb;
  for (int n = 0; n < C->nt; ++n)
    for (int m = 0; m < C->mt; ++m) {
      if ((uplo == LOWER && m < n) || (uplo == UPPER && m > n)) continue;
      std::vector<KPair> kp;
      for (int k = 0; k < kt; ++k)   // C(m,n) += op(A)(m,k) op(B)(n,k)^H
        kp.push_back(KPair{nt ? A->off(m, k) : A->off(k, m), nt ? B->off(n, k) : B->off(k, n),
                           nt ? A->cols(k) : A->rows(k), 0});
      g->add(C->off(m, n), C->rows(m), C->cols(n), kp, m == n ? (uplo == LOWER ? 1 : 2) : 0);
    }
  char *a = A->data, *b = B->data, *cc = C->data;
  const int lda = A->lld, ldb = B->lld, ldc = C->lld;
  const int ta = nt ? NOTRANS : ct, tb = nt ? ct : NOTRANS;
  int t = prev;
  if (!C->ctx->dist()) {
    if (!g->upload(*P)) return -2;
    t = P->task(1, [=](hipStream_t s) { return g->launch(prec, ta, tb, alpha, a, lda, b, ldb, beta, cc, ldc, s); },
                {prev});
  }
  int last = t;
  if (herm && fixdiag) {
    // Hermitian rank-k (zherk): C's diagonal is real.  diag := (diag + conj(diag)) / 2 on the
    // diagonal tiles (geadd, diagonal part, conjugate transpose of the tile onto itself)
    std::vector<TileItem> d;
    int mm = 0;
    for (int k = 0; k < C->mt && k < C->nt; ++k) {
      if (!C->local(k, k)) continue;
      d.push_back(TileItem{C->off(k, k), C->off(k, k), C->rows(k), C->cols(k), k * C->mb, k * C->nb});
      mm = std::max(mm, std::max(C->rows(k), C->cols(k)));
    }
    if (d.empty()) return last;
    DevPtr dd = dev_upload(d);
    if (!dd) return -2;
    P->keep.push_back(dd);
    const Scalar half(prec, 0.5);
    const int n = (int)d.size();
    last = P->task(1, [=](hipStream_t s) {
      return dpl_geadd(prec, 5, CONJTRANS, n, dd->p, mm, mm, half.ptr(), cc, ldc, half.ptr(), cc, ldc, 0, s);
    }, {t});
  }
  return last;
}

static NatProgram* rank_k(dplasma_context_t* ctx, int prec, int uplo, int trans, const Scalar& alpha,
                          dplasma_desc_t* dA, const Scalar& beta, dplasma_desc_t* dC, bool herm, const char* name) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx_dist(c, {A, C}, prec)) return fail(nullptr, std::string(name) + ": descriptors of another context");
  const bool nt = trans == NOTRANS;
  const int an = nt ? A->m : A->n;
  if ((uplo != LOWER && uplo != UPPER) || C->m != C->n || an != C->m || C->mb != C->nb ||
      (nt ? A->mb : A->nb) != C->mb)
    return fail(nullptr, std::string(name) + ": operands do not conform");
  NatProgram* P = new_program(c, name, false);
  if (add_rank_k(*P, prec, uplo, trans, alpha, A, A, beta, C, herm, -1) == -2)
    return fail(P, std::string(name) + ": device allocation failed");
  return P;
}

// C = alpha op(A) op(B)^H + conj(alpha) op(B) op(A)^H + beta C (her2k; syr2k: alpha both times, ^T):
// two launches of the GEMM engine on the triangle, the second accumulating (src/zher2k_*.jdf)
static NatProgram* rank_2k(dplasma_context_t* ctx, int prec, int uplo, int trans, const Scalar& alpha,
                           const Scalar& alpha2, dplasma_desc_t* dA, dplasma_desc_t* dB, const Scalar& beta,
                           dplasma_desc_t* dC, bool herm, const char* name) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx_dist(c, {A, B, C}, prec)) return fail(nullptr, std::string(name) + ": descriptors of another context");
  const bool nt = trans == NOTRANS;
  if ((uplo != LOWER && uplo != UPPER) || C->m != C->n || (nt ? A->m : A->n) != C->m || A->m != B->m ||
      A->n != B->n || A->mb != B->mb || A->nb != B->nb || C->mb != C->nb || (nt ? A->mb : A->nb) != C->mb)
    return fail(nullptr, std::string(name) + ": operands do not conform");
  NatProgram* P = new_program(c, name, false);
  const Scalar one(prec, 1.0);
  // both passes use the adjoint for her2k (op(B)^H, op(A)^H); the real diagonal is restored after the second
  int t = add_rank_k(*P, prec, uplo, trans, alpha, A, B, beta, C, herm, -1, false);
  if (t != -2) t = add_rank_k(*P, prec, uplo, trans, alpha2, B, A, one, C, herm, t, true);
  if (t == -2) return fail(P, std::string(name) + ": device allocation failed");
  return P;
}

NatProgram* nat_herk(dplasma_context_t* ctx, int prec, int uplo, int trans, double alpha, dplasma_desc_t* A,
                     double beta, dplasma_desc_t* C) {
  if (prec != P_C && prec != P_Z) return fail(nullptr, "herk: complex precisions only");
  return rank_k(ctx, prec, uplo, trans, Scalar(prec, alpha), A, Scalar(prec, beta), C, true, "herk");
}

NatProgram* nat_syrk(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                     const void* beta, dplasma_desc_t* C) {
  return rank_k(ctx, prec, uplo, trans, Scalar(prec, alpha), A, Scalar(prec, beta), C, false, "syrk");
}

NatProgram* nat_her2k(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      dplasma_desc_t* B, double beta, dplasma_desc_t* C) {
  if (prec != P_C && prec != P_Z) return fail(nullptr, "her2k: complex precisions only");
  double a[2] = {0.0, 0.0};
  if (prec == P_C) {
    float f[2];
    std::memcpy(f, alpha, sizeof(f));
    a[0] = f[0];
    a[1] = f[1];
  } else {
    std::memcpy(a, alpha, sizeof(a));
  }
  return rank_2k(ctx, prec, uplo, trans, Scalar(prec, a[0], a[1]), Scalar(prec, a[0], -a[1]), A, B,
                 Scalar(prec, beta), C, true, "her2k");
}

NatProgram* nat_syr2k(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      dplasma_desc_t* B, const void* beta, dplasma_desc_t* C) {
  return rank_2k(ctx, prec, uplo, trans, Scalar(prec, alpha), Scalar(prec, alpha), A, B, Scalar(prec, beta), C, false,
                 "syr2k");
}

// ----------------------------------------------------------------------------- element-wise maps
// geadd / tradd / lacpy / laset / lascal (models/aux.py): one grid-stride launch over the tiles that
// meet the uplo part; the kernels mask by GLOBAL element coordinates (TileItem gi / gj), so a diagonal
// tile is cut at the matrix diagonal exactly as the reference's map2 LOWER / UPPER tasks do.
static int part_of(int uplo) { return uplo == LOWER ? 1 : uplo == UPPER ? 2 : 0; }



namespace {
std::shared_ptr<NatDesc> work_desc(NatProgram& P, const NatDesc& A);
}

static NatProgram* map_add(dplasma_context_t* ctx, int prec, int uplo, int trans, const Scalar& alpha,
                           dplasma_desc_t* dA, const Scalar& beta, dplasma_desc_t* dB, int copy, const char* name) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec)) return fail(nullptr, std::string(name) + ": descriptors of another context");
  const bool nt = trans == NOTRANS;
  if ((nt ? A->m : A->n) != B->m || (nt ? A->n : A->m) != B->n || (nt ? A->mb : A->nb) != B->mb ||
      (nt ? A->nb : A->mb) != B->nb)
    return fail(nullptr, std::string(name) + ": operands do not conform");
  NatProgram* P = new_program(c, name, false);
  int trans_eff = trans;
  const NatDesc* src = A;
  int first = -1;
  if (c->dist() && !nt) {   // the grid: op(A) is first transposed tile by tile into B's distribution
    auto W = work_desc(*P, *B);
    if (!W || !nat_dist_mirror_into(*P, *A, UPPERLOWER, trans, *W))
      return fail(P, std::string(name) + ": device allocation failed");
    src = W.get();
    trans_eff = NOTRANS;
    first = (int)P->tasks.size() - 1;
  }
  auto mb = std::make_shared<MapBatch>();
  mb->build(*B, uplo, src, trans_eff);
  if (!mb->upload(*P)) return fail(P, std::string(name) + ": device allocation failed");
  const int part = part_of(uplo), lda = src->lld, ldb = B->lld;
  const char* a = src->data;
  char* b = B->data;
  P->task(1, [=](hipStream_t s) {
    if (mb->n() == 0) return 0;
    return dpl_geadd(prec, part, trans_eff, mb->n(), mb->items(), mb->mm, mb->nn, alpha.ptr(), a, lda, beta.ptr(), b,
                     ldb, copy, s);
  }, {first, last_on(*P, 0), last_on(*P, 2)});
  return P;
}

NatProgram* nat_geadd(dplasma_context_t* ctx, int prec, int trans, const void* alpha, dplasma_desc_t* A,
                      const void* beta, dplasma_desc_t* B) {
  return map_add(ctx, prec, UPPERLOWER, trans, Scalar(prec, alpha), A, Scalar(prec, beta), B, 0, "geadd");
}

NatProgram* nat_tradd(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      const void* beta, dplasma_desc_t* B) {
  return map_add(ctx, prec, uplo, trans, Scalar(prec, alpha), A, Scalar(prec, beta), B, 0, "tradd");
}

NatProgram* nat_lacpy(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A, dplasma_desc_t* B) {
  return map_add(ctx, prec, uplo, NOTRANS, Scalar(prec, 1.0), A, Scalar(prec, 0.0), B, 1, "lacpy");
}

NatProgram* nat_laset(dplasma_context_t* ctx, int prec, int uplo, const void* alpha, const void* beta,
                      dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return fail(nullptr, "laset: descriptor of another context");
  NatProgram* P = new_program(c, "laset", false);
  auto mb = std::make_shared<MapBatch>();
  mb->build(*A, uplo, nullptr, NOTRANS);
  if (!mb->upload(*P)) return fail(P, "laset: device allocation failed");
  const Scalar al(prec, alpha), be(prec, beta);
  const int part = part_of(uplo), lda = A->lld;
  char* a = A->data;
  P->task(1, [=](hipStream_t s) {
    if (mb->n() == 0) return 0;
    return dpl_laset(prec, part, mb->n(), mb->items(), mb->mm, mb->nn, al.ptr(), be.ptr(), a, lda, s);
  }, {});
  return P;
}

// A := alpha A on this rank's tiles of the uplo part, appended to P after everything already in it
// (also the beta scaling of a grid GEMM with an empty k range, native_dist.cpp)
bool nat_add_lascal(NatProgram& P, int uplo, const Scalar& al, NatDesc& A) {
  auto mb = std::make_shared<MapBatch>();
  mb->build(A, uplo, nullptr, NOTRANS);
  if (!mb->upload(P)) return false;
  const int prec = A.prec, part = part_of(uplo), lda = A.lld;
  char* a = A.data;
  int deps[NAT_NSTREAM];
  for (int q = 0; q < NAT_NSTREAM; ++q) deps[q] = last_on(P, q);
  P.task(1, [=](hipStream_t s) {
    if (mb->n() == 0) return 0;
    return dpl_lascal(prec, part, mb->n(), mb->items(), mb->mm, mb->nn, al.ptr(), a, lda, s);
  }, {deps[0], deps[1], deps[2]});
  return true;
}

NatProgram* nat_lascal(dplasma_context_t* ctx, int prec, int uplo, const void* alpha, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return fail(nullptr, "lascal: descriptor of another context");
  NatProgram* P = new_program(c, "lascal", false);
  if (!nat_add_lascal(*P, uplo, Scalar(prec, alpha), *A)) return fail(P, "lascal: device allocation failed");
  return P;
}

// ----------------------------------------------------------------------------- norms
// lange / lantr (models/aux.py): one dpl_tile_norm launch gives per-tile partials (max, column sums,
// row sums or a scaled sum of squares), combined on the host -- the reference's STEP1..STEP4 reduction
// of zlange_*_cyclic.jdf on one process.
enum { NORM_ONE = 171, NORM_FRB = 174, NORM_INF = 175, NORM_MAX = 177, UNIT = 132 };

static double norm_tiles(NatDesc& A, int ntype, int uplo, bool unit, hipStream_t st, bool& ok) {
  ok = false;
  const int kind = ntype == NORM_MAX ? 0 : ntype == NORM_ONE ? 1 : ntype == NORM_INF ? 2 : ntype == NORM_FRB ? 3 : -1;
  if (kind < 0) return 0.0;
  std::vector<TileItem> it;
  std::vector<std::pair<int, int>> mn;
  int mm = 0, nn = 0;
  for (int n = 0; n < A.nt; ++n)
    for (int m = 0; m < A.mt; ++m) {
      if ((uplo == LOWER && m < n) || (uplo == UPPER && m > n)) continue;
      if (!A.local(m, n)) continue;   // a multi-process context: partials of this rank's tiles, combined below
      it.push_back(TileItem{A.off(m, n), 0, A.rows(m), A.cols(n), m * A.mb, n * A.nb});
      mn.emplace_back(m, n);
      mm = std::max(mm, A.rows(m));
      nn = std::max(nn, A.cols(n));
    }
  const int os = kind == 0 ? 1 : kind == 1 ? nn : kind == 2 ? mm : 2;
  std::vector<double> h(it.size() * os);
  // the norm reads A after everything already queued on the context (every stream)
  if (hipDeviceSynchronize() != hipSuccess) return 0.0;
  if (!it.empty()) {
    DevPtr d = dev_upload(it), out = dev_alloc(sizeof(double) * it.size() * os, true);
    if (!d || !out) return 0.0;
    if (dpl_tile_norm(A.prec, kind, part_of(uplo), unit ? 1 : 0, (int)it.size(), d->p, A.data, A.lld,
                      (double*)out->p, os, st) != 0)
      return 0.0;
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), out->p, sizeof(double) * h.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return 0.0;
  }
  NatComm* comm = A.ctx->comm;
  double r = 0.0;
  if (kind == 0) {
    for (double v : h) r = std::max(r, v);
    if (comm && comm->allreduce(&r, 1, true) != 0) return 0.0;
  } else if (kind == 3) {   // (scale, ssq) per tile -> sqrt(sum scale^2 ssq), rescaled by the largest scale
    double big = 0.0;
    for (size_t t = 0; t < it.size(); ++t) big = std::max(big, h[2 * t]);
    if (comm && comm->allreduce(&big, 1, true) != 0) return 0.0;
    double q2 = 0.0;
    if (big > 0)
      for (size_t t = 0; t < it.size(); ++t) {
        const double q = h[2 * t] / big;
        q2 += q * q * h[2 * t + 1];
      }
    if (comm && comm->allreduce(&q2, 1, false) != 0) return 0.0;
    r = big > 0 ? big * std::sqrt(q2) : 0.0;
  } else {                  // column (one) / row (inf) sums over the tiles of a tile column / row
    std::vector<double> acc(kind == 1 ? A.n : A.m, 0.0);
    for (size_t t = 0; t < it.size(); ++t) {
      const int base = kind == 1 ? mn[t].second * A.nb : mn[t].first * A.mb;
      const int len = kind == 1 ? A.cols(mn[t].second) : A.rows(mn[t].first);
      for (int j = 0; j < len; ++j) acc[base + j] += h[t * os + j];
    }
    if (comm && !acc.empty() && comm->allreduce(acc.data(), (int)acc.size(), false) != 0) return 0.0;
    for (double v : acc) r = std::max(r, v);
  }
  ok = true;
  return r;
}

double nat_lange(dplasma_context_t* ctx, int prec, int ntype, dplasma_desc_t* dA) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {A}, prec)) { dpl_set_error("lange: descriptor of another context"); return NAN; }
  bool ok;
  const double r = norm_tiles(*A, ntype, UPPERLOWER, false, ctx->nat->st[1], ok);
  if (!ok) { dpl_set_error("lange: unsupported norm or kernel failure"); return NAN; }
  return r;
}

double nat_lantr(dplasma_context_t* ctx, int prec, int ntype, int uplo, int diag, dplasma_desc_t* dA) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {A}, prec) || (uplo != LOWER && uplo != UPPER)) {
    dpl_set_error("lantr: bad descriptor or uplo");
    return NAN;
  }
  bool ok;
  const double r = norm_tiles(*A, ntype, uplo, diag == UNIT, ctx->nat->st[1], ok);
  if (!ok) { dpl_set_error("lantr: unsupported norm or kernel failure"); return NAN; }
  return r;
}

static NatProgram* generator(dplasma_context_t* ctx, int prec, int kind, int uplo, const Scalar& bump,
                             dplasma_desc_t* dA, unsigned long long seed, const char* name) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return fail(nullptr, std::string(name) + ": descriptor of another context");
  NatProgram* P = new_program(c, name, false);
  std::vector<TileItem> it;
  int mm = 0, nn = 0;
  for (int n = 0; n < A->nt; ++n)
    for (int m = 0; m < A->mt; ++m) {
      if ((uplo == LOWER && m < n) || (uplo == UPPER && m > n)) continue;
      if (!A->local(m, n)) continue;   // global element coordinates: every rank draws its own tiles
      it.push_back(TileItem{A->off(m, n), 0, A->rows(m), A->cols(n), m * A->mb, n * A->nb});
      mm = std::max(mm, A->rows(m));
      nn = std::max(nn, A->cols(n));
    }
  DevPtr d = dev_upload(it);
  if (!d) return fail(P, std::string(name) + ": device allocation failed");
  P->keep.push_back(d);
  const int ni = (int)it.size(), lda = A->lld;
  const long long gM = A->m;
  char* base = A->data;
  P->task(1, [=](hipStream_t s) {
    if (ni == 0) return 0;
    return dpl_generate(prec, kind, ni, d->p, mm, nn, base, lda, gM, seed, bump.ptr(), s);
  }, {});
  return P;
}

NatProgram* nat_plghe(dplasma_context_t* ctx, int prec, double bump, int uplo, dplasma_desc_t* A,
                      unsigned long long seed) {
  return generator(ctx, prec, 1, uplo, Scalar(prec, bump), A, seed, "plghe");
}

NatProgram* nat_plgsy(dplasma_context_t* ctx, int prec, const void* bump, int uplo, dplasma_desc_t* A,
                      unsigned long long seed) {
  return generator(ctx, prec, 2, uplo, Scalar(prec, bump), A, seed, "plgsy");
}

NatProgram* nat_plrnt(dplasma_context_t* ctx, int prec, int diagdom, dplasma_desc_t* A, unsigned long long seed) {
  if (diagdom) return fail(nullptr, "plrnt: diagdom is not available on a native context");
  return generator(ctx, prec, 0, UPPERLOWER, Scalar(prec, 0.0), A, seed, "plrnt");
}

// ----------------------------------------------------------------------------- execution
int nat_execute(dplasma_context_t* ctx, NatProgram* P) {
  if (!P) return -1;
  int rc = P->run();
  if (rc == 0) rc = P->wait();
  int res = rc == 0 ? P->result : -1;
  if (rc != 0) dpl_set_error(("native " + P->name + ": kernel launch failed").c_str());
  else if (res < 0) {
    // the dataflow tile kernels report a bounded-spin timeout (or another internal failure) as a
    // negative info: never a numerical result, always an error
    dpl_set_error(("native " + P->name + ": tile kernel failure (info " + std::to_string(res) + ")").c_str());
    res = -1;
  }
  (void)ctx;
  delete P;
  return res;
}

dplasma_taskpool_t* nat_wrap(NatProgram* P) {
  if (!P) return nullptr;
  dplasma_taskpool_t* tp = new dplasma_taskpool_s;
  tp->nat = P;
  return tp;
}

int nat_unsupported(const char* op) {
  dpl_set_error((std::string(op) + ": not available on a native context (dplasma_init_native)").c_str());
  return -1;
}

bool dpl_native(const dplasma_context_t* ctx) { return ctx && ctx->nat; }

int nat_ctx_attr(const dplasma_context_t* ctx, bool rank) { return rank ? ctx->nat->rank : ctx->nat->world; }

extern "C" {

static NatCtx* nat_ctx_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    dpl_set_error("dplasma_init_native: no such GPU");
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  NatCtx* c = new NatCtx;
  c->device = device;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  bool ok = true;
  for (int s = 0; s < NAT_NSTREAM; ++s)
    ok = ok && hipStreamCreateWithPriority(&c->st[s], hipStreamNonBlocking, s == 1 ? lo : hi) == hipSuccess &&
         hipEventCreateWithFlags(&c->join[s], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    dpl_set_error("dplasma_init_native: stream creation failed");
    nat_ctx_destroy(c);
    return nullptr;
  }
  return c;
}

DPL_CAPI dplasma_context_t* dplasma_init_native(int device) {
  NatCtx* c = nat_ctx_create(device);
  if (!c) return nullptr;
  dplasma_context_t* ctx = new dplasma_context_s;
  ctx->nat = c;
  return ctx;
}

// one process per GPU of a P x (world / P) grid (the reference's MPI ranks): tiles move between the
// ranks through RCCL (one GPU per rank) or node-local files (ranks sharing a GPU; one-GPU rehearsals),
// see native_comm.cpp; rdv_dir is a fresh directory every rank of the job can reach (the rendezvous)
DPL_CAPI dplasma_context_t* dplasma_init_native_dist(int device, int rank, int world, int P, const char* rdv_dir) {
  if (world < 1 || rank < 0 || rank >= world || P < 1 || world % P != 0) {
    dpl_set_error("dplasma_init_native_dist: rank / world / P do not form a P x Q grid");
    return nullptr;
  }
  NatCtx* c = nat_ctx_create(device);
  if (!c) return nullptr;
  c->rank = rank;
  c->world = world;
  c->P = P;
  c->Q = world / P;
  c->myrow = rank / c->Q;
  c->mycol = rank % c->Q;
  const char* lb = std::getenv("DPLASMA_LOOPBACK");
  c->loop = world == 1 && lb && *lb == '1';
  if (world > 1 || c->loop) {
    std::string err;
    c->comm = nat_comm_create(rank, world, device, rdv_dir, err);
    if (!c->comm) {
      dpl_set_error(("dplasma_init_native_dist: " + err).c_str());
      nat_ctx_destroy(c);
      return nullptr;
    }
  }
  dplasma_context_t* ctx = new dplasma_context_s;
  ctx->nat = c;
  return ctx;
}

}  // extern "C"

void nat_ctx_destroy(NatCtx* c) {
  if (c->comm) nat_comm_destroy(c->comm);
  c->comm = nullptr;
  for (int s = 0; s < NAT_NSTREAM; ++s) {
    if (c->st[s]) {
      (void)hipStreamSynchronize(c->st[s]);
      (void)hipStreamDestroy(c->st[s]);
    }
    if (c->join[s]) (void)hipEventDestroy(c->join[s]);
  }
  delete c;
}

void nat_fini(dplasma_context_t* ctx) { nat_ctx_destroy(ctx->nat); }

dplasma_desc_t* nat_desc(dplasma_context_t* ctx, int prec, int mb, int nb, int m, int n, int P, int Q, void* data,
                         int lld, int on_device) {
  NatCtx* c = ctx->nat;
  if (P <= 0 || Q <= 0) P = c->P, Q = c->Q;   // the context's grid
  if (prec == P_I) P = Q = 1;   // pivot vectors: replicated on every rank of a grid
  if ((!prec_ok(prec) && prec != P_I) || mb <= 0 || nb <= 0 || m < 0 || n < 0 ||
      (prec != P_I && (P != c->P || Q != c->Q))) {
    dpl_set_error("native descriptor: the context's process grid (P = Q = 1 on one process), positive tile "
                  "sizes, s/d/c/z");
    return nullptr;
  }
  if (data && !on_device) {
    dpl_set_error("native descriptor: caller memory must be device memory of the context's GPU");
    return nullptr;
  }
  NatDesc* d = new NatDesc;
  d->ctx = ctx->nat;
  d->prec = prec;
  d->es = esize(prec);
  d->mb = mb;
  d->nb = nb;
  d->m = m;
  d->n = n;
  d->mt = (m + mb - 1) / mb;
  d->nt = (n + nb - 1) / nb;
  d->P = P;
  d->Q = Q;
  d->myrow = P > 1 ? c->myrow : 0;
  d->mycol = Q > 1 ? c->mycol : 0;
  d->lm = nat_numroc(m, mb, d->myrow, P);
  d->ln = nat_numroc(n, nb, d->mycol, Q);
  if (data) {
    if (lld < std::max(1, d->lm)) {
      delete d;
      dpl_set_error("native descriptor: lld < m");
      return nullptr;
    }
    d->data = (char*)data;
    d->lld = lld;
  } else {
    // 128-byte aligned columns for the vector paths; pivot vectors (int32, 1 x n) stay contiguous
    d->lld = prec == P_I ? std::max(1, d->lm) : std::max(16, (d->lm + 15) / 16 * 16);
    void* p = nullptr;
    const size_t bytes = (size_t)d->lld * std::max(1, d->ln) * d->es;
    // the zeros must have landed before any kernel of the context's non-blocking streams touches the
    // buffer: a private stream + hipStreamSynchronize (see dpl_zero_sync in csrc/kernels/common.h)
    if (hipMalloc(&p, bytes) != hipSuccess || nat_zero_sync(p, bytes) != hipSuccess) {
      delete d;
      dpl_set_error("native descriptor: device allocation failed");
      return nullptr;
    }
    d->data = (char*)p;
    d->owned = true;
  }
  dplasma_desc_t* h = new dplasma_desc_s;
  h->nat = d;
  return h;
}

void nat_desc_free(dplasma_desc_t* A) { delete A->nat; }

// host LAPACK-layout matrix (the whole m x n matrix on every rank) <-> this rank's tiles
int nat_desc_io(const dplasma_desc_t* A, void* host, int lda, bool to_device) {
  const NatDesc* d = A->nat;
  if (lda < std::max(1, d->m)) return nat_unsupported("desc_set/get_lapack: lda < m");
  for (int s = 0; s < NAT_NSTREAM; ++s)
    if (hipStreamSynchronize(d->ctx->st[s]) != hipSuccess) return -1;
  if (d->m == 0 || d->n == 0) return 0;
  const size_t hp = (size_t)lda * d->es, dp = (size_t)d->lld * d->es;
  if (!d->dist()) {
    const size_t w = (size_t)d->m * d->es;
    const hipError_t e = to_device ? hipMemcpy2D(d->data, dp, host, hp, w, d->n, hipMemcpyHostToDevice)
                                   : hipMemcpy2D(host, hp, d->data, dp, w, d->n, hipMemcpyDeviceToHost);
    return e == hipSuccess ? 0 : -1;
  }
  for (int j = d->mycol; j < d->nt; j += d->Q)
    for (int i = d->myrow; i < d->mt; i += d->P) {
      char* h = (char*)host + ((size_t)i * d->mb + (size_t)j * d->nb * lda) * d->es;
      char* g = d->data + d->off(i, j) * d->es;
      const size_t w = (size_t)d->rows(i) * d->es;
      const hipError_t e = to_device ? hipMemcpy2D(g, dp, h, hp, w, d->cols(j), hipMemcpyHostToDevice)
                                     : hipMemcpy2D(h, hp, g, dp, w, d->cols(j), hipMemcpyDeviceToHost);
      if (e != hipSuccess) return -1;
    }
  return 0;
}

int nat_add(dplasma_context_t* ctx, dplasma_taskpool_t* tp) {
  if (!tp->nat || tp->nat->ctx != ctx->nat) return nat_unsupported("add_taskpool: taskpool of another context");
  ctx->nat->queue.push_back(tp->nat);
  return 0;
}

int nat_start(dplasma_context_t* ctx) {
  for (NatProgram* P : ctx->nat->queue)
    if (!P->enqueued && P->run() != 0) return -1;
  return 0;
}

int nat_wait(dplasma_context_t* ctx) {
  int rc = nat_start(ctx);
  for (NatProgram* P : ctx->nat->queue)
    if (P->enqueued && P->wait() != 0) rc = -1;
  ctx->nat->queue.clear();
  return rc;
}

int nat_result(const dplasma_taskpool_t* tp) { return tp->nat->result; }

void nat_free(dplasma_taskpool_t* tp) {
  NatProgram* P = tp->nat;
  if (P->enqueued) (void)P->wait();
  // a taskpool added but destroyed before dplasma_context_wait must leave its context's queue
  auto& q = P->ctx->queue;
  q.erase(std::remove(q.begin(), q.end(), P), q.end());
  delete P;
}

// ============================================================================= level-3 extras, LU
// TRMM / SYMM / HEMM (models/blas3.py): the triangular / symmetric operand is first expanded into a
// program-owned full-tile workspace (the triangle, zeros elsewhere -- unit diagonal if asked -- or the
// mirrored symmetric / Hermitian matrix), so the product is ONE launch of the MFMA GEMM engine whose
// k-runs cover exactly the non-zero tiles.  LU with partial pivoting (models/lu.py, one process):
// per panel, gather -> recursive panel LU (dgetrf2 recursion: 64-column persistent blocks, laswp,
// TRSM, MFMA GEMM) -> device-derived net row moves applied in place -> write-back -> U row TRSM ->
// trailing GEMM; pivots go to the IPIV descriptor on the device (1-based, global).
namespace {

std::shared_ptr<NatDesc> work_desc(NatProgram& P, const NatDesc& A) {
  auto w = std::make_shared<NatDesc>();
  w->ctx = A.ctx;
  w->prec = A.prec;
  w->es = A.es;
  w->mb = A.mb;
  w->nb = A.nb;
  w->m = A.m;
  w->n = A.n;
  w->mt = A.mt;
  w->nt = A.nt;
  w->P = A.P, w->Q = A.Q, w->myrow = A.myrow, w->mycol = A.mycol, w->lm = A.lm, w->ln = A.ln;   // A's distribution
  w->lld = std::max(16, (A.lm + 15) / 16 * 16);
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)w->lld * std::max(1, A.ln) * A.es) != hipSuccess) return nullptr;
  w->data = (char*)p;
  w->owned = true;
  P.wdesc.push_back(w);
  return w;
}

// W := expansion of A's uplo triangle: mode 0 -- triangle (zeros elsewhere; unit diagonal if unit),
// 1 -- symmetric (the other triangle mirrored with a transpose), 2 -- Hermitian (conjugate mirror,
// real diagonal).  Tasks on stream 1, in order after `prev`; returns the last task (or -2 on failure).
int add_expand(NatProgram& P, const NatDesc& A, int uplo, bool unit, int mode, NatDesc& W, int prev) {
  const int prec = A.prec;
  const Scalar zero(prec, 0.0), one(prec, 1.0), half(prec, 0.5);
  auto all = std::make_shared<MapBatch>(), tri = std::make_shared<MapBatch>(), mir = std::make_shared<MapBatch>();
  all->build(W, UPPERLOWER, nullptr, NOTRANS);
  tri->build(W, uplo, &A, NOTRANS);
  const int mtrans = mode == 2 ? CONJTRANS : TRANS;
  if (mode > 0 && !W.dist()) mir->build(W, uplo == LOWER ? UPPER : LOWER, &A, mtrans);
  if (mode > 0 && W.dist())   // the grid: diagonal tiles mirror in place, the others through nat_dist_mirror_into
    for (int k = 0; k < W.mt && k < W.nt; ++k)
      if (W.local(k, k)) {
        mir->it.push_back(TileItem{A.off(k, k), W.off(k, k), W.rows(k), W.cols(k), k * W.mb, k * W.nb});
        mir->mm = std::max(mir->mm, W.rows(k));
        mir->nn = std::max(mir->nn, W.cols(k));
      }
  if (!all->upload(P) || !tri->upload(P) || !mir->upload(P)) return -2;
  const int lda = A.lld, ldw = W.lld, tpart = part_of(uplo), mpart = uplo == LOWER ? 4 : 3;
  const char* a = A.data;
  char* w = W.data;
  if (mode == 0)
    prev = P.task(1, [=](hipStream_t s) {
      if (all->n() == 0) return 0;
      return dpl_laset(prec, 0, all->n(), all->items(), all->mm, all->nn, zero.ptr(), zero.ptr(), w, ldw, s);
    }, {prev});
  prev = P.task(1, [=](hipStream_t s) {
    if (tri->n() == 0) return 0;
    return dpl_geadd(prec, tpart, NOTRANS, tri->n(), tri->items(), tri->mm, tri->nn, one.ptr(), a, lda, zero.ptr(), w,
                     ldw, 1, s);
  }, {prev});
  if (mode > 0)
    prev = P.task(1, [=](hipStream_t s) {
      if (mir->n() == 0) return 0;
      return dpl_geadd(prec, mpart, mtrans, mir->n(), mir->items(), mir->mm, mir->nn, one.ptr(), a, lda, zero.ptr(),
                       w, ldw, 1, s);
    }, {prev});
  if (mode > 0 && W.dist()) {
    if (!nat_dist_mirror_into(P, A, uplo, mtrans, W)) return -2;
    prev = (int)P.tasks.size() - 1;
  }
  if ((mode == 0 && unit) || (mode == 2 && (prec == P_C || prec == P_Z))) {
    std::vector<TileItem> d;
    int mm = 0;
    for (int k = 0; k < W.mt && k < W.nt; ++k) {
      if (!W.local(k, k)) continue;
      d.push_back(TileItem{W.off(k, k), W.off(k, k), W.rows(k), W.cols(k), k * W.mb, k * W.nb});
      mm = std::max(mm, std::max(W.rows(k), W.cols(k)));
    }
    if (d.empty()) return prev;
    DevPtr dd = dev_upload(d);
    if (!dd) return -2;
    P.keep.push_back(dd);
    const int nd = (int)d.size();
    if (mode == 0)   // unit diagonal
      prev = P.task(1, [=](hipStream_t s) {
        return dpl_laset(prec, 5, nd, dd->p, mm, mm, zero.ptr(), one.ptr(), w, ldw, s);
      }, {prev});
    else             // diag := (diag + conj(diag)) / 2
      prev = P.task(1, [=](hipStream_t s) {
        return dpl_geadd(prec, 5, CONJTRANS, nd, dd->p, mm, mm, half.ptr(), w, ldw, half.ptr(), w, ldw, 0, s);
      }, {prev});
  }
  return prev;
}

}  // namespace

NatProgram* nat_trmm(dplasma_context_t* ctx, int prec, int side, int uplo, int trans, int diag, const void* alpha,
                     dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec)) return fail(nullptr, "trmm: descriptors of another context or precision");
  const bool left = side == LEFT, notrans = trans == NOTRANS;
  const int order = left ? B->m : B->n;
  if (A->m != A->n || A->m != order || A->mb != A->nb || (left ? B->mb : B->nb) != A->nb ||
      (uplo != LOWER && uplo != UPPER))
    return fail(nullptr, "trmm: operands do not conform");
  NatProgram* P = new_program(c, "trmm", false);
  auto T = work_desc(*P, *A), W = work_desc(*P, *B);
  if (!T || !W) return fail(P, "trmm: device allocation failed");
  int prev = add_expand(*P, *A, uplo, diag == UNIT, 0, *T, -1);
  auto cp = std::make_shared<MapBatch>();
  cp->build(*W, UPPERLOWER, B, NOTRANS);
  if (prev == -2 || !cp->upload(*P)) return fail(P, "trmm: device allocation failed");
  const Scalar one(prec, 1.0), zero(prec, 0.0), al(prec, alpha);
  char *bb = B->data, *wd = W->data, *td = T->data;
  const int ldb = B->lld, ldw = W->lld, ldt = T->lld;
  prev = P->task(1, [=](hipStream_t s) {
    if (cp->n() == 0) return 0;
    return dpl_geadd(prec, 0, NOTRANS, cp->n(), cp->items(), cp->mm, cp->nn, one.ptr(), bb, ldb, zero.ptr(), wd, ldw,
                     1, s);
  }, {prev});
  if (c->dist()) {   // the expanded triangle times the copy of B: the SUMMA GEMM over the grid
    const bool ok = left ? nat_dist_gemm_into(*P, prec, trans, NOTRANS, al, *T, *W, zero, *B)
                         : nat_dist_gemm_into(*P, prec, NOTRANS, trans, al, *W, *T, zero, *B);
    return ok ? P : fail(P, "trmm: device allocation failed");
  }
  // B(m,n) = alpha sum_k op(T)(m,k) W(k,n) (left) / alpha sum_k W(m,k) op(T)(k,n) (right), k over the
  // triangle only: op(A) is lower iff (uplo == Lower) == (trans == NoTrans)
  const bool lower_op = (uplo == LOWER) == notrans;
  auto g = std::make_shared<Gemm>();
  for (int n = 0; n < B->nt; ++n)
    for (int m = 0; m < B->mt; ++m) {
      std::vector<KPair> kp;
      const int i = left ? m : n;
      const int k0 = left ? (lower_op ? 0 : i) : (lower_op ? i : 0);
      const int k1 = left ? (lower_op ? i + 1 : A->mt) : (lower_op ? A->mt : i + 1);
      for (int k = k0; k < k1; ++k) {
        if (left)
          kp.push_back(KPair{notrans ? T->off(m, k) : T->off(k, m), W->off(k, n), A->rows(k), 0});
        else
          kp.push_back(KPair{W->off(m, k), notrans ? T->off(k, n) : T->off(n, k), A->rows(k), 0});
      }
      g->add(B->off(m, n), B->rows(m), B->cols(n), kp, 0);
    }
  if (!g->upload(*P)) return fail(P, "trmm: device allocation failed");
  if (left)
    P->task(1, [=](hipStream_t s) { return g->launch(prec, trans, NOTRANS, al, td, ldt, wd, ldw, zero, bb, ldb, s); },
            {prev});
  else
    P->task(1, [=](hipStream_t s) { return g->launch(prec, NOTRANS, trans, al, wd, ldw, td, ldt, zero, bb, ldb, s); },
            {prev});
  return P;
}

static NatProgram* symm_like(dplasma_context_t* ctx, int prec, int side, int uplo, const void* alpha,
                             dplasma_desc_t* dA, dplasma_desc_t* dB, const void* beta, dplasma_desc_t* dC, bool herm) {
  const char* name = herm ? "hemm" : "symm";
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx_dist(c, {A, B, C}, prec)) return fail(nullptr, std::string(name) + ": descriptors of another context");
  const bool left = side == LEFT;
  if (A->m != A->n || A->mb != A->nb || B->m != C->m || B->n != C->n || B->mb != C->mb || B->nb != C->nb ||
      (left ? C->m : C->n) != A->m || (left ? C->mb : C->nb) != A->nb || (uplo != LOWER && uplo != UPPER))
    return fail(nullptr, std::string(name) + ": operands do not conform");
  NatProgram* P = new_program(c, name, false);
  auto S = work_desc(*P, *A);
  if (!S) return fail(P, std::string(name) + ": device allocation failed");
  const int prev = add_expand(*P, *A, uplo, false, herm ? 2 : 1, *S, -1);
  if (prev == -2) return fail(P, std::string(name) + ": device allocation failed");
  if (c->dist()) {   // the expanded operand times B: the SUMMA GEMM over the grid
    const Scalar al(prec, alpha), be(prec, beta);
    const bool ok = left ? nat_dist_gemm_into(*P, prec, NOTRANS, NOTRANS, al, *S, *B, be, *C)
                         : nat_dist_gemm_into(*P, prec, NOTRANS, NOTRANS, al, *B, *S, be, *C);
    return ok ? P : fail(P, std::string(name) + ": device allocation failed");
  }
  auto g = std::make_shared<Gemm>();
  for (int n = 0; n < C->nt; ++n)
    for (int m = 0; m < C->mt; ++m) {
      std::vector<KPair> kp;
      for (int k = 0; k < A->mt; ++k)
        kp.push_back(left ? KPair{S->off(m, k), B->off(k, n), A->rows(k), 0}
                          : KPair{B->off(m, k), S->off(k, n), A->rows(k), 0});
      g->add(C->off(m, n), C->rows(m), C->cols(n), kp, 0);
    }
  if (prev == -2 || !g->upload(*P)) return fail(P, std::string(name) + ": device allocation failed");
  const Scalar al(prec, alpha), be(prec, beta);
  const char *sd = S->data, *bd = B->data;
  char* cd = C->data;
  const int lds = S->lld, ldb = B->lld, ldc = C->lld;
  if (left)
    P->task(1, [=](hipStream_t s) { return g->launch(prec, NOTRANS, NOTRANS, al, sd, lds, bd, ldb, be, cd, ldc, s); },
            {prev});
  else
    P->task(1, [=](hipStream_t s) { return g->launch(prec, NOTRANS, NOTRANS, al, bd, ldb, sd, lds, be, cd, ldc, s); },
            {prev});
  return P;
}

NatProgram* nat_symm(dplasma_context_t* ctx, int prec, int side, int uplo, const void* alpha, dplasma_desc_t* A,
                     dplasma_desc_t* B, const void* beta, dplasma_desc_t* C) {
  return symm_like(ctx, prec, side, uplo, alpha, A, B, beta, C, false);
}

NatProgram* nat_hemm(dplasma_context_t* ctx, int prec, int side, int uplo, const void* alpha, dplasma_desc_t* A,
                     dplasma_desc_t* B, const void* beta, dplasma_desc_t* C) {
  if (prec != P_C && prec != P_Z) return fail(nullptr, "hemm: complex precisions only");
  return symm_like(ctx, prec, side, uplo, alpha, A, B, beta, C, true);
}

// lansy / lanhe: the norm of the expanded symmetric / Hermitian matrix (synchronous, like lange)
static double norm_sym(dplasma_context_t* ctx, int prec, int ntype, int uplo, dplasma_desc_t* dA, bool herm) {
  NatDesc* A = dA ? dA->nat : nullptr;
  const char* name = herm ? "lanhe" : "lansy";
  if (!same_ctx_dist(ctx->nat, {A}, prec) || (uplo != LOWER && uplo != UPPER) || A->m != A->n || A->mb != A->nb) {
    dpl_set_error((std::string(name) + ": bad descriptor or uplo").c_str());
    return NAN;
  }
  // (a multi-process context: the mirrored triangle is exchanged, then the partial norms all-reduced)
  NatProgram* P = new_program(ctx->nat, name, false);
  auto S = work_desc(*P, *A);
  if (!S || add_expand(*P, *A, uplo, false, herm ? 2 : 1, *S, -1) == -2) {
    delete P;
    dpl_set_error((std::string(name) + ": device allocation failed").c_str());
    return NAN;
  }
  auto keep = P->wdesc;    // the expanded matrix outlives the program
  if (P->run() != 0 || P->wait() != 0) {
    delete P;
    dpl_set_error((std::string(name) + ": kernel launch failed").c_str());
    return NAN;
  }
  delete P;
  bool ok;
  const double r = norm_tiles(*S, ntype, UPPERLOWER, false, ctx->nat->st[1], ok);
  if (!ok) { dpl_set_error((std::string(name) + ": unsupported norm or kernel failure").c_str()); return NAN; }
  return r;
}

double nat_lansy(dplasma_context_t* ctx, int prec, int ntype, int uplo, dplasma_desc_t* A) {
  return norm_sym(ctx, prec, ntype, uplo, A, false);
}

double nat_lanhe(dplasma_context_t* ctx, int prec, int ntype, int uplo, dplasma_desc_t* A) {
  if (prec != P_C && prec != P_Z) { dpl_set_error("lanhe: complex precisions only"); return NAN; }
  return norm_sym(ctx, prec, ntype, uplo, A, true);
}

// ----------------------------------------------------------------------------- TRTRI / LAUUM / POTRI
// trtri: inv(T) of A's uplo triangle as one blocked TRSM of an identity right-hand side (the MFMA
// TRSM path: per block row a strip solve + one GEMM), its triangle copied back (strictly, for a unit
// diagonal).  lauum: L^H L (lower) / U U^H (upper) as one rank-k launch over the triangle of the
// expanded factor (zeros outside it).  potri = trtri + lauum, poinv = potrf + potri (src/zpotri_wrapper.c,
// src/zpoinv_wrapper.c: the same algebra as the reference's tile algorithms, batched per launch).
namespace {

int add_trtri(NatProgram& P, int uplo, int diag, NatDesc& A, int prev) {
  const int prec = A.prec;
  auto X = work_desc(P, A);
  if (!X) return -2;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  auto all = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
  all->build(*X, UPPERLOWER, nullptr, NOTRANS);
  back->build(A, uplo, X.get(), NOTRANS);
  if (!all->upload(P) || !back->upload(P)) return -2;
  char *xd = X->data, *ad = A.data;
  const int ldx = X->lld, lda = A.lld;
  prev = P.task(1, [=](hipStream_t s) {   // X := I
    if (all->n() == 0) return 0;
    return dpl_laset(prec, 0, all->n(), all->items(), all->mm, all->nn, zero.ptr(), one.ptr(), xd, ldx, s);
  }, {prev});
  if (A.ctx->dist() ? !nat_dist_trsm_into(P, LEFT, uplo, NOTRANS, diag, one, A, *X)
                    : !add_trsm(P, LEFT, uplo, NOTRANS, diag, one, A, *X, 1, prev))
    return -2;
  // strictly lower / upper for a unit diagonal (the diagonal of A is not referenced), else with it
  const int part = uplo == LOWER ? (diag == UNIT ? 3 : 1) : (diag == UNIT ? 4 : 2);
  return P.task(1, [=](hipStream_t s) {
    if (back->n() == 0) return 0;
    return dpl_geadd(prec, part, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), xd, ldx,
                     zero.ptr(), ad, lda, 1, s);
  }, {last_on(P, 0), last_on(P, 1), last_on(P, 2)});
}

int add_lauum(NatProgram& P, int uplo, NatDesc& A, int prev) {
  const int prec = A.prec;
  auto T = work_desc(P, A);
  if (!T) return -2;
  prev = add_expand(P, A, uplo, false, 0, *T, prev);
  if (prev == -2) return -2;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  const bool herm = prec == P_C || prec == P_Z;
  // lower: A = T^H T = op(T) op(T)^H with op = ^H;  upper: A = T T^H
  const int trans = uplo == LOWER ? (herm ? CONJTRANS : TRANS) : NOTRANS;
  return add_rank_k(P, prec, uplo, trans, one, T.get(), T.get(), zero, &A, herm, prev);
}

bool square_tiles(const NatDesc* A, int uplo) {
  return A && A->m == A->n && A->mb == A->nb && (uplo == LOWER || uplo == UPPER);
}

}  // namespace

NatProgram* nat_trtri(dplasma_context_t* ctx, int prec, int uplo, int diag, dplasma_desc_t* dA) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {A}, prec) || !square_tiles(A, uplo))
    return fail(nullptr, "trtri: square matrix with square tiles and uplo Lower/Upper required");
  NatProgram* P = new_program(ctx->nat, "trtri", false);
  if (add_trtri(*P, uplo, diag, *A, -1) == -2) return fail(P, "trtri: device allocation failed");
  return P;
}

NatProgram* nat_lauum(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {A}, prec) || !square_tiles(A, uplo))
    return fail(nullptr, "lauum: square matrix with square tiles and uplo Lower/Upper required");
  NatProgram* P = new_program(ctx->nat, "lauum", false);
  if (add_lauum(*P, uplo, *A, -1) == -2) return fail(P, "lauum: device allocation failed");
  return P;
}

NatProgram* nat_potri(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(ctx->nat, {A}, prec) || !square_tiles(A, uplo))
    return fail(nullptr, "potri: square matrix with square tiles and uplo Lower/Upper required");
  NatProgram* P = new_program(ctx->nat, "potri", false);
  int t = add_trtri(*P, uplo, NONUNIT, *A, -1);
  if (t != -2) t = add_lauum(*P, uplo, *A, t);
  if (t == -2) return fail(P, "potri: device allocation failed");
  return P;
}

NatProgram* nat_poinv(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA) {
  NatProgram* P = nat_potrf(ctx, prec, uplo, dA);
  if (!P) return nullptr;
  // the inversion (update stream) starts after the factorisation's last panel-stream task
  int t = add_trtri(*P, uplo, NONUNIT, *dA->nat, last_on(*P, 0));
  if (t != -2) t = add_lauum(*P, uplo, *dA->nat, t);
  if (t == -2) return fail(P, "poinv: device allocation failed");
  return P;
}

// ----------------------------------------------------------------------------- LU (partial pivoting)
namespace {

constexpr int LU_BW = 64;   // base-case width of the recursive panel (dpl_lu_block)

struct LuScratch {
  DevPtr pv, piv, ws, cnt, mdst, msrc, mcnt, rowoff, coloff, ncols;
};

// the dgetrf2 recursion of ops.PanelLU on the panel pv (m x n, ld): tasks on stream 1 after prev
int add_panel_lu(NatProgram& P, int prec, char* pv, int ld, int m, int c0, int n, const LuScratch& S, int* info,
                 int info_base, int prev, bool pivot = true) {
  const Scalar one(prec, 1.0), m_one(prec, -1.0);
  int* piv = (int*)S.piv->p;
  void* ws = S.ws->p;
  int* cnt = (int*)S.cnt->p;
  if (n <= LU_BW) {
    return P.task(1, [=](hipStream_t s) {
      return dpl_lu_block(prec, pv, ld, m, c0, c0 + n, piv, ws, cnt, info, info_base, pivot ? 1 : 0, s);
    }, {prev});
  }
  const int n1 = (n / 2 + 15) / 16 * 16, c1 = c0 + n1;
  prev = add_panel_lu(P, prec, pv, ld, m, c0, n1, S, info, info_base, prev, pivot);
  if (prev < 0) return prev;
  if (pivot)
    prev = P.task(1, [=](hipStream_t s) { return dpl_laswp_panel(prec, pv, ld, m, c1, c0 + n, piv, c0, c1, info, s); }, {prev});
  auto tr = std::make_shared<Trsm1>();
  tr->tri = c0 + (long long)c0 * ld;
  tr->add(c0 + (long long)c1 * ld, n1, n - n1);
  if (!tr->upload(P, prec, LEFT)) return -2;
  prev = P.task(1, [=](hipStream_t s) {
    return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, pv, ld, pv, ld, s);
  }, {prev});
  if (m > c1) {
    auto g = std::make_shared<Gemm>();
    g->add(c1 + (long long)c1 * ld, m - c1, n - n1, {KPair{c1 + (long long)c0 * ld, c0 + (long long)c1 * ld, n1, 0}},
           0);
    if (!g->upload(P)) return -2;
    prev = P.task(1, [=](hipStream_t s) {
      return g->launch(prec, NOTRANS, NOTRANS, m_one, pv, ld, pv, ld, one, pv, ld, s);
    }, {prev});
  }
  prev = add_panel_lu(P, prec, pv, ld, m, c1, n - n1, S, info, info_base, prev, pivot);
  if (prev < 0 || !pivot) return prev;
  return P.task(1, [=](hipStream_t s) { return dpl_laswp_panel(prec, pv, ld, m, c0, c1, piv, c1, c0 + n, info, s); }, {prev});
}

bool lu_scratch(NatProgram& P, const NatDesc& A, LuScratch& S) {
  S.pv = dev_alloc((size_t)std::max(1, A.m) * A.nb * A.es, false);
  S.piv = dev_alloc(sizeof(int) * (A.nb + 16), true);
  S.ws = dev_alloc((size_t)dpl_lu_block_ws_bytes(std::max(1, A.m)) + 64, true);
  S.cnt = dev_alloc(64, true);
  S.mdst = dev_alloc(sizeof(int) * 2 * (A.mb + 16), true);
  S.msrc = dev_alloc(sizeof(int) * 2 * (A.mb + 16), true);
  S.mcnt = dev_alloc(64, true);
  std::vector<long long> ro(A.mt), co(A.nt);
  std::vector<int> nc(A.nt);
  for (int m = 0; m < A.mt; ++m) ro[m] = A.off(m, 0);
  for (int n = 0; n < A.nt; ++n) {
    co[n] = A.off(0, n);
    nc[n] = A.cols(n);
  }
  S.rowoff = dev_upload(ro);
  S.coloff = dev_upload(co);
  S.ncols = dev_upload(nc);
  for (const DevPtr& d : {S.pv, S.piv, S.ws, S.cnt, S.mdst, S.msrc, S.mcnt, S.rowoff, S.coloff, S.ncols}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  return true;
}

// row interchanges of panel step k (rows r0 + piv[j] <-> r0 + j, j < kmin, sequential) applied to every
// tile column of B in place (forward) or undone (inverse: the net moves with source and destination swapped)
int add_row_moves(NatProgram& P, const NatDesc& B, const LuScratch& S, const DevPtr& rowoff, const DevPtr& coloff,
                  const DevPtr& ncols, int r0, int kmin, bool inverse, int prev) {
  const int prec = B.prec, ld = B.lld, mb = B.mb, nb = B.nb, mt = B.mt, nt = B.nt, maxcnt = 2 * mb;
  char* b = B.data;
  const int* piv = (const int*)S.piv->p;
  int *dst = (int*)S.mdst->p, *src = (int*)S.msrc->p, *cnt = (int*)S.mcnt->p;
  const long long *ro = (const long long*)rowoff->p, *co = (const long long*)coloff->p;
  const int* nc = (const int*)ncols->p;
  // an out-of-range pivot: info -1001 (lu_piv.hip report_bad_pivot), nothing moved -- a solve program (getrs,
  // laswp) gets an info word for it, so the caller sees a failure instead of a silently wrong result
  if (!P.info) P.info = dev_alloc(sizeof(int), true);
  if (!P.info) return -2;
  int* info = (int*)P.info->p;
  const int mrel = B.m - r0;
  prev = P.task(1, [=](hipStream_t s) { return dpl_piv_moves(piv, kmin, mrel, dst, src, cnt, info, s); }, {prev});
  return P.task(1, [=](hipStream_t s) {
    return dpl_rows_permute(prec, b, ld, mb, r0, ro, mt, co, nc, nt, nb, inverse ? src : dst, inverse ? dst : src, cnt,
                            maxcnt, info, s);
  }, {prev});
}

// IP == nullptr: getrf_nopiv (the same panel recursion and updates without interchanges)
bool add_getrf(NatProgram& P, NatDesc& A, NatDesc* IP, int& last) {
  const bool pivot = IP != nullptr;
  const int prec = A.prec, mb = A.mb, ld = A.lld;
  const int kt = std::min(A.mt, A.nt);
  LuScratch S;
  if (!lu_scratch(P, A, S)) return false;
  char* a = A.data;
  char* pvb = (char*)S.pv->p;
  int* info = (int*)P.info->p;
  int* ipg = pivot ? (int*)IP->data : nullptr;
  const Scalar one(prec, 1.0), m_one(prec, -1.0), zero(prec, 0.0);
  int prev = last;
  for (int k = 0; k < kt; ++k) {
    const int kb = A.cols(k), r0 = k * mb, mp = A.m - r0, kmin = std::min(mp, kb);
    // gather column k (tiles m >= k) into the contiguous panel (ld = mp)
    auto gat = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
    for (int m = k; m < A.mt; ++m) {
      gat->it.push_back(TileItem{A.off(m, k), (long long)(m - k) * mb, A.rows(m), kb, 0, 0});
      back->it.push_back(TileItem{(long long)(m - k) * mb, A.off(m, k), A.rows(m), kb, 0, 0});
      gat->mm = back->mm = std::max(gat->mm, A.rows(m));
    }
    gat->nn = back->nn = kb;
    if (!gat->upload(P) || !back->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      return dpl_geadd(prec, 0, NOTRANS, gat->n(), gat->items(), gat->mm, gat->nn, one.ptr(), a, ld, zero.ptr(), pvb,
                       mp, 1, s);
    }, {prev});
    prev = add_panel_lu(P, prec, pvb, mp, mp, 0, kmin, S, info, r0, prev, pivot);
    if (prev < 0) return false;
    if (kb > kmin) {   // wide last panel: the columns past the last row get the swaps and U = L^-1 A
      const int* piv = (const int*)S.piv->p;
      if (pivot)
        prev = P.task(1, [=](hipStream_t s) { return dpl_laswp_panel(prec, pvb, mp, mp, kmin, kb, piv, 0, kmin, info, s); },
                      {prev});
      auto tr = std::make_shared<Trsm1>();
      tr->tri = 0;
      tr->add((long long)kmin * mp, kmin, kb - kmin);
      if (!tr->upload(P, prec, LEFT)) return false;
      prev = P.task(1, [=](hipStream_t s) {
        return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, pvb, mp, pvb, mp, s);
      }, {prev});
    }
    // pivots -> IPIV (1-based, global); net row moves on every tile column; factored panel back
    const int* piv = (const int*)S.piv->p;
    if (pivot) {
      prev = P.task(1, [=](hipStream_t s) { return dpl_ipiv_shift(piv, ipg + r0, kmin, r0 + 1, s); }, {prev});
      prev = add_row_moves(P, A, S, S.rowoff, S.coloff, S.ncols, r0, kmin, false, prev);
    }
    prev = P.task(1, [=](hipStream_t s) {
      return dpl_geadd(prec, 0, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), pvb, mp, zero.ptr(),
                       a, ld, 1, s);
    }, {prev});
    if (k + 1 >= A.nt) continue;
    // U row: A(k, n) := L11^-1 A(k, n); trailing update A(m, n) -= L(m, k) U(k, n)
    auto tr = std::make_shared<Trsm1>();
    tr->tri = 0;
    for (int n = k + 1; n < A.nt; ++n) tr->add(A.off(k, n), kmin, A.cols(n));
    if (!tr->upload(P, prec, LEFT)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, pvb, mp, a, ld, s);
    }, {prev});
    if (k + 1 >= A.mt) continue;
    auto g = std::make_shared<Gemm>();
    for (int n = k + 1; n < A.nt; ++n)
      for (int m = k + 1; m < A.mt; ++m)
        g->add(A.off(m, n), A.rows(m), A.cols(n), {KPair{(long long)(m - k) * mb, A.off(k, n), kmin, 0}}, 0);
    if (!g->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      return g->launch(prec, NOTRANS, NOTRANS, m_one, pvb, mp, a, ld, one, a, ld, s);
    }, {prev});
  }
  last = prev;
  return true;
}

// The net row interchanges of one panel step (rows r0 + j <-> r0 + piv[j], j < kmin, in order; piv on the
// device, 0-based within the panel) applied to every local tile column of B on a grid: planned on the host
// at run time (one synchronisation), rows that cross process rows travel point to point within the process
// column, every source row read before any destination is written.  RB: scratch for 2 x (mb + 16) rows.
// IT: item staging allocated once per program (3 regions of 2 (mb + 16) TileItems: pack / local unpack /
// remote unpack), so a panel step neither allocates nor frees device memory (hipFree synchronises the device)
int add_rowmoves_dist(NatProgram& P, NatDesc& B, const int* piv, int r0, int kmin, const DevPtr& RB, const DevPtr& IT,
                      int prev) {
  NatComm* comm = P.ctx->comm;
  const int prec = B.prec, mb = B.mb, ld = B.lld, es = B.es, Pg = B.P, Q = B.Q, ln = B.ln;
  const int myrow = B.myrow, mycol = B.mycol;
  char *a = B.data, *rb = (char*)RB->p;
  TileItem* itb = (TileItem*)IT->p;
  const size_t itr = (size_t)2 * (mb + 16);   // items per region
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  auto lrow = [=](int r) { return (long long)((r / mb) / Pg) * mb + r % mb; };   // local row of a global row
  return P.task(1, [=](hipStream_t s) {
    if (ln == 0 || kmin == 0) return 0;
    std::vector<int> hp(kmin);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(hp.data(), piv, sizeof(int) * kmin, hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    // row -> row whose content it holds, touched rows only (std::map: references stay valid while the
    // swaps insert, and every rank walks the moves in the same ascending order)
    std::map<int, int> content;
    auto find = [&](int r) -> int& { return content.try_emplace(r, r).first->second; };
    for (int j = 0; j < kmin; ++j) std::swap(find(r0 + j), find(r0 + hp[j]));
    std::vector<TileItem> pack, ul, ur;
    std::vector<NatMsg> snd, rcv;
    const long long rs = ln;   // one packed row: ln contiguous entries
    int ns = 0, nr = 0;
    char* sbuf = rb;
    char* rbuf = rb + (size_t)2 * (mb + 16) * ln * es;
    for (const auto& [d, src] : content) {
      if (d == src) continue;
      const int pd = (d / mb) % Pg, ps = (src / mb) % Pg;
      if (ps == myrow) {
        pack.push_back(TileItem{lrow(src), ns * rs, 1, ln, 0, 0});
        if (pd == myrow) ul.push_back(TileItem{ns * rs, lrow(d), 1, ln, 0, 0});
        else snd.push_back(NatMsg{pd * Q + mycol, sbuf + (size_t)ns * rs * es, (size_t)rs * es});
        ++ns;
      } else if (pd == myrow) {
        ur.push_back(TileItem{nr * rs, lrow(d), 1, ln, 0, 0});
        rcv.push_back(NatMsg{ps * Q + mycol, rbuf + (size_t)nr * rs * es, (size_t)rs * es});
        ++nr;
      }
    }
    // each list has its own item region (the task began with a stream synchronisation, so no launch of
    // the previous step still reads them); the host copies are synchronous (pageable sources)
    auto launch = [&](const std::vector<TileItem>& it, int region, const char* src, int lds, char* dst, int ldd) -> int {
      if (it.empty()) return 0;
      if (it.size() > itr) return -1;
      TileItem* d = itb + region * itr;
      if (hipMemcpy(d, it.data(), it.size() * sizeof(TileItem), hipMemcpyHostToDevice) != hipSuccess) return -1;
      return dpl_geadd(prec, 0, NOTRANS, (int)it.size(), d, 1, ln, one.ptr(), src, lds, zero.ptr(), dst, ldd, 1, s);
    };
    int rc = launch(pack, 0, a, ld, sbuf, 1);
    if (rc == 0) rc = comm->exchange(snd, rcv, s);
    if (rc == 0) rc = launch(ul, 1, sbuf, 1, a, ld);
    if (rc == 0) rc = launch(ur, 2, rbuf, 1, a, ld);
    return rc;
  }, {prev});
}

// getrs (NoTrans) on a grid: the pivots of every panel step applied to B's rows, then L (unit) and U solves
bool add_getrs_dist(NatProgram& P, NatDesc& A, NatDesc& IP, NatDesc& B) {
  const int kt = std::min(A.mt, A.nt), mb = A.mb;
  DevPtr RB = dev_alloc((size_t)2 * 2 * (mb + 16) * std::max(1, B.ln) * B.es, false);
  DevPtr PV = dev_alloc(sizeof(int) * (mb + 16), false);
  DevPtr IT = dev_alloc(sizeof(TileItem) * 3 * 2 * (mb + 16), false);
  if (!RB || !PV || !IT) return false;
  P.keep.push_back(RB);
  P.keep.push_back(PV);
  P.keep.push_back(IT);
  const int* ipg = (const int*)IP.data;
  int* pv = (int*)PV->p;
  int prev = (int)P.tasks.size() - 1;   // after everything so far (a factorisation)
  for (int k = 0; k < kt; ++k) {
    const int r0 = k * mb, kmin = std::min(A.m - r0, A.cols(k));
    // IPIV holds 1-based global rows: back to 0-based within the panel for the planner
    prev = P.task(1, [=](hipStream_t s) { return dpl_ipiv_shift(ipg + r0, pv, kmin, -(r0 + 1), s); },
                  {prev, last_on(P, 0), last_on(P, 2)});
    prev = add_rowmoves_dist(P, B, pv, r0, kmin, RB, IT, prev);
  }
  const Scalar one(B.prec, 1.0);
  return nat_dist_trsm_into(P, LEFT, LOWER, NOTRANS, UNIT, one, A, B) &&
         nat_dist_trsm_into(P, LEFT, UPPER, NOTRANS, NONUNIT, one, A, B);
}

// LU with partial pivoting on a P x Q grid (multi-process native context; reference src/zgetrf_1d.jdf /
// zgetrf_ptgpanel.jdf): per panel step every rank receives the whole panel (one exchange), factors it
// redundantly with the device recursion above -- identical inputs and deterministic kernels give every rank
// the same pivots and factors, the role of the reference's distributed pivot search --, applies the net
// row interchanges to its local tile columns (rows that cross process rows travel point to point within
// the process column; the moves are planned on the host from the pivots, one synchronisation per panel),
// writes its panel tiles back, the panel's process row solves its U row, U travels down the process
// columns, and one MFMA GEMM launch updates the local trailing tiles.  All on one stream, in order.
bool add_getrf_dist(NatProgram& P, NatDesc& A, NatDesc& IP) {
  NatCtx* c = P.ctx;
  NatComm* comm = c->comm;
  const int prec = A.prec, mb = A.mb, ld = A.lld, es = A.es, me = c->rank, Pg = A.P, Qg = A.Q;
  const int kt = std::min(A.mt, A.nt), ln = A.ln;
  LuScratch S;
  if (!lu_scratch(P, A, S)) return false;
  const size_t st = (size_t)mb * A.nb;
  DevPtr TS = dev_alloc((size_t)std::max(1, A.mt) * st * es, false), US = dev_alloc((size_t)std::max(1, A.nt) * st * es, false);
  DevPtr RB = dev_alloc((size_t)2 * 2 * (mb + 16) * std::max(1, ln) * es, false);   // row-move send / receive rows
  DevPtr IT = dev_alloc(sizeof(TileItem) * 3 * 2 * (mb + 16), false);                 // their copy items
  if (!TS || !US || !RB || !IT) return false;
  for (const DevPtr& d : {TS, US, RB, IT}) P.keep.push_back(d);
  char *a = A.data, *pvb = (char*)S.pv->p, *ts = (char*)TS->p, *us = (char*)US->p, *rb = (char*)RB->p;
  int* info = (int*)P.info->p;
  int* ipg = (int*)IP.data;
  const int* piv = (const int*)S.piv->p;
  const Scalar one(prec, 1.0), m_one(prec, -1.0), zero(prec, 0.0);
  int prev = -1;
  for (int k = 0; k < kt; ++k) {
    const int kb = A.cols(k), r0 = k * mb, mp = A.m - r0, kmin = std::min(mp, kb);
    // ---- 1. the panel to every rank: owners pack, one exchange, scatter into the contiguous panel (ld mp)
    auto pk = std::make_shared<MapBatch>(), sc = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
    auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
    for (int m = k; m < A.mt; ++m) {
      const int src = A.owner(m, k);
      char* slot = ts + (size_t)m * st * es;
      if (src == me) {
        pk->it.push_back(TileItem{A.off(m, k), (long long)m * (long long)st, A.rows(m), kb, 0, 0});
        back->it.push_back(TileItem{(long long)(m - k) * mb, A.off(m, k), A.rows(m), kb, 0, 0});
        for (int r = 0; r < c->world; ++r)
          if (r != me) sends->push_back(NatMsg{r, slot, st * es});
      } else {
        recvs->push_back(NatMsg{src, slot, st * es});
      }
      sc->it.push_back(TileItem{(long long)m * (long long)st, (long long)(m - k) * mb, A.rows(m), kb, 0, 0});
      pk->mm = sc->mm = back->mm = std::max(pk->mm, A.rows(m));
    }
    pk->nn = sc->nn = back->nn = kb;
    if (!pk->upload(P) || !sc->upload(P) || !back->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      int rc = pk->n() ? dpl_geadd(prec, 0, NOTRANS, pk->n(), pk->items(), pk->mm, pk->nn, one.ptr(), a, ld, zero.ptr(),
                                   ts, mb, 1, s) : 0;
      if (rc == 0) rc = comm->exchange(*sends, *recvs, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, NOTRANS, sc->n(), sc->items(), sc->mm, sc->nn, one.ptr(), ts, mb, zero.ptr(), pvb, mp, 1, s);
      return rc;
    }, {prev});
    // ---- 2. the panel factorisation (every rank, the same result)
    prev = add_panel_lu(P, prec, pvb, mp, mp, 0, kmin, S, info, r0, prev);
    if (prev < 0) return false;
    if (kb > kmin) {
      prev = P.task(1, [=](hipStream_t s) { return dpl_laswp_panel(prec, pvb, mp, mp, kmin, kb, piv, 0, kmin, info, s); }, {prev});
      auto tr = std::make_shared<Trsm1>();
      tr->tri = 0;
      tr->add((long long)kmin * mp, kmin, kb - kmin);
      if (!tr->upload(P, prec, LEFT)) return false;
      prev = P.task(1, [=](hipStream_t s) { return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, pvb, mp, pvb, mp, s); },
                    {prev});
    }
    prev = P.task(1, [=](hipStream_t s) { return dpl_ipiv_shift(piv, ipg + r0, kmin, r0 + 1, s); }, {prev});
    // ---- 3. net row interchanges on this rank's tile columns, planned from the pivots
    prev = add_rowmoves_dist(P, A, piv, r0, kmin, RB, IT, prev);
    // ---- 4. my tiles of the factored panel back into A
    prev = P.task(1, [=](hipStream_t s) {
      if (back->n() == 0) return 0;
      return dpl_geadd(prec, 0, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), pvb, mp, zero.ptr(),
                       a, ld, 1, s);
    }, {prev});
    if (k + 1 >= A.nt) continue;
    // ---- 5. U row (the panel's process row) and 6. U down the process columns
    auto tr = std::make_shared<Trsm1>();
    auto pu = std::make_shared<MapBatch>();
    tr->tri = 0;
    auto usend = std::make_shared<std::vector<NatMsg>>(), urecv = std::make_shared<std::vector<NatMsg>>();
    for (int n = k + 1; n < A.nt; ++n) {
      const int src = A.owner(k, n);
      char* slot = us + (size_t)n * st * es;
      if (src == me) {
        tr->add(A.off(k, n), kmin, A.cols(n));
        pu->it.push_back(TileItem{A.off(k, n), (long long)n * (long long)st, kmin, A.cols(n), 0, 0});
        pu->mm = std::max(pu->mm, kmin);
        pu->nn = std::max(pu->nn, A.cols(n));
      }
      std::set<int> cs;   // ranks holding trailing tiles (m > k) of tile column n
      for (int m = k + 1; m < std::min(A.mt, k + 1 + Pg); ++m) cs.insert(A.owner(m, n));
      cs.erase(src);
      if (src == me)
        for (int r : cs) usend->push_back(NatMsg{r, slot, st * es});
      else if (cs.count(me))
        urecv->push_back(NatMsg{src, slot, st * es});
    }
    if (!tr->it.empty()) {
      if (!tr->upload(P, prec, LEFT) || !pu->upload(P)) return false;
      prev = P.task(1, [=](hipStream_t s) {
        int rc = tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, pvb, mp, a, ld, s);
        if (rc == 0)
          rc = dpl_geadd(prec, 0, NOTRANS, pu->n(), pu->items(), pu->mm, pu->nn, one.ptr(), a, ld, zero.ptr(), us, mb, 1, s);
        return rc;
      }, {prev});
    }
    prev = P.task(1, [=](hipStream_t s) { return comm->exchange(*usend, *urecv, s); }, {prev});
    // ---- 7. trailing update of my tiles
    if (k + 1 >= A.mt) continue;
    auto g = std::make_shared<Gemm>();
    for (int n = k + 1; n < A.nt; ++n)
      for (int m = k + 1; m < A.mt; ++m)
        if (A.local(m, n))
          g->add(A.off(m, n), A.rows(m), A.cols(n), {KPair{(long long)(m - k) * mb, (long long)n * (long long)st, kmin, 0}},
                 0);
    if (g->empty()) continue;
    if (!g->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      return g->launch(prec, NOTRANS, NOTRANS, m_one, pvb, mp, us, mb, one, a, ld, s);
    }, {prev});
  }
  return true;
}

// Row-interchange scratch for the rows of B (relative pivots, net move lists, B's tile offset tables): the
// laswp of getrs and of laswp itself
bool row_swap_scratch(NatProgram& P, NatDesc& B, int blk, LuScratch& S) {
  S.piv = dev_alloc(sizeof(int) * (blk + 16), true);
  S.mdst = dev_alloc(sizeof(int) * 2 * (blk + 16), true);
  S.msrc = dev_alloc(sizeof(int) * 2 * (blk + 16), true);
  S.mcnt = dev_alloc(64, true);
  std::vector<long long> ro(B.mt), co(B.nt);
  std::vector<int> nc(B.nt);
  for (int m = 0; m < B.mt; ++m) ro[m] = B.off(m, 0);
  for (int n = 0; n < B.nt; ++n) {
    co[n] = B.off(0, n);
    nc[n] = B.cols(n);
  }
  S.rowoff = dev_upload(ro);
  S.coloff = dev_upload(co);
  S.ncols = dev_upload(nc);
  for (const DevPtr& d : {S.piv, S.mdst, S.msrc, S.mcnt, S.rowoff, S.coloff, S.ncols}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  return true;
}

// the interchanges ipg[r0 .. r0 + kmin) (global, 1-based, sequential) on the rows of B (inverse: undone)
int add_swap_block(NatProgram& P, NatDesc& B, const LuScratch& S, const int* ipg, int r0, int kmin, bool inverse,
                   int prev) {
  int* piv = (int*)S.piv->p;
  prev = P.task(1, [=](hipStream_t s) { return dpl_ipiv_shift(ipg + r0, piv, kmin, -(r0 + 1), s); }, {prev});
  return add_row_moves(P, B, S, S.rowoff, S.coloff, S.ncols, r0, kmin, inverse, prev);
}

// op(A) X = B with A = P L U from add_getrf (reference getrs: laswp + two TRSM, or the transposed order)
bool add_getrs(NatProgram& P, int trans, NatDesc& A, NatDesc& IP, NatDesc& B, int& last) {
  const int kt = std::min(A.mt, A.nt);
  LuScratch S;
  if (!row_swap_scratch(P, B, std::max(A.mb, A.nb), S)) return false;
  const int* ipg = (const int*)IP.data;
  const Scalar one(B.prec, 1.0);
  int prev = last;
  auto swaps = [&](int k, bool inverse) {
    const int r0 = k * A.mb, kmin = std::min(A.m - r0, A.cols(k));
    prev = add_swap_block(P, B, S, ipg, r0, kmin, inverse, prev);
  };
  auto solve = [&](int uplo, int tr, int diag) {
    if (!add_trsm(P, LEFT, uplo, tr, diag, one, A, B, 1, prev)) return false;
    prev = last_on(P, 1);
    return true;
  };
  if (trans == NOTRANS) {
    for (int k = 0; k < kt; ++k) swaps(k, false);
    if (!solve(LOWER, NOTRANS, UNIT) || !solve(UPPER, NOTRANS, NONUNIT)) return false;
  } else {
    if (!solve(UPPER, trans, NONUNIT) || !solve(LOWER, trans, UNIT)) return false;
    for (int k = kt - 1; k >= 0; --k) swaps(k, true);
  }
  last = prev;
  return true;
}

bool lu_conform(const NatDesc* A, const NatDesc* IP) {
  return A && IP && A->mb == A->nb && A->mb <= 512 && IP->prec == P_I && IP->m == 1 && IP->lld == 1 &&
         IP->n >= std::min(A->m, A->n);
}

}  // namespace

// A := P A with the interchanges of IPIV (1-based, sequential; dplasma_zlaswp): inc > 0 in order, inc < 0
// undone in reverse order -- blocks of A's tile height on the device row-move kernels (one process)
NatProgram* nat_laswp(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dIP, int inc) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "laswp: descriptors of another context or precision");
  if (c->dist()) return fail(nullptr, "laswp: one process only on a native context");
  if (IP->prec != P_I || IP->m != 1 || IP->lld != 1 || A->mb > 512)
    return fail(nullptr, "laswp: IPIV must be a 1 x n int descriptor, A tiles of at most 512 rows");
  NatProgram* P = new_program(c, "laswp", false);
  LuScratch S;
  if (!row_swap_scratch(*P, *A, A->mb, S)) return fail(P, "laswp: device allocation failed");
  const int np = std::min(IP->n, A->m), nblk = (np + A->mb - 1) / A->mb;
  const int* ipg = (const int*)IP->data;
  int prev = -1;
  for (int q = 0; q < nblk; ++q) {
    const int k = inc > 0 ? q : nblk - 1 - q;
    const int r0 = k * A->mb, kmin = std::min(np - r0, A->mb);
    prev = add_swap_block(*P, *A, S, ipg, r0, kmin, inc < 0, prev);
  }
  return P;
}

// B := L^-1 P B with the getrf_1d factors (dplasma_ztrsmpl_ptgpanel; models/lu.py trsmpl_ptgpanel): the
// forward interchanges of getrs and its unit-lower TRSM, no upper solve
NatProgram* nat_trsmpl_ptgpanel(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dIP,
                                dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "trsmpl_ptgpanel: descriptors of another context or precision (one process)");
  if (!lu_conform(A, IP) || A->m != A->n || B->m != A->n || B->mb != A->mb)
    return fail(nullptr, "trsmpl_ptgpanel: operands do not conform");
  NatProgram* P = new_program(c, "trsmpl_ptgpanel", false);
  LuScratch S;
  if (!row_swap_scratch(*P, *B, A->mb, S)) return fail(P, "trsmpl_ptgpanel: device allocation failed");
  const int* ipg = (const int*)IP->data;
  int prev = -1;
  for (int k = 0; k < std::min(A->mt, A->nt); ++k) {
    const int r0 = k * A->mb, kmin = std::min(A->m - r0, A->cols(k));
    prev = add_swap_block(*P, *B, S, ipg, r0, kmin, false, prev);
  }
  if (!add_trsm(*P, LEFT, LOWER, NOTRANS, UNIT, Scalar(prec, 1.0), *A, *B, 1, prev))
    return fail(P, "trsmpl_ptgpanel: device allocation failed");
  return P;
}

// The diagonal scalings of the LDL^H family (models/ldl.py; reference src/ztrdsm.jdf, src/ztrmdm.jdf), one
// dpl_diag_scale launch each: trdsm B := D^-1 B (row i of tile (k, n) divided by D(i, i) of A's tile (k, k));
// trmdm: the strictly lower part of A := L D^-1 (column j of tile (m, k), m >= k, divided by D(j, j)).  D
// itself is never written, so every tile reads it in the same launch.
static NatProgram* diag_scale(NatCtx* c, int prec, const char* name, NatDesc& A, NatDesc& B, bool trmdm) {
  std::vector<TileItem> it;
  int mm = 0, nn = 0;
  auto add = [&](int k, int m, int n) {
    it.push_back(TileItem{A.off(k, k), B.off(m, n), B.rows(m), B.cols(n), m * B.mb, n * B.nb});
    mm = std::max(mm, B.rows(m));
    nn = std::max(nn, B.cols(n));
  };
  if (trmdm) {
    for (int k = 0; k < std::min(A.mt, A.nt); ++k)
      for (int m = k; m < A.mt; ++m) add(k, m, k);
  } else {
    for (int k = 0; k < B.mt; ++k)
      for (int n = 0; n < B.nt; ++n) add(k, k, n);
  }
  NatProgram* P = new_program(c, name, false);
  if (it.empty()) return P;
  DevPtr d = dev_upload(it);
  if (!d) return fail(P, "diagonal scaling: device allocation failed");
  P->keep.push_back(d);
  const int n = (int)it.size(), part = trmdm ? 3 : 0, lda = A.lld, ldb = B.lld;
  const char* a = A.data;
  char* b = B.data;
  P->task(1, [=](hipStream_t s) {
    return dpl_diag_scale(prec, part, trmdm ? 1 : 0, n, d->p, mm, nn, a, lda, b, ldb, s);
  }, {});
  return P;
}

NatProgram* nat_trdsm(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, B}, prec)) return fail(nullptr, "trdsm: descriptors of another context or precision (one process)");
  if (A->mb != A->nb || B->mb != A->mb || A->m < B->m || A->n < B->m)
    return fail(nullptr, "trdsm: operands do not conform");
  return diag_scale(c, prec, "trdsm", *A, *B, false);
}

NatProgram* nat_trmdm(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {A}, prec)) return fail(nullptr, "trmdm: a descriptor of another context or precision (one process)");
  if (A->mb != A->nb) return fail(nullptr, "trmdm: square tiles");
  return diag_scale(c, prec, "trmdm", *A, *A, true);
}

// LDL^H without pivoting (dplasma_zhetrf; models/ldl.py hetrf_New; reference src/zhetrf.jdf), one process.  Step
// k: the Hermitian diagonal tile is completed from its lower triangle into a scratch tile and factored by the
// no-pivot LU recursion (U = D L^H); its lower triangle (L_kk, D_k) goes back to A(k, k).  The column below is
// solved against L_kk^H (giving L D), kept as W, divided by D, and the trailing lower triangle is updated
// A(m, n) -= W(m, k) L(n, k)^H by one batched MFMA GEMM (diagonal tiles masked to their lower part).
NatProgram* nat_hetrf(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {A}, prec)) return fail(nullptr, "hetrf: a descriptor of another context or precision (one process)");
  if (A->mb != A->nb || A->m != A->n || A->mb > 512) return fail(nullptr, "hetrf: a square matrix of square tiles <= 512");
  NatProgram* P = new_program(c, "hetrf", true);
  LuScratch S;
  DevPtr dt = dev_alloc((size_t)A->nb * A->nb * A->es, false);
  if (!P->info || !dt || !lu_scratch(*P, *A, S)) return fail(P, "hetrf: device allocation failed");
  P->keep.push_back(dt);
  const int ct = (prec == P_C || prec == P_Z) ? CONJTRANS : TRANS;
  const int mb = A->mb, ld = A->lld;
  char* a = A->data;
  char* t = (char*)dt->p;
  char* w = (char*)S.pv->p;
  int* info = (int*)P->info->p;
  const Scalar one(prec, 1.0), m_one(prec, -1.0), zero(prec, 0.0);
  int prev = -1;
  for (int k = 0; k < A->mt; ++k) {
    const int kb = A->cols(k), r0 = k * mb;
    auto in = std::make_shared<MapBatch>(), out = std::make_shared<MapBatch>();
    in->it.push_back(TileItem{A->off(k, k), 0, kb, kb, r0, r0});
    out->it.push_back(TileItem{0, A->off(k, k), kb, kb, r0, r0});
    in->mm = in->nn = out->mm = out->nn = kb;
    if (!in->upload(*P) || !out->upload(*P)) return fail(P, "hetrf: device allocation failed");
    prev = P->task(1, [=](hipStream_t s) {   // lower triangle, then strictly upper := (strictly lower)^H
      int e = dpl_geadd(prec, 1, NOTRANS, 1, in->items(), kb, kb, one.ptr(), a, ld, zero.ptr(), t, kb, 1, s);
      return e ? e : dpl_geadd(prec, 4, ct, 1, in->items(), kb, kb, one.ptr(), a, ld, zero.ptr(), t, kb, 1, s);
    }, {prev});
    prev = add_panel_lu(*P, prec, t, kb, kb, 0, kb, S, info, r0, prev, false);
    if (prev < 0) return fail(P, "hetrf: device allocation failed");
    prev = P->task(1, [=](hipStream_t s) {
      return dpl_geadd(prec, 1, NOTRANS, 1, out->items(), kb, kb, one.ptr(), t, kb, zero.ptr(), a, ld, 1, s);
    }, {prev});
    if (k + 1 >= A->mt) continue;
    const int ldw = A->m - (k + 1) * mb;
    auto tr = std::make_shared<Trsm1>();
    auto keep = std::make_shared<MapBatch>(), sc = std::make_shared<MapBatch>();
    auto g = std::make_shared<Gemm>();
    for (int m = k + 1; m < A->mt; ++m) {
      tr->add(A->off(m, k), A->rows(m), kb);
      keep->it.push_back(TileItem{A->off(m, k), (long long)(m - k - 1) * mb, A->rows(m), kb, 0, 0});
      sc->it.push_back(TileItem{A->off(k, k), A->off(m, k), A->rows(m), kb, m * mb, r0});
      keep->mm = sc->mm = std::max(keep->mm, A->rows(m));
      for (int n = k + 1; n <= m; ++n)
        g->add(A->off(m, n), A->rows(m), A->cols(n), {KPair{(long long)(m - k - 1) * mb, A->off(n, k), kb, 0}},
               m == n ? 1 : 0);
    }
    keep->nn = sc->nn = kb;
    if (!tr->upload(*P, prec, RIGHT) || !keep->upload(*P) || !sc->upload(*P) || !g->upload(*P))
      return fail(P, "hetrf: device allocation failed");
    prev = P->task(1, [=](hipStream_t s) {   // A(m, k) := A(m, k) L_kk^-H = L(m, k) D_k
      return tr->launch(prec, RIGHT, LOWER, ct, UNIT, one, t, kb, a, ld, s);
    }, {prev});
    prev = P->task(1, [=](hipStream_t s) {   // W := L D; A(m, k) := L(m, k)
      int e = dpl_geadd(prec, 0, NOTRANS, keep->n(), keep->items(), keep->mm, keep->nn, one.ptr(), a, ld, zero.ptr(),
                        w, ldw, 1, s);
      return e ? e : dpl_diag_scale(prec, 0, 1, sc->n(), sc->items(), sc->mm, sc->nn, a, ld, a, ld, s);
    }, {prev});
    prev = P->task(1, [=](hipStream_t s) {
      return g->launch(prec, NOTRANS, ct, m_one, w, ldw, a, ld, one, a, ld, s);
    }, {prev});
  }
  return P;
}

// x := (L D L^H)^-1 b with the hetrf factors (dplasma_zhetrs; models/ldl.py hetrs): two unit-lower TRSMs around
// trdsm; with a butterfly (hebut's U_but_vec, level > 0) x := U (L D L^H)^-1 U^T b
static NatProgram* hetrs_solve(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, B}, prec)) return fail(nullptr, "hetrs: descriptors of another context or precision (one process)");
  if (uplo != LOWER || A->mb != A->nb || A->m != A->n || B->m != A->n || B->mb != A->mb)
    return fail(nullptr, "hetrs: operands do not conform (lower factors, square tiles)");
  const int ct = (prec == P_C || prec == P_Z) ? CONJTRANS : TRANS;
  NatProgram* P = new_program(c, "hetrs", false);
  const Scalar one(prec, 1.0);
  std::vector<TileItem> it;
  int mm = 0, nn = 0;
  for (int k = 0; k < B->mt; ++k)
    for (int n = 0; n < B->nt; ++n) {
      it.push_back(TileItem{A->off(k, k), B->off(k, n), B->rows(k), B->cols(n), k * B->mb, n * B->nb});
      mm = std::max(mm, B->rows(k));
      nn = std::max(nn, B->cols(n));
    }
  DevPtr d = dev_upload(it);
  if (!d || !add_trsm(*P, LEFT, LOWER, NOTRANS, UNIT, one, *A, *B, 1, -1)) return fail(P, "hetrs: device allocation failed");
  P->keep.push_back(d);
  const int n = (int)it.size(), lda = A->lld, ldb = B->lld;
  const char* a = A->data;
  char* b = B->data;
  const int t = P->task(1, [=](hipStream_t s) {
    return dpl_diag_scale(prec, 0, 0, n, d->p, mm, nn, a, lda, b, ldb, s);
  }, {last_on(*P, 1)});
  if (!add_trsm(*P, LEFT, LOWER, ct, UNIT, one, *A, *B, 1, t)) return fail(P, "hetrs: device allocation failed");
  return P;
}

int nat_hetrs(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA, dplasma_desc_t* dB, const void* U_but_vec,
              int level) {
  int nat_gebmm(dplasma_context_t*, int, dplasma_desc_t*, const void*, int, int);
  const bool but = U_but_vec && level > 0;
  const int ct = (prec == P_C || prec == P_Z) ? CONJTRANS : TRANS;
  if (but)
    if (int rc = nat_gebmm(ctx, prec, dB, U_but_vec, level, ct)) return rc;
  if (int rc = nat_execute(ctx, hetrs_solve(ctx, prec, uplo, dA, dB))) return rc;
  return but ? nat_gebmm(ctx, prec, dB, U_but_vec, level, NOTRANS) : 0;
}

// ----------------------------------------------------------------------------- random butterflies (RBT)
// models/ldl.py gebmm / gebut / hebut; reference src/zhebut.jdf, zgebut.jdf, zgebmm.jdf.  On a native context the
// butterfly is a HOST array of levels x n values of A's precision (row l = the random diagonal R of level l,
// entries exp(u / 10), u the plrnt values of seed 3872), as hebut returns it (malloc; the caller frees it).
// Level l is block diagonal with 2^l butterflies W = 1/sqrt(2) [R0 R1; R0 -R1] of order n / 2^l; each level is
// one element-wise device pass (dpl_butterfly).  One process.
static double but_val(const void* U, int prec, size_t e) {
  switch (prec) {
    case P_S: return ((const float*)U)[e];
    case P_D: return ((const double*)U)[e];
    case P_C: return ((const float*)U)[2 * e];
    default: return ((const double*)U)[2 * e];
  }
}

// A := B_l A (side LEFT) or A B_l (RIGHT), B_l transposed when tr: one element-wise pass over A on the device
// (csrc/kernels/butterfly.hip, O(m n); the reference's segment updates, src/cores/core_zhebut.c:21-46)
static int but_apply(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, const void* U, int l, bool tr, int side) {
  NatDesc* A = dA->nat;
  const int n = side == LEFT ? A->m : A->n;
  const int size = n >> l;
  if (size < 2) return 0;   // order / 2^l < 2: the level is the identity scaled by nothing -- reject upstream
  std::vector<double> r(n);
  const size_t row = (size_t)l * n;
  for (int e = 0; e < n; ++e) r[e] = but_val(U, prec, row + e);
  DevPtr rd = dev_upload(r);
  if (!rd) return (fail(nullptr, "butterfly: device allocation failed"), -1);
  NatCtx* c = ctx->nat;
  hipStream_t st = c->st[0];
  const int big = 1 << 30;
  const int rc = dpl_butterfly(prec, side, tr ? TRANS : NOTRANS, A->m, A->n, size, (const double*)rd->p, A->data, 0,
                               0, big, big, A->lld, st);
  if (rc != 0) return (fail(nullptr, "butterfly: launch failed"), -1);
  if (hipStreamSynchronize(st) != hipSuccess) return (fail(nullptr, "butterfly: device error"), -1);
  (void)ctx;
  return 0;
}

static bool but_ok(NatCtx* c, int prec, NatDesc* A, int n, const void* U, int level, const char* op) {
  if (!same_ctx(c, {A}, prec)) return (fail(nullptr, std::string(op) + ": a descriptor of another context (one process)"), false);
  if (!U || level < 0 || level > 30 || n % (1 << level))
    return (fail(nullptr, std::string(op) + ": a butterfly vector and an order that is a multiple of 2^level"), false);
  return true;
}

int nat_gebmm(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, const void* U, int level, int trans) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!A || !but_ok(ctx->nat, prec, A, A->m, U, level, "gebmm")) return -1;
  for (int q = 0; q < level; ++q) {   // U A = B_0 (B_1 (... B_{L-1} A)); U^T A = B_{L-1}^T (... B_0^T A)
    const int l = trans == NOTRANS ? level - 1 - q : q;
    if (int rc = but_apply(ctx, prec, dA, U, l, trans != NOTRANS, LEFT)) return rc;
  }
  return 0;
}

int nat_gebut(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, const void* U, int level) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!A || !but_ok(ctx->nat, prec, A, A->n, U, level, "gebut") || A->m != A->n)
    return A ? (fail(nullptr, "gebut: a square matrix"), -1) : -1;
  if (int rc = nat_gebmm(ctx, prec, dA, U, level, TRANS)) return rc;
  for (int l = 0; l < level; ++l)   // (U^T A) U = ((U^T A) B_0) B_1 ...
    if (int rc = but_apply(ctx, prec, dA, U, l, false, RIGHT)) return rc;
  return 0;
}

int nat_hebut(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, void** U_out, int level) {
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!U_out || !A) return (fail(nullptr, "hebut: U_but_ptr and A"), -1);
  if (!same_ctx(ctx->nat, {A}, prec)) return (fail(nullptr, "hebut: a descriptor of another context (one process)"), -1);
  const int n = A->n;
  if (A->m != n || level < 0 || level > 30 || n % (1 << level))
    return (fail(nullptr, "hebut: a square matrix whose order is a multiple of 2^level"), -1);
  // the random diagonals: plrnt values of an (n * level) x 1 real matrix, seed 3872 (ldl.butterfly_vectors)
  const int len = std::max(1, n * level);
  dplasma_desc_t* R = nat_desc(ctx, P_D, std::min(len, 4096), 1, len, 1, 1, 1, nullptr, 0, 1);
  std::vector<double> u(len);
  int rc = R ? nat_execute(ctx, nat_plrnt(ctx, P_D, 0, R, 3872)) : -1;
  if (rc == 0) rc = nat_desc_io(R, u.data(), len, false);
  if (R) nat_desc_free(R), delete R;
  if (rc != 0) return rc;
  void* U = std::calloc((size_t)len, A->es);
  if (!U) return (fail(nullptr, "hebut: host allocation failed"), -1);
  for (int e = 0; e < n * level; ++e) {
    const double v = std::exp(u[e] / 10.0);
    if (prec == P_S || prec == P_C) ((float*)U)[(prec == P_C ? 2 : 1) * e] = (float)v;
    else ((double*)U)[(prec == P_Z ? 2 : 1) * e] = v;
  }
  rc = nat_gebut(ctx, prec, dA, U, level);
  if (rc != 0) {
    std::free(U);
    return rc;
  }
  *U_out = U;
  return 0;
}

// dplasma_zprint (src/zprint.jdf; models/aux.py print_matrix): the uplo part of A tile by tile, in the
// Python layer's format, from a host copy (one process)
int nat_print(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {A}, prec)) return nat_unsupported("print: a descriptor of another context (one process)");
  std::vector<char> h((size_t)std::max(1, A->m) * std::max(1, A->n) * A->es);
  if (nat_desc_io(dA, h.data(), std::max(1, A->m), false) != 0) return -1;
  const bool cplx = prec == P_C || prec == P_Z;
  auto at = [&](long long i, long long j, double& re, double& im) {
    const size_t e = (size_t)(i + j * A->m);
    im = 0.0;
    switch (prec) {
      case P_S: re = ((const float*)h.data())[e]; break;
      case P_D: re = ((const double*)h.data())[e]; break;
      case P_C: re = ((const float*)h.data())[2 * e]; im = ((const float*)h.data())[2 * e + 1]; break;
      default: re = ((const double*)h.data())[2 * e]; im = ((const double*)h.data())[2 * e + 1]; break;
    }
  };
  for (int n = 0; n < A->nt; ++n)
    for (int m = 0; m < A->mt; ++m) {
      if ((uplo == LOWER && m < n) || (uplo == UPPER && m > n)) continue;
      std::printf("A(%d,%d) [%dx%d]\n", m, n, A->rows(m), A->cols(n));
      for (int i = 0; i < A->rows(m); ++i) {
        std::printf(" ");
        for (int j = 0; j < A->cols(n); ++j) {
          double re, im;
          at((long long)m * A->mb + i, (long long)n * A->nb + j, re, im);
          if (cplx)
            std::printf(" %.6g%+.6gj", re, im);
          else
            std::printf(" % .6e", re);
        }
        std::printf("\n");
      }
    }
  std::fflush(stdout);
  return 0;
}

NatProgram* nat_getrf_1d(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dIP) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "getrf_1d: descriptors of another context or precision");
  if (!lu_conform(A, IP)) return fail(nullptr, "getrf_1d: square tiles <= 512 and an IPIV of min(M, N) entries");
  NatProgram* P = new_program(c, "getrf_1d", true);
  int last = -1;
  if (!P->info || !(c->dist() ? add_getrf_dist(*P, *A, *IP) : add_getrf(*P, *A, IP, last)))
    return fail(P, "getrf_1d: device allocation failed");
  return P;
}

NatProgram* nat_getrs(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* dA, dplasma_desc_t* dIP,
                      dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "getrs: descriptors of another context or precision");
  if (!lu_conform(A, IP) || A->m != A->n || B->m != A->n || B->mb != A->mb)
    return fail(nullptr, "getrs: operands do not conform");
  if (c->dist() && trans != NOTRANS) return fail(nullptr, "getrs: a multi-process context solves A X = B only");
  NatProgram* P = new_program(c, "getrs", false);
  int last = -1;
  if (!(c->dist() ? add_getrs_dist(*P, *A, *IP, *B) : add_getrs(*P, trans, *A, *IP, *B, last)))
    return fail(P, "getrs: device allocation failed");
  return P;
}

NatProgram* nat_gesv_1d(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dIP,
                        dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "gesv_1d: descriptors of another context or precision");
  if (!lu_conform(A, IP) || A->m != A->n || B->m != A->n || B->mb != A->mb)
    return fail(nullptr, "gesv_1d: operands do not conform");
  NatProgram* P = new_program(c, "gesv_1d", true);
  int last = -1;
  const bool ok = c->dist() ? add_getrf_dist(*P, *A, *IP) && add_getrs_dist(*P, *A, *IP, *B)
                            : add_getrf(*P, *A, IP, last) && add_getrs(*P, NOTRANS, *A, *IP, *B, last);
  if (!P->info || !ok) return fail(P, "gesv_1d: device allocation failed");
  return P;
}

// LU without pivoting (models/lu.py getrf_nopiv; reference src/zgetrf_nopiv.jdf): one process
NatProgram* nat_getrf_nopiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {A}, prec)) return fail(nullptr, "getrf_nopiv: a descriptor of another context or precision");
  if (A->mb != A->nb || A->mb > 512) return fail(nullptr, "getrf_nopiv: square tiles <= 512");
  NatProgram* P = new_program(c, "getrf_nopiv", true);
  int last = -1;
  if (!P->info || !add_getrf(*P, *A, nullptr, last)) return fail(P, "getrf_nopiv: device allocation failed");
  return P;
}

// ----------------------------------------------------------------------------- LU, incremental pivoting
// The tile algorithm of src/zgetrf_incpiv.jdf (GETRF(k) -> GESSM(k, n) -> TSTRF(k, m) -> SSSSM(k, m, n)) on the
// tile kernels of csrc/kernels/lu_incpiv.hip, one batched launch per task class and step (GESSM over the
// row, SSSSM over the row for each m): TSTRF(k, m) on the panel stream, SSSSM(k, m, *) on the update stream
// (TSTRF(k, m+1) overlaps SSSSM(k, m, *)).  L: (MT*IB) x N of IB x NB tiles, IPIV: M x NT of MB x 1 tiles
// (tests/testing_zgetrf_incpiv.c:51-62).  One process.
namespace {

struct IncItem {   // = lu_incpiv.hip LuItem (96 bytes)
  long long p0, p1, p2, p3;
  int ld0, ld1, ld2, ld3;
  int m, n, k, pad;
  long long p4, p5;
  int ld4, ld5, aux0, aux1;
};
static_assert(sizeof(IncItem) == 96, "LuItem layout");

bool incpiv_conform(const NatDesc* A, const NatDesc* L, const NatDesc* IP) {
  return A && L && IP && A->mb == A->nb && A->nb <= 256 && L->mb >= 1 && L->mb <= 32 && L->nb == A->nb &&
         L->mt >= A->mt && L->nt >= A->nt && IP->prec == P_I && IP->mb == A->mb && IP->m >= A->m && IP->n >= A->nt;
}

struct IncBatch {
  std::vector<IncItem> it;
  int max_m = 0, max_n = 0;
  DevPtr d;
  void add(const IncItem& x) {
    it.push_back(x);
    max_m = std::max(max_m, x.m);
    max_n = std::max(max_n, x.n);
  }
  bool upload(NatProgram& P) {
    if (it.empty()) return true;
    d = dev_upload(it);
    if (!d) return false;
    P.keep.push_back(d);
    return true;
  }
};

// B := L^-1 P B with the factors of add_getrf_incpiv (GESSM on block row k, SSSSM down the rows); stream 1
bool add_trsmpl_incpiv(NatProgram& P, NatDesc& A, NatDesc& L, NatDesc& IP, NatDesc& B, int& last) {
  const int prec = A.prec, es = A.es, ib = L.mb, kt = std::min(A.mt, A.nt);
  auto ad = [&](NatDesc& D, int i, int j) { return (long long)(D.data + D.off(i, j) * D.es); };
  int prev = last;
  for (int k = 0; k < kt; ++k) {
    auto g = std::make_shared<IncBatch>();
    for (int n = 0; n < B.nt; ++n)
      g->add(IncItem{0, ad(B, k, n), ad(A, k, k), ad(IP, k, k), 0, B.lld, A.lld, 0, B.rows(k), B.cols(n),
                     std::min(A.rows(k), A.cols(k)), 0, 0, 0, 0, 0, 0, 0});
    if (!g->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) { return dpl_gessm(prec, (int)g->it.size(), g->d->p, g->max_n, s); }, {prev});
    for (int m = k + 1; m < A.mt; ++m) {
      auto q = std::make_shared<IncBatch>();
      for (int n = 0; n < B.nt; ++n)
        q->add(IncItem{ad(B, k, n), ad(B, m, n), ad(L, m, k), ad(IP, m, k), B.lld, B.lld, L.lld, 0, B.rows(m), B.cols(n),
                       A.cols(k), 0, ad(A, m, k), 0, A.lld, 0, 0, 0});
      if (!q->upload(P)) return false;
      const int NB = A.nb;
      prev = P.task(1, [=](hipStream_t s) { return dpl_ssssm(prec, (int)q->it.size(), q->d->p, q->max_n, ib, NB, s); },
                    {prev});
    }
  }
  (void)es;
  last = prev;
  return true;
}

bool add_getrf_incpiv(NatProgram& P, NatDesc& A, NatDesc& L, NatDesc& IP, int& last) {
  const int prec = A.prec, ib = L.mb, NB = A.nb, kt = std::min(A.mt, A.nt);
  int* info = (int*)P.info->p;
  auto ad = [&](NatDesc& D, int i, int j) { return (long long)(D.data + D.off(i, j) * D.es); };
  int prev_pan = last, prev_upd = last;
  for (int k = 0; k < kt; ++k) {
    auto gf = std::make_shared<IncBatch>();
    gf->add(IncItem{0, ad(A, k, k), 0, ad(IP, k, k), 0, A.lld, 0, 0, A.rows(k), A.cols(k), k * A.nb, 0, 0, 0, 0, 0, 0, 0});
    if (!gf->upload(P)) return false;
    // the diagonal tile is final once every SSSSM of step k-1 has run (update stream)
    int pan = P.task(0, [=](hipStream_t s) { return dpl_getrf_tile(prec, 1, gf->d->p, info, s); }, {prev_pan, prev_upd});
    int upd = prev_upd;
    if (k + 1 < A.nt) {
      auto g = std::make_shared<IncBatch>();
      for (int n = k + 1; n < A.nt; ++n)
        g->add(IncItem{0, ad(A, k, n), ad(A, k, k), ad(IP, k, k), 0, A.lld, A.lld, 0, A.rows(k), A.cols(n),
                       std::min(A.rows(k), A.cols(k)), 0, 0, 0, 0, 0, 0, 0});
      if (!g->upload(P)) return false;
      upd = P.task(1, [=](hipStream_t s) { return dpl_gessm(prec, (int)g->it.size(), g->d->p, g->max_n, s); }, {pan, upd});
    }
    for (int m = k + 1; m < A.mt; ++m) {
      auto t = std::make_shared<IncBatch>();
      t->add(IncItem{ad(A, k, k), ad(A, m, k), ad(L, m, k), ad(IP, m, k), A.lld, A.lld, L.lld, 0, A.rows(m), A.cols(k),
                     k * A.nb, 0, 0, 0, 0, 0, 0, 0});
      if (!t->upload(P)) return false;
      const int mm = t->max_m;
      // TSTRF(k, m) needs only TSTRF(k, m-1) (the U tile, panel stream order); SSSSM(k, m, *) reads its L / IPIV
      pan = P.task(0, [=](hipStream_t s) { return dpl_tstrf(prec, 1, t->d->p, ib, NB, mm, info, s); }, {pan});
      if (k + 1 < A.nt) {
        auto q = std::make_shared<IncBatch>();
        for (int n = k + 1; n < A.nt; ++n)
          q->add(IncItem{ad(A, k, n), ad(A, m, n), ad(L, m, k), ad(IP, m, k), A.lld, A.lld, L.lld, 0, A.rows(m), A.cols(n),
                         A.cols(k), 0, ad(A, m, k), 0, A.lld, 0, 0, 0});
        if (!q->upload(P)) return false;
        upd = P.task(1, [=](hipStream_t s) { return dpl_ssssm(prec, (int)q->it.size(), q->d->p, q->max_n, ib, NB, s); },
                     {pan, upd});
      }
    }
    prev_pan = pan;
    prev_upd = upd;
  }
  last = P.task(1, [](hipStream_t) { return 0; }, {prev_pan, prev_upd});
  return true;
}

}  // namespace

NatProgram* nat_getrf_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dL,
                             dplasma_desc_t* dIP) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *L = dL ? dL->nat : nullptr, *IP = dIP ? dIP->nat : nullptr;
  if (!same_ctx(c, {A, L}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "getrf_incpiv: descriptors of another context or precision");
  if (!incpiv_conform(A, L, IP))
    return fail(nullptr, "getrf_incpiv: square tiles <= 256, L of (IB <= 32) x NB tiles, IPIV of MB x 1 tiles");
  NatProgram* P = new_program(c, "getrf_incpiv", true);
  int last = -1;
  if (!P->info || !add_getrf_incpiv(*P, *A, *L, *IP, last)) return fail(P, "getrf_incpiv: device allocation failed");
  return P;
}

static bool incpiv_solve_ok(const NatDesc* A, const NatDesc* B) {
  return B && A->m == A->n && B->m == A->m && B->mb == A->mb;
}

NatProgram* nat_trsmpl_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dL,
                              dplasma_desc_t* dIP, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *L = dL ? dL->nat : nullptr, *IP = dIP ? dIP->nat : nullptr,
          *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, L, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "trsmpl_incpiv: descriptors of another context or precision");
  if (!incpiv_conform(A, L, IP) || !incpiv_solve_ok(A, B)) return fail(nullptr, "trsmpl_incpiv: operands do not conform");
  NatProgram* P = new_program(c, "trsmpl_incpiv", false);
  int last = -1;
  if (!add_trsmpl_incpiv(*P, *A, *L, *IP, *B, last)) return fail(P, "trsmpl_incpiv: device allocation failed");
  return P;
}

// op(A) X = B, NoTrans (the reference getrs_incpiv: trsmpl + the upper solve)
NatProgram* nat_getrs_incpiv(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* dA, dplasma_desc_t* dL,
                             dplasma_desc_t* dIP, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *L = dL ? dL->nat : nullptr, *IP = dIP ? dIP->nat : nullptr,
          *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, L, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "getrs_incpiv: descriptors of another context or precision");
  if (trans != NOTRANS) return fail(nullptr, "getrs_incpiv: NoTrans only (as the reference)");
  if (!incpiv_conform(A, L, IP) || !incpiv_solve_ok(A, B)) return fail(nullptr, "getrs_incpiv: operands do not conform");
  NatProgram* P = new_program(c, "getrs_incpiv", false);
  int last = -1;
  if (!add_trsmpl_incpiv(*P, *A, *L, *IP, *B, last) ||
      !add_trsm(*P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(prec, 1.0), *A, *B, 1, last))
    return fail(P, "getrs_incpiv: device allocation failed");
  return P;
}

NatProgram* nat_gesv_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dL,
                            dplasma_desc_t* dIP, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *L = dL ? dL->nat : nullptr, *IP = dIP ? dIP->nat : nullptr,
          *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, L, B}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "gesv_incpiv: descriptors of another context or precision");
  if (!incpiv_conform(A, L, IP) || !incpiv_solve_ok(A, B)) return fail(nullptr, "gesv_incpiv: operands do not conform");
  NatProgram* P = new_program(c, "gesv_incpiv", true);
  int last = -1;
  if (!P->info || !add_getrf_incpiv(*P, *A, *L, *IP, last) || !add_trsmpl_incpiv(*P, *A, *L, *IP, *B, last) ||
      !add_trsm(*P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(prec, 1.0), *A, *B, 1, last))
    return fail(P, "gesv_incpiv: device allocation failed");
  return P;
}

dplasma_desc_t* nat_desc_int(dplasma_context_t* ctx, int mb, int nb, int m, int n) {
  return nat_desc(ctx, P_I, mb, nb, m, n, 1, 1, nullptr, 0, 1);
}

// ----------------------------------------------------------------------------- QR (flat TS tree)
// models/qr_panel.py's single-domain schedule in C++: panel k = rows k*mb.. of tile column k, one persistent
// Householder launch (dpl_qr_panel, in place in the LAPACK-layout matrix, explicit V in a parity buffer, the
// full T into the T descriptor's side buffer); NEXT (column k+1) on the panel stream, REST on the update
// stream, both  C -= V op(T) (V^H C)  as three batched MFMA GEMM launches.
namespace {

struct QrWork {
  DevPtr V[2], ws, W[2], W2[2];
  int ldv = 0;
};

bool qr_conform(const NatDesc* A, const NatDesc* T) {
  return A && T && A->mb == A->nb && A->nb <= 256 && T->nb == A->nb && T->mt >= A->mt && T->nt >= A->nt &&
         T->mb >= 1 && T->mb <= A->nb;
}

// C(r0 tile.., cols) := op(Q_k) C, Q_k = I - V T V^H (left; qt: T^H); V rows = rows r0*mb.. of C (M rows)
bool add_left_apply(NatProgram& P, int prec, NatDesc& C, int r0, int M, int kf, char* V, int ldv, char* Tk, int ldt,
                    bool qt, char* W, char* W2, const std::vector<int>& cols, int stream, int dep, int& out) {
  out = dep;
  if (cols.empty() || kf <= 0) return true;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  long long wo = 0;
  for (int j : cols) {
    const int nj = C.cols(j);
    g1->add(wo, kf, nj, {KPair{0, C.off(r0, j), M, 0}}, 0);
    g2->add(wo, kf, nj, {KPair{0, wo, kf, 0}}, 0);
    for (int i = r0; i < C.mt; ++i) g3->add(C.off(i, j), C.rows(i), nj, {KPair{(long long)(i - r0) * C.mb, wo, kf, 0}}, 0);
    wo += (long long)kf * nj;
  }
  if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return false;
  char* c = C.data;
  const int ldc = C.lld;
  int t = P.task(stream, [=](hipStream_t s) {
    return g1->launch(prec, CONJTRANS, NOTRANS, one, V, ldv, c, ldc, zero, W, kf, s);
  }, {dep});
  t = P.task(stream, [=](hipStream_t s) {
    return g2->launch(prec, qt ? CONJTRANS : NOTRANS, NOTRANS, one, Tk, ldt, W, kf, zero, W2, kf, s);
  }, {t});
  out = P.task(stream, [=](hipStream_t s) {
    return g3->launch(prec, NOTRANS, NOTRANS, m_one, V, ldv, W2, kf, one, c, ldc, s);
  }, {t});
  return true;
}

// C := C op(Q_k) (right): W = C(:, r0..) V, W2 = W op(T), C(:, r0..) -= W2 V^H   (C.nb == the panel's mb)
bool add_right_apply(NatProgram& P, int prec, NatDesc& C, int r0, int M, int kf, char* V, int ldv, char* Tk, int ldt,
                     bool qt, char* W, char* W2, int ldw, int stream, int dep, int& out) {
  out = dep;
  if (kf <= 0 || C.mt == 0) return true;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  for (int i = 0; i < C.mt; ++i) {
    const long long wo = (long long)i * C.mb;
    g1->add(wo, C.rows(i), kf, {KPair{C.off(i, r0), 0, M, 0}}, 0);
    g2->add(wo, C.rows(i), kf, {KPair{wo, 0, kf, 0}}, 0);
    for (int j = r0; j < C.nt; ++j) g3->add(C.off(i, j), C.rows(i), C.cols(j), {KPair{wo, (long long)(j - r0) * C.nb, kf, 0}}, 0);
  }
  if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return false;
  char* c = C.data;
  const int ldc = C.lld;
  int t = P.task(stream, [=](hipStream_t s) {
    return g1->launch(prec, NOTRANS, NOTRANS, one, c, ldc, V, ldv, zero, W, ldw, s);
  }, {dep});
  t = P.task(stream, [=](hipStream_t s) {
    return g2->launch(prec, NOTRANS, qt ? CONJTRANS : NOTRANS, one, W, ldw, Tk, ldt, zero, W2, ldw, s);
  }, {t});
  out = P.task(stream, [=](hipStream_t s) {
    return g3->launch(prec, NOTRANS, CONJTRANS, m_one, W2, ldw, V, ldv, one, c, ldc, s);
  }, {t});
  return true;
}

bool add_geqrf(NatProgram& P, NatDesc& A, NatDesc& T, int& last) {
  const int prec = A.prec, nb = A.nb, es = A.es;
  const int kt = std::min(A.mt, A.nt);
  QrWork Wk;
  Wk.ldv = std::max(16, (A.m + 15) / 16 * 16);
  const size_t wlen = (size_t)nb * std::max(1, A.n);
  for (int b = 0; b < 2; ++b) {
    Wk.V[b] = dev_alloc((size_t)Wk.ldv * nb * es, true);
    Wk.W[b] = dev_alloc(wlen * es, false);
    Wk.W2[b] = dev_alloc(wlen * es, false);
  }
  Wk.ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(prec, nb, nb) + 256, true);
  T.fullT = dev_alloc((size_t)std::max(1, kt) * nb * nb * es, true);
  T.fullT_nb = nb;
  T.fullT_kt = kt;
  for (const DevPtr& d : {Wk.V[0], Wk.V[1], Wk.W[0], Wk.W[1], Wk.W2[0], Wk.W2[1], Wk.ws, T.fullT}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  char* a = A.data;
  char* tf = (char*)T.fullT->p;
  char* t = T.data;
  int* info = (int*)P.info->p;
  const int lda = A.lld, ldv = Wk.ldv, ldT = T.lld, ib = T.mb;
  int prev_next = -1, prev_rest = -1, prev_rest2 = -1;
  for (int k = 0; k < kt; ++k) {
    const int M = A.m - k * A.mb, kb = A.cols(k), kf = std::min(M, kb), buf = k & 1;
    char* V = (char*)Wk.V[buf]->p;
    char* Tk = tf + (size_t)k * nb * nb * es;
    char* ws = (char*)Wk.ws->p;
    char* pk = a + A.off(k, k) * es;
    const int pan = P.task(0, [=](hipStream_t s) {
      return dpl_qr_panel(prec, pk, lda, 0, 0, M, kb, kf, V, ldv, Tk, nb, ws, info, s);
    }, {prev_next, prev_rest2});
    // the reference layout: IB x IB diagonal blocks of T into tile T(k, k)
    std::vector<TileItem> ti;
    for (int b0 = 0; b0 < kf; b0 += ib) {
      const int bs = std::min(ib, kf - b0);
      ti.push_back(TileItem{(long long)k * nb * nb + b0 + (long long)b0 * nb, T.off(k, k) + (long long)b0 * ldT, bs, bs, 0, 0});
    }
    auto d_ti = dev_upload(ti);
    if (!d_ti) return false;
    P.keep.push_back(d_ti);
    const int nti = (int)ti.size();
    const Scalar one(prec, 1.0), zero(prec, 0.0);
    int tst = P.task(0, [=](hipStream_t s) {
      return dpl_geadd(prec, 0, NOTRANS, nti, d_ti->p, ib, ib, one.ptr(), tf, nb, zero.ptr(), t, ldT, 1, s);
    }, {pan});
    int nxt = tst, rst = prev_rest;
    std::vector<int> cn, cr;
    for (int j = k + 1; j < A.nt; ++j) (j == k + 1 ? cn : cr).push_back(j);
    if (!add_left_apply(P, prec, A, k, M, kf, V, ldv, Tk, nb, true, (char*)Wk.W[0]->p, (char*)Wk.W2[0]->p, cn, 0,
                        P.task(0, [](hipStream_t) { return 0; }, {tst, prev_rest}), nxt))
      return false;
    if (!cr.empty()) {
      if (!add_left_apply(P, prec, A, k, M, kf, V, ldv, Tk, nb, true, (char*)Wk.W[1]->p, (char*)Wk.W2[1]->p, cr, 1,
                          P.task(1, [](hipStream_t) { return 0; }, {pan, prev_rest}), rst))
        return false;
    }
    prev_rest2 = prev_rest;
    prev_next = nxt;
    prev_rest = rst;
  }
  last = P.task(1, [](hipStream_t) { return 0; }, {prev_next, prev_rest});
  return true;
}

// V of panel k rebuilt from A (unit diagonal, zeros above) into V (ld ldv)
int add_build_v(NatProgram& P, NatDesc& A, int k, char* V, int ldv, int stream, int dep) {
  const int prec = A.prec, kb = A.cols(k);
  std::vector<TileItem> it;
  for (int i = k; i < A.mt; ++i)
    it.push_back(TileItem{A.off(i, k), (long long)(i - k) * A.mb, A.rows(i), kb, (i - k) * A.mb, 0});
  std::vector<TileItem> lt;
  for (const TileItem& x : it) lt.push_back(TileItem{x.b_off, 0, x.m, x.n, x.gi, x.gj});
  auto d_it = dev_upload(it), d_lt = dev_upload(lt);
  if (!d_it || !d_lt) return -2;
  P.keep.push_back(d_it);
  P.keep.push_back(d_lt);
  const int n = (int)it.size(), mb = A.mb, lda = A.lld;
  char* a = A.data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  int t = P.task(stream, [=](hipStream_t s) {
    return dpl_laset(prec, 0, n, d_lt->p, mb, kb, zero.ptr(), one.ptr(), V, ldv, s);
  }, {dep});
  return P.task(stream, [=](hipStream_t s) {   // part 3: strictly below the (stacked) diagonal
    return dpl_geadd(prec, 3, NOTRANS, n, d_it->p, mb, kb, one.ptr(), a, lda, zero.ptr(), V, ldv, 1, s);
  }, {t});
}

// C := op(Q) C (left) or C op(Q) (right) with Q from the native geqrf (A, T)
bool add_unmqr(NatProgram& P, int side, int trans, NatDesc& A, NatDesc& T, NatDesc& C, int& last) {
  const int prec = A.prec, nb = A.nb, es = A.es, kt = std::min(A.mt, A.nt);
  const bool left = side == LEFT, qt = trans != NOTRANS;
  const int ldv = std::max(16, (A.m + 15) / 16 * 16);
  const int ldw = std::max(16, (C.m + 15) / 16 * 16);
  const size_t wlen = left ? (size_t)nb * std::max(1, C.n) : (size_t)ldw * nb;
  DevPtr V = dev_alloc((size_t)ldv * nb * es, true), W = dev_alloc(wlen * es, false), W2 = dev_alloc(wlen * es, false);
  if (!V || !W || !W2) return false;
  for (const DevPtr& d : {V, W, W2}) P.keep.push_back(d);
  char* tf = (char*)T.fullT->p;
  std::vector<int> order;
  // left: Q^H C applies panel 0 first, Q C the last first; right: C Q panel 0 first, C Q^H the last first
  const bool forward = left ? qt : !qt;
  for (int s = 0; s < kt; ++s) order.push_back(forward ? s : kt - 1 - s);
  int prev = last;
  for (int k : order) {
    const int M = A.m - k * A.mb, kf = std::min(M, A.cols(k));
    prev = add_build_v(P, A, k, (char*)V->p, ldv, 1, prev);
    if (prev < -1) return false;
    char* Tk = tf + (size_t)k * nb * nb * es;
    std::vector<int> cols;
    for (int j = 0; j < C.nt; ++j) cols.push_back(j);
    int out = prev;
    bool ok = left ? add_left_apply(P, prec, C, k, M, kf, (char*)V->p, ldv, Tk, nb, qt, (char*)W->p, (char*)W2->p, cols,
                                    1, prev, out)
                   : add_right_apply(P, prec, C, k, M, kf, (char*)V->p, ldv, Tk, nb, qt, (char*)W->p, (char*)W2->p,
                                     ldw, 1, prev, out);
    if (!ok) return false;
    prev = out;
  }
  last = prev;
  return true;
}

// a non-owning view of the leading r x c part of D (same tiling and storage)
std::shared_ptr<NatDesc> lead_view(NatDesc& D, int r, int c) {
  auto v = std::make_shared<NatDesc>();
  v->ctx = D.ctx;
  v->prec = D.prec;
  v->es = D.es;
  v->mb = D.mb;
  v->nb = D.nb;
  v->m = r;
  v->n = c;
  v->mt = (r + D.mb - 1) / D.mb;
  v->nt = (c + D.nb - 1) / D.nb;
  v->lld = D.lld;
  v->data = D.data;
  v->owned = false;
  return v;
}

bool has_fullT(const NatDesc& A, const NatDesc& T) {
  return T.fullT && T.fullT_nb == A.nb && T.fullT_kt >= std::min(A.mt, A.nt);
}

}  // namespace

NatProgram* nat_geqrf(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr;
  if (!same_ctx_dist(c, {A, T}, prec)) return fail(nullptr, "geqrf: descriptors of another context or precision");
  if (!qr_conform(A, T)) return fail(nullptr, "geqrf: square tiles <= 256 and a T of (IB x NB) tiles covering A");
  if (c->dist()) return nat_dist_geqrf(c, *A, *T);
  NatProgram* P = new_program(c, "geqrf", true);
  int last = -1;
  if (!P->info || !add_geqrf(*P, *A, *T, last)) return fail(P, "geqrf: device allocation failed");
  return P;
}

NatProgram* nat_unmqr(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_desc_t* dA, dplasma_desc_t* dT,
                      dplasma_desc_t* dC) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx_dist(c, {A, T, C}, prec)) return fail(nullptr, "unmqr: descriptors of another context or precision");
  if (!qr_conform(A, T) || !has_fullT(*A, *T)) return fail(nullptr, "unmqr: T must come from the native geqrf of A");
  if ((side == LEFT && (C->m != A->m || C->mb != A->mb)) || (side == RIGHT && (C->n != A->m || C->nb != A->mb)))
    return fail(nullptr, "unmqr: C does not conform to Q");
  if (c->dist()) {
    if (side != LEFT) return fail(nullptr, "unmqr: a multi-process context applies Q from the left");
    return nat_dist_unmqr(c, trans, *A, *T, *C);
  }
  NatProgram* P = new_program(c, "unmqr", false);
  int last = -1;
  if (!add_unmqr(*P, side, trans, *A, *T, *C, last)) return fail(P, "unmqr: device allocation failed");
  return P;
}

// Q (M x K) := the first K columns of the orthogonal factor: Q = I(:, :K), then Q := Q_geqrf Q
NatProgram* nat_ungqr(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT, dplasma_desc_t* dQ) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *Q = dQ ? dQ->nat : nullptr;
  if (!same_ctx(c, {A, T, Q}, prec)) return fail(nullptr, "ungqr: descriptors of another context or precision");
  if (!qr_conform(A, T) || !has_fullT(*A, *T) || Q->m != A->m || Q->mb != A->mb || Q->n > A->m)
    return fail(nullptr, "ungqr: T from the native geqrf of A, Q with A's rows");
  NatProgram* P = new_program(c, "ungqr", false);
  std::vector<TileItem> it;
  for (int i = 0; i < Q->mt; ++i)
    for (int j = 0; j < Q->nt; ++j) it.push_back(TileItem{Q->off(i, j), 0, Q->rows(i), Q->cols(j), i * Q->mb, j * Q->nb});
  auto d_it = dev_upload(it);
  if (!d_it) return fail(P, "ungqr: device allocation failed");
  P->keep.push_back(d_it);
  const int n = (int)it.size(), mb = Q->mb, nb = Q->nb, ldq = Q->lld;
  char* q = Q->data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  int last = P->task(1, [=](hipStream_t s) {
    return dpl_laset(prec, 0, n, d_it->p, mb, nb, zero.ptr(), one.ptr(), q, ldq, s);
  }, {});
  if (!add_unmqr(*P, LEFT, NOTRANS, *A, *T, *Q, last)) return fail(P, "ungqr: device allocation failed");
  return P;
}

// X = R^{-1} (Q^H B)(0:N) for a factored M >= N matrix (B's first N rows receive X)
static bool add_geqrs(NatProgram& P, NatDesc& A, NatDesc& T, NatDesc& B, int& last) {
  if (!add_unmqr(P, LEFT, CONJTRANS, A, T, B, last)) return false;
  auto R = lead_view(A, A.n, A.n), X = lead_view(B, A.n, B.n);
  P.wdesc.push_back(R);
  P.wdesc.push_back(X);
  return add_trsm(P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(A.prec, 1.0), *R, *X, 1, last);
}

NatProgram* nat_geqrs(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, T, B}, prec)) return fail(nullptr, "geqrs: descriptors of another context or precision");
  if (!qr_conform(A, T) || !has_fullT(*A, *T) || A->m < A->n || B->m != A->m || B->mb != A->mb)
    return fail(nullptr, "geqrs: T from the native geqrf of an M >= N matrix A, B with A's rows");
  NatProgram* P = new_program(c, "geqrs", false);
  int last = -1;
  if (!add_geqrs(*P, *A, *T, *B, last)) return fail(P, "geqrs: device allocation failed");
  return P;
}

// ----------------------------------------------------------------------------- LQ (flat tree)
// A = L Q is the conjugate transpose of the QR factorization A^H = Q_r R (L = R^H, Q = Q_r^H, the same
// reflectors and T factors; LAPACK's row-stored conj(v) is exactly column v of Q_r conjugate-transposed).
// So the LQ family runs the QR engine above on W = A^H, one process: gelqf transposes A into W, factors W,
// transposes back; unmlq / unglq / gelqs rebuild W from the factored A and apply Q_r with the side and
// the transposition flipped.  The two O(MN) transposes are one launch each beside the O(MN min(M, N))
// factorization.  (models/lq.py is the tile-DAG version; reference src/zgelqf.jdf, zunmlq*.jdf.)
namespace {

// W := op-shaped work matrix of S^H (S.n x S.m, square tiles)
std::shared_ptr<NatDesc> ctrans_desc(NatProgram& P, const NatDesc& S) {
  auto w = std::make_shared<NatDesc>();
  w->ctx = S.ctx;
  w->prec = S.prec;
  w->es = S.es;
  w->mb = S.nb;
  w->nb = S.mb;
  w->m = S.n;
  w->n = S.m;
  w->mt = S.nt;
  w->nt = S.mt;
  w->lm = w->m;
  w->ln = w->n;
  w->lld = std::max(16, (w->m + 15) / 16 * 16);
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)w->lld * std::max(1, w->n) * S.es) != hipSuccess) return nullptr;
  w->data = (char*)p;
  w->owned = true;
  P.wdesc.push_back(w);
  return w;
}

// D := S^H (D is S.n x S.m), on stream 1 after prev
int add_ctrans(NatProgram& P, const NatDesc& S, NatDesc& D, int prev) {
  auto mb = std::make_shared<MapBatch>();
  mb->build(D, UPPERLOWER, &S, CONJTRANS);
  if (!mb->upload(P)) return -2;
  const int prec = S.prec, lds = S.lld, ldd = D.lld;
  const char* s = S.data;
  char* d = D.data;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  return P.task(1, [=](hipStream_t st) {
    return dpl_geadd(prec, 0, CONJTRANS, mb->n(), mb->items(), mb->mm, mb->nn, one.ptr(), s, lds, zero.ptr(), d, ldd,
                     1, st);
  }, {prev});
}

bool lq_conform(const NatDesc* A, const NatDesc* T) {
  const int kt = std::min(A->mt, A->nt);
  return A->mb == A->nb && A->nb <= 256 && T->nb == A->nb && T->mt >= kt && T->nt >= kt && T->mb >= 1 &&
         T->mb <= A->nb;
}

bool add_gelqf(NatProgram& P, NatDesc& A, NatDesc& T, int& last) {
  auto W = ctrans_desc(P, A);
  if (!W) return false;
  last = add_ctrans(P, A, *W, last);
  if (last < -1 || !add_geqrf(P, *W, T, last)) return false;
  last = add_ctrans(P, *W, A, last);
  return last >= -1;
}

// C := op(Q) C or C op(Q) with Q = Q_r^H from the native gelqf of A
bool add_unmlq(NatProgram& P, int side, int trans, NatDesc& A, NatDesc& T, NatDesc& C, int& last) {
  auto W = ctrans_desc(P, A);
  if (!W) return false;
  last = add_ctrans(P, A, *W, last);
  if (last < -1) return false;
  return add_unmqr(P, side, trans == NOTRANS ? CONJTRANS : NOTRANS, *W, T, C, last);
}

bool has_fullT_lq(const NatDesc& A, const NatDesc& T) {
  return T.fullT && T.fullT_nb == A.nb && T.fullT_kt >= std::min(A.mt, A.nt);
}

}  // namespace

NatProgram* nat_gelqf(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr;
  if (!same_ctx(c, {A, T}, prec)) return fail(nullptr, "gelqf: descriptors of another context or precision");
  if (!lq_conform(A, T)) return fail(nullptr, "gelqf: square tiles <= 256 and a T of (IB x NB) tiles covering A");
  NatProgram* P = new_program(c, "gelqf", true);
  int last = -1;
  if (!P->info || !add_gelqf(*P, *A, *T, last)) return fail(P, "gelqf: device allocation failed");
  return P;
}

NatProgram* nat_unmlq(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_desc_t* dA, dplasma_desc_t* dT,
                      dplasma_desc_t* dC) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *C = dC ? dC->nat : nullptr;
  if (!same_ctx(c, {A, T, C}, prec)) return fail(nullptr, "unmlq: descriptors of another context or precision");
  if (!lq_conform(A, T) || !has_fullT_lq(*A, *T)) return fail(nullptr, "unmlq: T must come from the native gelqf of A");
  if ((side == LEFT && (C->m != A->n || C->mb != A->nb)) || (side == RIGHT && (C->n != A->n || C->nb != A->nb)))
    return fail(nullptr, "unmlq: C does not conform to Q");
  NatProgram* P = new_program(c, "unmlq", false);
  int last = -1;
  if (!add_unmlq(*P, side, trans, *A, *T, *C, last)) return fail(P, "unmlq: device allocation failed");
  return P;
}

// Q (K x N) := the first K rows of the LQ orthogonal factor = (the first K columns of Q_r)^H
NatProgram* nat_unglq(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT, dplasma_desc_t* dQ) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *Q = dQ ? dQ->nat : nullptr;
  if (!same_ctx(c, {A, T, Q}, prec)) return fail(nullptr, "unglq: descriptors of another context or precision");
  if (!lq_conform(A, T) || !has_fullT_lq(*A, *T) || Q->n != A->n || Q->nb != A->nb || Q->mb != A->mb || Q->m > A->n)
    return fail(nullptr, "unglq: T from the native gelqf of A, Q with A's columns");
  NatProgram* P = new_program(c, "unglq", false);
  auto W = ctrans_desc(*P, *A), Qt = ctrans_desc(*P, *Q);
  if (!W || !Qt) return fail(P, "unglq: device allocation failed");
  std::vector<TileItem> it;
  for (int i = 0; i < Qt->mt; ++i)
    for (int j = 0; j < Qt->nt; ++j) it.push_back(TileItem{Qt->off(i, j), 0, Qt->rows(i), Qt->cols(j), i * Qt->mb, j * Qt->nb});
  auto d_it = dev_upload(it);
  if (!d_it) return fail(P, "unglq: device allocation failed");
  P->keep.push_back(d_it);
  const int n = (int)it.size(), mb = Qt->mb, nb = Qt->nb, ldq = Qt->lld;
  char* q = Qt->data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  int last = P->task(1, [=](hipStream_t s) {
    return dpl_laset(prec, 0, n, d_it->p, mb, nb, zero.ptr(), one.ptr(), q, ldq, s);
  }, {});
  last = add_ctrans(*P, *A, *W, last);
  if (last < -1 || !add_unmqr(*P, LEFT, NOTRANS, *W, *T, *Qt, last)) return fail(P, "unglq: device allocation failed");
  if (add_ctrans(*P, *Qt, *Q, last) < -1) return fail(P, "unglq: device allocation failed");
  return P;
}

// minimum-norm solution of an M <= N system (reference src/zgelqs_wrapper.c): B(0:M) := L^-1 B(0:M), then
// B := Q^H B (B's N rows receive X)
static bool add_gelqs(NatProgram& P, NatDesc& A, NatDesc& T, NatDesc& B, int& last) {
  auto L = lead_view(A, A.m, A.m), Y = lead_view(B, A.m, B.n);
  P.wdesc.push_back(L);
  P.wdesc.push_back(Y);
  if (!add_trsm(P, LEFT, LOWER, NOTRANS, NONUNIT, Scalar(A.prec, 1.0), *L, *Y, 1, last)) return false;
  last = last_on(P, 1);
  return add_unmlq(P, LEFT, CONJTRANS, A, T, B, last);
}

NatProgram* nat_gelqs(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, dplasma_desc_t* dT, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx(c, {A, T, B}, prec)) return fail(nullptr, "gelqs: descriptors of another context or precision");
  if (!lq_conform(A, T) || !has_fullT_lq(*A, *T) || A->m > A->n || B->m < A->n || B->mb != A->nb)
    return fail(nullptr, "gelqs: T from the native gelqf of an M <= N matrix A, B with N rows");
  NatProgram* P = new_program(c, "gelqs", false);
  int last = -1;
  if (!add_gelqs(*P, *A, *T, *B, last)) return fail(P, "gelqs: device allocation failed");
  return P;
}

// least squares (M >= N: QR) or minimum norm (M < N: LQ), NoTrans (reference src/zgels_wrapper.c)
NatProgram* nat_gels(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* dA, dplasma_desc_t* dT,
                     dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr, *B = dB ? dB->nat : nullptr;
  if (!same_ctx_dist(c, {A, T, B}, prec)) return fail(nullptr, "gels: descriptors of another context or precision");
  if (trans != NOTRANS) return fail(nullptr, "gels: NoTrans (native engine)");
  if (c->dist()) {
    if (A->m < A->n || !qr_conform(A, T) || B->m != A->m || B->mb != A->mb)
      return fail(nullptr, "gels: a multi-process context solves M >= N least squares (T of IB x NB tiles, B with A's rows)");
    return nat_dist_gels(c, *A, *T, *B);
  }
  NatProgram* P = new_program(c, "gels", true);
  int last = -1;
  if (A->m >= A->n) {
    if (!qr_conform(A, T) || B->m != A->m || B->mb != A->mb)
      return fail(P, "gels: T of (IB x NB) tiles covering A, B with A's rows");
    if (!P->info || !add_geqrf(*P, *A, *T, last) || !add_geqrs(*P, *A, *T, *B, last))
      return fail(P, "gels: device allocation failed");
  } else {
    if (!lq_conform(A, T) || B->m < A->n || B->mb != A->nb)
      return fail(P, "gels: T of (IB x NB) tiles covering A, B with N rows");
    if (!P->info || !add_gelqf(*P, *A, *T, last) || !add_gelqs(*P, *A, *T, *B, last))
      return fail(P, "gels: device allocation failed");
  }
  return P;
}

// ----------------------------------------------------------------------------- tree-driven QR / LQ (*_param)
// dplasma_zgeqrf_param and its family (reference src/zgeqrf_param.jdf, zunmqr_param*.jdf, zungqr_param.jdf) on
// one process, driven by a native reduction tree (native_qrtree.cpp).  Each panel step k follows the tree's
// plan: every TS domain (a GEQRT head with the rows it TS-kills) is ONE stacked Householder panel (rows
// gathered into a panel buffer, dpl_qr_panel, written back: R in the head tile, V below the diagonal and in
// the killed tiles), then every TT kill (p, m) in plan order is the panel of the two stacked triangles
// [R_p; R_m] (V = [I; V2], V2 upper triangular into A(m, k)'s upper part, A(p, k)'s R replaced) -- the
// stacked-domain design of models/qr_panel.py, with the same trailing update C -= V op(T) (V^H C) as three
// batched MFMA GEMM launches per entry.  T: the full nb x nb compact-WY factor of every entry in a slot of the
// TS (domains) / TT (kills) descriptor's side buffer, its IB x IB diagonal blocks in the reference-layout
// tile TS(head, k) / TT(m, k) (LQ: tile (k, row)).  The apply rebuilds each entry's V from A and replays the
// entries forward (Q^H) or backward (Q).  The LQ variants run the QR engine on A^H (native gelqf's scheme).
namespace {

struct QpEntry {
  bool tt = false;
  std::vector<int> rows, voff;   // tile rows (rows[0]: head / annihilator) and their offsets in the stack
  int M = 0, kf = 0, k = 0;
  int trow = 0;                  // T slot row: the domain head / the TT-killed row
};

// the entries of every panel step, in execution order
std::vector<std::vector<QpEntry>> qp_entries(const nq::Tree& t, const NatDesc& A) {
  const int kt = std::min(A.mt, A.nt);
  std::vector<std::vector<QpEntry>> out(kt);
  for (int k = 0; k < kt; ++k) {
    std::vector<int> heads;
    std::vector<nq::Kill> kills;
    t.plan(k, heads, kills);
    const int kb = A.cols(k);
    for (int h : heads) {
      QpEntry e;
      e.k = k;
      e.rows.push_back(h);
      for (const nq::Kill& x : kills)
        if (x.type == nq::KILLED_BY_TS && x.piv == h) e.rows.push_back(x.m);
      e.trow = h;
      out[k].push_back(e);
    }
    for (const nq::Kill& x : kills) {
      if (x.type == nq::KILLED_BY_TS) continue;
      QpEntry e;
      e.tt = true;
      e.k = k;
      e.rows = {x.piv, x.m};
      e.trow = x.m;
      out[k].push_back(e);
    }
    for (QpEntry& e : out[k]) {
      int c = 0;
      for (int r : e.rows) {
        e.voff.push_back(c);
        c += A.rows(r);
      }
      e.M = c;
      e.kf = std::min(c, kb);
    }
  }
  return out;
}

bool tree_fits(const nq::Tree* t, const NatDesc& A) { return t && t->mt == A.mt && t->nt == A.nt; }

// C(rows_i, cols) := op(H) C(rows_i, cols), H = I - V T V^H, V rows = the stacked rows (row tile i at voff_i of V)
bool add_left_apply_rows(NatProgram& P, int prec, NatDesc& C, const std::vector<int>& rows, const std::vector<int>& voff,
                         int kf, char* V, int ldv, char* Tk, int ldt, bool qt, char* W, char* W2,
                         const std::vector<int>& cols, int stream, int dep, int& out) {
  out = dep;
  if (cols.empty() || kf <= 0) return true;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  long long wo = 0;
  for (int j : cols) {
    const int nj = C.cols(j);
    std::vector<KPair> kp;
    for (size_t i = 0; i < rows.size(); ++i) kp.push_back(KPair{voff[i], C.off(rows[i], j), C.rows(rows[i]), 0});
    g1->add(wo, kf, nj, kp, 0);
    g2->add(wo, kf, nj, {KPair{0, wo, kf, 0}}, 0);
    for (size_t i = 0; i < rows.size(); ++i)
      g3->add(C.off(rows[i], j), C.rows(rows[i]), nj, {KPair{voff[i], wo, kf, 0}}, 0);
    wo += (long long)kf * nj;
  }
  if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return false;
  char* c = C.data;
  const int ldc = C.lld;
  int t = P.task(stream, [=](hipStream_t s) { return g1->launch(prec, CONJTRANS, NOTRANS, one, V, ldv, c, ldc, zero, W, kf, s); },
                 {dep});
  t = P.task(stream, [=](hipStream_t s) {
    return g2->launch(prec, qt ? CONJTRANS : NOTRANS, NOTRANS, one, Tk, ldt, W, kf, zero, W2, kf, s);
  }, {t});
  out = P.task(stream, [=](hipStream_t s) { return g3->launch(prec, NOTRANS, NOTRANS, m_one, V, ldv, W2, kf, one, c, ldc, s); },
               {t});
  return true;
}

// C(:, cols_i) := C(:, cols_i) op(H) (right; C's column tile cols_i pairs with V's row tile i): W = sum C V_i,
// W2 = W op(T), C(:, cols_i) -= W2 V_i^H
bool add_right_apply_rows(NatProgram& P, int prec, NatDesc& C, const std::vector<int>& rows, const std::vector<int>& voff,
                          int kf, char* V, int ldv, char* Tk, int ldt, bool qt, char* W, char* W2, int ldw, int stream,
                          int dep, int& out) {
  out = dep;
  if (kf <= 0 || C.mt == 0) return true;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  for (int i = 0; i < C.mt; ++i) {
    const long long wo = (long long)i * C.mb;
    std::vector<KPair> kp;
    for (size_t r = 0; r < rows.size(); ++r) kp.push_back(KPair{C.off(i, rows[r]), voff[r], C.cols(rows[r]), 0});
    g1->add(wo, C.rows(i), kf, kp, 0);
    g2->add(wo, C.rows(i), kf, {KPair{wo, 0, kf, 0}}, 0);
    for (size_t r = 0; r < rows.size(); ++r)
      g3->add(C.off(i, rows[r]), C.rows(i), C.cols(rows[r]), {KPair{wo, voff[r], kf, 0}}, 0);
  }
  if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return false;
  char* c = C.data;
  const int ldc = C.lld;
  int t = P.task(stream, [=](hipStream_t s) { return g1->launch(prec, NOTRANS, NOTRANS, one, c, ldc, V, ldv, zero, W, ldw, s); },
                 {dep});
  t = P.task(stream, [=](hipStream_t s) {
    return g2->launch(prec, NOTRANS, qt ? CONJTRANS : NOTRANS, one, W, ldw, Tk, ldt, zero, W2, ldw, s);
  }, {t});
  out = P.task(stream, [=](hipStream_t s) {
    return g3->launch(prec, NOTRANS, CONJTRANS, m_one, W2, ldw, V, ldv, one, c, ldc, s);
  }, {t});
  return true;
}

// tile copies between A(rows_i, k) and the stack (part: 0 full, 2 upper incl. the diagonal, tile coordinates)
int add_stack_copy(NatProgram& P, const NatDesc& A, const QpEntry& e, char* buf, int ldb, bool to_stack, int part,
                   int stream, int dep) {
  std::vector<TileItem> it;
  const int kb = A.cols(e.k);
  for (size_t i = 0; i < e.rows.size(); ++i) {
    const long long ao = A.off(e.rows[i], e.k), so = e.voff[i];
    it.push_back(to_stack ? TileItem{ao, so, A.rows(e.rows[i]), kb, 0, 0} : TileItem{so, ao, A.rows(e.rows[i]), kb, 0, 0});
  }
  auto d = dev_upload(it);
  if (!d) return -2;
  P.keep.push_back(d);
  const int n = (int)it.size(), prec = A.prec, lda = A.lld, mb = A.mb;
  char* a = A.data;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  return P.task(stream, [=](hipStream_t s) {
    return to_stack ? dpl_geadd(prec, part, NOTRANS, n, d->p, mb, kb, one.ptr(), a, lda, zero.ptr(), buf, ldb, 1, s)
                    : dpl_geadd(prec, part, NOTRANS, n, d->p, mb, kb, one.ptr(), buf, ldb, zero.ptr(), a, lda, 1, s);
  }, {dep});
}

// an entry's explicit V (unit diagonal, zeros above) rebuilt from the factored A into V (ld ldv)
int add_entry_v(NatProgram& P, const NatDesc& A, const QpEntry& e, char* V, int ldv, int stream, int dep) {
  const int prec = A.prec, kb = A.cols(e.k), mb = A.mb, lda = A.lld;
  std::vector<TileItem> lt, ct;
  for (size_t i = 0; i < e.rows.size(); ++i) {
    const int r = e.rows[i];
    lt.push_back(TileItem{0, e.voff[i], A.rows(r), kb, e.voff[i], 0});   // stacked diagonal ones, zeros elsewhere
    if (e.tt) {
      if (i == 1) ct.push_back(TileItem{A.off(r, e.k), e.voff[i], A.rows(r), kb, 0, 0});   // V2: the upper part
    } else {
      ct.push_back(TileItem{A.off(r, e.k), e.voff[i], A.rows(r), kb, e.voff[i], 0});       // strictly below the stacked diagonal
    }
  }
  for (TileItem& x : lt) std::swap(x.a_off, x.b_off);   // laset items address B through a_off
  auto dl = dev_upload(lt), dc = dev_upload(ct);
  if (!dl || !dc) return -2;
  P.keep.push_back(dl);
  P.keep.push_back(dc);
  const int nl = (int)lt.size(), nc = (int)ct.size(), part = e.tt ? 2 : 3;
  char* a = A.data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  const int t = P.task(stream, [=](hipStream_t s) {
    return dpl_laset(prec, 0, nl, dl->p, mb, kb, zero.ptr(), one.ptr(), V, ldv, s);
  }, {dep});
  return P.task(stream, [=](hipStream_t s) {
    return dpl_geadd(prec, part, NOTRANS, nc, dc->p, mb, kb, one.ptr(), a, lda, zero.ptr(), V, ldv, 1, s);
  }, {t});
}

struct QpBufs {
  DevPtr P, V, W, W2, ws;
  int ld = 0;
};

bool qp_bufs(NatProgram& P, const NatDesc& A, const std::vector<std::vector<QpEntry>>& ents, size_t wlen, QpBufs& b) {
  int maxM = 16;
  for (const auto& st : ents)
    for (const QpEntry& e : st) maxM = std::max(maxM, e.M);
  b.ld = (maxM + 15) / 16 * 16;
  const int es = A.es, nb = A.nb;
  b.P = dev_alloc((size_t)b.ld * nb * es, true);
  b.V = dev_alloc((size_t)b.ld * nb * es, true);
  b.W = dev_alloc(wlen * es, false);
  b.W2 = dev_alloc(wlen * es, false);
  b.ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(A.prec, nb, nb) + 256, true);
  for (const DevPtr& d : {b.P, b.V, b.W, b.W2, b.ws}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  return true;
}

// T slots: one nb x nb factor per (trow, k) of the entries of one kind, in the descriptor's side buffer
bool qp_slots(NatProgram& P, NatDesc& T, const NatDesc& A, const std::vector<std::vector<QpEntry>>& ents, bool tt) {
  const int kt = (int)ents.size(), nb = A.nb;
  T.tidx.assign((size_t)kt * A.mt, -1);
  T.tidx_mt = A.mt;
  long long n = 0;
  for (const auto& st : ents)
    for (const QpEntry& e : st)
      if (e.tt == tt) T.tidx[(size_t)e.k * A.mt + e.trow] = n++;
  T.fullT = dev_alloc((size_t)std::max(1LL, n) * nb * nb * A.es, true);
  T.fullT_nb = nb;
  T.fullT_kt = -1;   // not a flat-tree T: the plain unmqr / ungqr refuse it
  if (!T.fullT) return false;
  P.keep.push_back(T.fullT);
  return true;
}

char* qp_slot(const NatDesc& T, const QpEntry& e) {
  const long long s = T.tidx[(size_t)e.k * T.tidx_mt + e.trow];
  return s < 0 ? nullptr : (char*)T.fullT->p + (size_t)s * T.fullT_nb * T.fullT_nb * T.es;
}

bool tree_T_ok(const NatDesc& T, const NatDesc& A, const std::vector<std::vector<QpEntry>>& ents, bool tt) {
  if (!T.fullT || T.fullT_nb != A.nb || T.tidx_mt != A.mt || T.tidx.size() < ents.size() * (size_t)A.mt) return false;
  for (const auto& st : ents)
    for (const QpEntry& e : st)
      if (e.tt == tt && T.tidx[(size_t)e.k * A.mt + e.trow] < 0) return false;
  return true;
}

// one entry of a tree step: stack, factor (T into its slot), write back, reference-layout T blocks (LQ: tile
// (k, trow)), trailing update of columns k+1..; tasks on `stream` after prev; returns the last task (< -1: failure)
int add_qp_factor_entry(NatProgram& P, NatDesc& A, NatDesc& TS, NatDesc& TT, const QpEntry& e, const QpBufs& b, bool lq,
                        int stream, int prev) {
  const int prec = A.prec, nb = A.nb, es = A.es;
  int* info = (int*)P.info->p;
  char *pb = (char*)b.P->p, *vb = (char*)b.V->p, *ws = (char*)b.ws->p;
  const int ld = b.ld;
  const int k = e.k, kb = A.cols(k), M = e.M, kf = e.kf;
  NatDesc& Td = e.tt ? TT : TS;
  char* Tk = qp_slot(Td, e);
  if (e.tt)   // the stack of two triangles: zeros below them
    prev = P.task(stream, [=](hipStream_t s) { return (int)hipMemsetAsync(pb, 0, (size_t)ld * kb * es, s); }, {prev});
  prev = add_stack_copy(P, A, e, pb, ld, true, e.tt ? 2 : 0, stream, prev);
  if (prev < -1) return prev;
  prev = P.task(stream, [=](hipStream_t s) { return dpl_qr_panel(prec, pb, ld, 0, 0, M, kb, kf, vb, ld, Tk, nb, ws, info, s); },
                {prev});
  prev = add_stack_copy(P, A, e, pb, ld, false, e.tt ? 2 : 0, stream, prev);
  if (prev < -1) return prev;
  const int ti = lq ? k : e.trow, tj = lq ? e.trow : k;
  if (ti < Td.mt && tj < Td.nt) {
    const int ib = Td.mb;
    std::vector<TileItem> it;
    for (int b0 = 0; b0 < kf; b0 += ib) {
      const int bs = std::min(ib, kf - b0);
      it.push_back(TileItem{b0 + (long long)b0 * nb, Td.off(ti, tj) + (long long)b0 * Td.lld, bs, bs, 0, 0});
    }
    auto d = dev_upload(it);
    if (!d) return -2;
    P.keep.push_back(d);
    const int n = (int)it.size(), ldT = Td.lld;
    char* td = Td.data;
    const Scalar one(prec, 1.0), zero(prec, 0.0);
    prev = P.task(stream, [=](hipStream_t s) {
      return dpl_geadd(prec, 0, NOTRANS, n, d->p, ib, ib, one.ptr(), Tk, nb, zero.ptr(), td, ldT, 1, s);
    }, {prev});
  }
  std::vector<int> cols;
  for (int j = k + 1; j < A.nt; ++j) cols.push_back(j);
  int out = prev;
  if (!add_left_apply_rows(P, prec, A, e.rows, e.voff, kf, vb, ld, Tk, nb, true, (char*)b.W->p, (char*)b.W2->p, cols,
                           stream, prev, out))
    return -2;
  return out;
}

bool add_geqrf_param(NatProgram& P, const nq::Tree& tree, NatDesc& A, NatDesc& TS, NatDesc& TT, bool lq, int& last) {
  const auto ents = qp_entries(tree, A);
  QpBufs b;
  if (!qp_bufs(P, A, ents, (size_t)A.nb * std::max(1, A.n), b) || !qp_slots(P, TS, A, ents, false) ||
      !qp_slots(P, TT, A, ents, true))
    return false;
  int prev = last;
  for (const auto& st : ents)
    for (const QpEntry& e : st) {
      prev = add_qp_factor_entry(P, A, TS, TT, e, b, lq, 0, prev);
      if (prev < -1) return false;
    }
  last = prev;
  return true;
}

// C := op(Q) C (left) or C op(Q) (right), Q from add_geqrf_param of A with the same tree
bool add_unmqr_param(NatProgram& P, const nq::Tree& tree, int side, int trans, NatDesc& A, NatDesc& TS, NatDesc& TT,
                     NatDesc& C, int& last) {
  const int prec = A.prec, nb = A.nb;
  const bool left = side == LEFT, qt = trans != NOTRANS;
  const auto ents = qp_entries(tree, A);
  if (!tree_T_ok(TS, A, ents, false) || !tree_T_ok(TT, A, ents, true)) return false;
  std::vector<const QpEntry*> order;
  for (const auto& st : ents)
    for (const QpEntry& e : st) order.push_back(&e);
  // left: Q^H C replays the factorisation order, Q C the reverse; right: C Q in order, C Q^H reversed
  if (left ? !qt : qt) std::reverse(order.begin(), order.end());
  const int ldw = std::max(16, (C.m + 15) / 16 * 16);
  const size_t wlen = left ? (size_t)nb * std::max(1, C.n) : (size_t)ldw * nb;
  QpBufs b;
  if (!qp_bufs(P, A, ents, wlen, b)) return false;
  char* vb = (char*)b.V->p;
  int prev = last;
  for (const QpEntry* e : order) {
    prev = add_entry_v(P, A, *e, vb, b.ld, 1, prev);
    if (prev < -1) return false;
    char* Tk = qp_slot(e->tt ? TT : TS, *e);
    int out = prev;
    bool ok;
    if (left) {
      std::vector<int> cols;
      for (int j = 0; j < C.nt; ++j) cols.push_back(j);
      ok = add_left_apply_rows(P, prec, C, e->rows, e->voff, e->kf, vb, b.ld, Tk, nb, qt, (char*)b.W->p, (char*)b.W2->p,
                               cols, 1, prev, out);
    } else {
      ok = add_right_apply_rows(P, prec, C, e->rows, e->voff, e->kf, vb, b.ld, Tk, nb, qt, (char*)b.W->p,
                                (char*)b.W2->p, ldw, 1, prev, out);
    }
    if (!ok) return false;
    prev = out;
  }
  last = prev;
  return true;
}

bool param_conform(const NatDesc* A, const NatDesc* TS, const NatDesc* TT) {
  return A && TS && TT && A->mb == A->nb && A->nb <= 256 && TS->nb == A->nb && TT->nb == A->nb && TS->mb >= 1 &&
         TT->mb >= 1 && TS->mb <= A->nb && TT->mb <= A->nb;
}

}  // namespace

// ----------------------------------------------------------------------------- tree-driven QR on a P x Q grid
// geqrf_param / unmqr_param (left) / ungqr_param / geqrs_param on a multi-process native context (the native
// flat geqrf's data movement, native_dist.cpp, generalised to a reduction tree).  Step k: tile column k (rows
// k..) goes to every rank in one exchange and every rank runs the tree's entries of the step on its copy, in
// plan order -- each TS domain / TT kill one stacked panel (dpl_qr_panel: deterministic, so every rank holds the
// same R, V and T, replicated T slots as on one process) -- and after each entry the reflector is applied to
// this rank's trailing tiles: W = V_e(local rows)^H C_loc, the partial W summed over the process column (one
// exchange), C_loc -= V_e (T_e^H W).  The apply (unmqr_param) rebuilds V_e's local rows from column k's tiles
// of this process row (sent along the row by the column's owner) and replays the entries forward (Q^H) or
// backward (Q) the same way.
namespace {

struct DistQp {
  DevPtr slots, pan, P, V, ws, W, W2, Wr, raw;
  int ldv = 0, ldp = 0, ldr = 0;
};

bool dist_qp_bufs(NatProgram& P, const NatDesc& A, const NatDesc& C, const std::vector<std::vector<QpEntry>>& ents,
                  DistQp& b) {
  const int es = A.es, nb = A.nb, mb = A.mb;
  int maxM = 16;
  for (const auto& st : ents)
    for (const QpEntry& e : st) maxM = std::max(maxM, e.M);
  b.ldv = std::max(16, (A.m + 15) / 16 * 16);
  b.ldp = (maxM + 15) / 16 * 16;
  b.ldr = std::max(16, (A.lm + 15) / 16 * 16);
  const size_t wlen = (size_t)nb * std::max(1, C.ln);
  b.slots = dev_alloc((size_t)std::max(1, A.mt) * mb * nb * es, false);
  b.pan = dev_alloc((size_t)b.ldv * nb * es, true);
  b.P = dev_alloc((size_t)b.ldp * nb * es, true);
  b.V = dev_alloc((size_t)b.ldp * nb * es, true);
  b.ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(A.prec, nb, nb) + 256, true);
  b.W = dev_alloc(wlen * es, true);
  b.W2 = dev_alloc(wlen * es, true);
  b.Wr = dev_alloc((size_t)std::max(1, A.P - 1) * wlen * es, true);
  b.raw = dev_alloc((size_t)b.ldr * nb * es, true);
  for (const DevPtr& d : {b.slots, b.pan, b.P, b.V, b.ws, b.W, b.W2, b.Wr, b.raw}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  return true;
}

// C(local rows of e, local columns j >= j0) := op(H_e) C, V_e rows at voff (ld ldv) of V; partial W summed over
// the process column.  Stream 1 after prev.
int add_dist_entry_apply(NatProgram& P, NatDesc& C, const QpEntry& e, char* V, int ldv, const char* Tk, int ldt, bool qt,
                         int j0, const DistQp& b, int prev) {
  NatComm* comm = P.ctx->comm;
  const int prec = C.prec, es = C.es, ldc = C.lld, me = P.ctx->rank, kf = e.kf;
  std::vector<int> cols;
  for (int j = j0; j < C.nt; ++j)
    if (j % C.Q == C.mycol) cols.push_back(j);
  if (cols.empty() || kf <= 0) return prev;
  std::vector<size_t> lr;   // indices of e's rows that are mine
  for (size_t i = 0; i < e.rows.size(); ++i)
    if (e.rows[i] % C.P == C.myrow) lr.push_back(i);
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  long long wo = 0;
  for (int j : cols) {
    const int nj = C.cols(j);
    std::vector<KPair> kp;
    for (size_t i : lr) kp.push_back(KPair{e.voff[i], C.off(e.rows[i], j), C.rows(e.rows[i]), 0});
    if (!kp.empty()) g1->add(wo, kf, nj, kp, 0);
    g2->add(wo, kf, nj, {KPair{0, wo, kf, 0}}, 0);
    for (size_t i : lr) g3->add(C.off(e.rows[i], j), C.rows(e.rows[i]), nj, {KPair{e.voff[i], wo, kf, 0}}, 0);
    wo += (long long)kf * nj;
  }
  if ((!g1->empty() && !g1->upload(P)) || !g2->upload(P) || (!g3->empty() && !g3->upload(P))) return -2;
  const size_t wbytes = (size_t)wo * es;
  char *W = (char*)b.W->p, *W2 = (char*)b.W2->p, *Wr = (char*)b.Wr->p, *c = C.data;
  auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
  int slot = 0;
  for (int r = 0; r < C.P; ++r) {
    const int peer = r * C.Q + C.mycol;
    if (peer == me) continue;
    sends->push_back(NatMsg{peer, W, wbytes});
    recvs->push_back(NatMsg{peer, Wr + (size_t)slot * wbytes, wbytes});
    ++slot;
  }
  const int nsl = slot;
  std::vector<TileItem> sum_it{TileItem{0, 0, kf, (int)(wo / kf), 0, 0}};
  DevPtr d_sum = dev_upload(sum_it);
  if (!d_sum) return -2;
  P.keep.push_back(d_sum);
  const int wcols = (int)(wo / kf);
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  return P.task(1, [=](hipStream_t s) {
    int rc = 0;
    if (g1->empty()) rc = hipMemsetAsync(W, 0, wbytes, s) == hipSuccess ? 0 : -1;
    else rc = g1->launch(prec, CONJTRANS, NOTRANS, one, V, ldv, c, ldc, zero, W, kf, s);
    if (rc == 0 && nsl) rc = comm->exchange(*sends, *recvs, s);
    for (int q = 0; q < nsl && rc == 0; ++q)
      rc = dpl_geadd(prec, 0, NOTRANS, 1, d_sum->p, kf, wcols, one.ptr(), Wr + (size_t)q * wbytes, kf, one.ptr(), W, kf, 0, s);
    if (rc == 0) rc = g2->launch(prec, qt ? CONJTRANS : NOTRANS, NOTRANS, one, Tk, ldt, W, kf, zero, W2, kf, s);
    if (rc == 0 && !g3->empty()) rc = g3->launch(prec, NOTRANS, NOTRANS, m_one, V, ldv, W2, kf, one, c, ldc, s);
    return rc;
  }, {prev});
}

bool dist_geqrf_param(NatProgram& P, const nq::Tree& tree, NatDesc& A, NatDesc& TS, NatDesc& TT) {
  NatComm* comm = P.ctx->comm;
  const int prec = A.prec, mb = A.mb, nb = A.nb, ld = A.lld, es = A.es, me = P.ctx->rank;
  const auto ents = qp_entries(tree, A);
  DistQp b;
  if (!dist_qp_bufs(P, A, A, ents, b) || !qp_slots(P, TS, A, ents, false) || !qp_slots(P, TT, A, ents, true)) return false;
  char *a = A.data, *sl = (char*)b.slots->p, *pan = (char*)b.pan->p, *pb = (char*)b.P->p, *vb = (char*)b.V->p;
  char* ws = (char*)b.ws->p;
  int* info = (int*)P.info->p;
  const int ldv = b.ldv, ldp = b.ldp;
  const size_t st = (size_t)mb * nb;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  int prev = -1;
  for (const auto& step : ents) {
    if (step.empty()) continue;
    const int k = step[0].k, kb = A.cols(k);
    // ---- tile column k (rows k..) to every rank, unpacked into the contiguous panel (tile m at row (m - k) mb)
    auto pk = std::make_shared<MapBatch>(), sc = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
    auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
    for (int m = k; m < A.mt; ++m) {
      const int src = A.owner(m, k);
      char* slot = sl + (size_t)m * st * es;
      if (src == me) {
        pk->it.push_back(TileItem{A.off(m, k), (long long)m * (long long)st, A.rows(m), kb, 0, 0});
        back->it.push_back(TileItem{(long long)(m - k) * mb, A.off(m, k), A.rows(m), kb, 0, 0});
        for (int r = 0; r < P.ctx->world; ++r)
          if (r != me) sends->push_back(NatMsg{r, slot, st * es});
      } else {
        recvs->push_back(NatMsg{src, slot, st * es});
      }
      sc->it.push_back(TileItem{(long long)m * (long long)st, (long long)(m - k) * mb, A.rows(m), kb, 0, 0});
      pk->mm = sc->mm = back->mm = std::max(pk->mm, A.rows(m));
    }
    pk->nn = sc->nn = back->nn = kb;
    if (!pk->upload(P) || !sc->upload(P) || !back->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      int rc = pk->n() ? dpl_geadd(prec, 0, NOTRANS, pk->n(), pk->items(), pk->mm, pk->nn, one.ptr(), a, ld, zero.ptr(), sl,
                                   mb, 1, s) : 0;
      if (rc == 0 && (!sends->empty() || !recvs->empty())) rc = comm->exchange(*sends, *recvs, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, NOTRANS, sc->n(), sc->items(), sc->mm, sc->nn, one.ptr(), sl, mb, zero.ptr(), pan, ldv, 1, s);
      return rc;
    }, {prev});
    // ---- the step's entries, each factored on every rank's panel copy, then applied to this rank's trailing tiles
    for (const QpEntry& e : step) {
      NatDesc& Td = e.tt ? TT : TS;
      char* Tk = qp_slot(Td, e);
      const int M = e.M, kf = e.kf, part = e.tt ? 2 : 0;
      auto g = std::make_shared<MapBatch>(), w = std::make_shared<MapBatch>();
      for (size_t i = 0; i < e.rows.size(); ++i) {
        const long long po = (long long)(e.rows[i] - k) * mb;
        g->it.push_back(TileItem{po, e.voff[i], A.rows(e.rows[i]), kb, 0, 0});
        w->it.push_back(TileItem{e.voff[i], po, A.rows(e.rows[i]), kb, 0, 0});
        g->mm = w->mm = std::max(g->mm, A.rows(e.rows[i]));
      }
      g->nn = w->nn = kb;
      if (!g->upload(P) || !w->upload(P)) return false;
      const bool tt = e.tt;
      prev = P.task(1, [=](hipStream_t s) {
        int rc = tt ? (hipMemsetAsync(pb, 0, (size_t)ldp * kb * es, s) == hipSuccess ? 0 : -1) : 0;
        if (rc == 0)
          rc = dpl_geadd(prec, part, NOTRANS, g->n(), g->items(), g->mm, g->nn, one.ptr(), pan, ldv, zero.ptr(), pb, ldp, 1, s);
        if (rc == 0) rc = dpl_qr_panel(prec, pb, ldp, 0, 0, M, kb, kf, vb, ldp, Tk, nb, ws, info, s);
        if (rc == 0)
          rc = dpl_geadd(prec, part, NOTRANS, w->n(), w->items(), w->mm, w->nn, one.ptr(), pb, ldp, zero.ptr(), pan, ldv, 1, s);
        return rc;
      }, {prev});
      if (Td.local(e.trow, k)) {   // reference layout: IB x IB diagonal blocks of T into tile (trow, k)
        const int ib = Td.mb;
        std::vector<TileItem> it;
        for (int b0 = 0; b0 < kf; b0 += ib) {
          const int bs = std::min(ib, kf - b0);
          it.push_back(TileItem{b0 + (long long)b0 * nb, Td.off(e.trow, k) + (long long)b0 * Td.lld, bs, bs, 0, 0});
        }
        auto d = dev_upload(it);
        if (!d) return false;
        P.keep.push_back(d);
        const int n = (int)it.size(), ldT = Td.lld;
        char* td = Td.data;
        prev = P.task(1, [=](hipStream_t s) {
          return dpl_geadd(prec, 0, NOTRANS, n, d->p, ib, ib, one.ptr(), Tk, nb, zero.ptr(), td, ldT, 1, s);
        }, {prev});
      }
      prev = add_dist_entry_apply(P, A, e, vb, ldp, Tk, nb, true, k + 1, b, prev);
      if (prev < -1) return false;
    }
    // ---- this rank's tiles of the factored column back into A
    if (back->n())
      prev = P.task(1, [=](hipStream_t s) {
        return dpl_geadd(prec, 0, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), pan, ldv, zero.ptr(), a, ld,
                         1, s);
      }, {prev});
  }
  return true;
}

// C := op(Q) C (left), Q from dist_geqrf_param of A with the same tree; C distributed like A's rows
bool dist_unmqr_param(NatProgram& P, const nq::Tree& tree, int trans, NatDesc& A, NatDesc& TS, NatDesc& TT, NatDesc& C) {
  NatComm* comm = P.ctx->comm;
  const int prec = A.prec, mb = A.mb, ld = A.lld, es = A.es, Q = A.Q;
  const bool qt = trans != NOTRANS;
  const auto ents = qp_entries(tree, A);
  if (!tree_T_ok(TS, A, ents, false) || !tree_T_ok(TT, A, ents, true)) return false;
  DistQp b;
  if (!dist_qp_bufs(P, A, C, ents, b)) return false;
  char *a = A.data, *raw = (char*)b.raw->p, *vb = (char*)b.V->p;
  const int ldr = b.ldr, ldp = b.ldp;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  const int kt = (int)ents.size();
  int prev = -1;
  for (int s = 0; s < kt; ++s) {
    const int k = qt ? s : kt - 1 - s;   // Q^H C: step 0 first; Q C: the last first
    if (ents[k].empty()) continue;
    const int kb = A.cols(k), pc = k % Q;
    // my process row's rows of column k (local tile rows >= k) from the column's owner in this row
    long long lr0 = A.lm;
    for (int m = k; m < A.mt; ++m)
      if (m % A.P == A.myrow) {
        lr0 = (long long)(m / A.P) * mb;
        break;
      }
    const long long rows = A.lm - lr0;
    auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
    const size_t rbytes = (size_t)ldr * kb * es;
    if (rows > 0) {
      if (A.mycol == pc) {
        for (int q = 0; q < Q; ++q)
          if (q != A.mycol) sends->push_back(NatMsg{A.myrow * Q + q, raw, rbytes});
      } else {
        recvs->push_back(NatMsg{A.myrow * Q + pc, raw, rbytes});
      }
    }
    const bool mine = A.mycol == pc && rows > 0;
    const long long coff = lr0 + (long long)(k / Q) * A.nb * ld;
    prev = P.task(1, [=](hipStream_t st) {
      int rc = 0;
      if (mine && hipMemcpy2DAsync(raw, (size_t)ldr * es, a + coff * es, (size_t)ld * es, (size_t)rows * es, kb,
                                   hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = -1;
      if (rc == 0 && (!sends->empty() || !recvs->empty())) rc = comm->exchange(*sends, *recvs, st);
      return rc;
    }, {prev});
    std::vector<const QpEntry*> order;
    for (const QpEntry& e : ents[k]) order.push_back(&e);
    if (!qt) std::reverse(order.begin(), order.end());
    for (const QpEntry* ep : order) {
      const QpEntry& e = *ep;
      // V_e's local rows (stack coordinates at voff) from raw: TS domain -- strictly below the stacked diagonal with
      // a unit diagonal; TT kill -- identity on the survivor's rows, the upper part of the victim's tile
      auto lt = std::make_shared<MapBatch>(), cp = std::make_shared<MapBatch>();
      for (size_t i = 0; i < e.rows.size(); ++i) {
        const int r = e.rows[i];
        if (r % A.P != A.myrow) continue;
        const long long ro = (long long)(r / A.P) * mb - lr0;
        lt->it.push_back(TileItem{e.voff[i], 0, A.rows(r), kb, e.voff[i], 0});
        if (!e.tt) cp->it.push_back(TileItem{ro, e.voff[i], A.rows(r), kb, e.voff[i], 0});
        else if (i == 1) cp->it.push_back(TileItem{ro, e.voff[i], A.rows(r), kb, 0, 0});
        lt->mm = cp->mm = std::max(lt->mm, A.rows(r));
      }
      lt->nn = cp->nn = kb;
      if (!lt->upload(P) || !cp->upload(P)) return false;
      const int part = e.tt ? 2 : 3;
      prev = P.task(1, [=](hipStream_t st) {
        int rc = lt->n() ? dpl_laset(prec, 0, lt->n(), lt->items(), lt->mm, lt->nn, zero.ptr(), one.ptr(), vb, ldp, st) : 0;
        if (rc == 0 && cp->n())
          rc = dpl_geadd(prec, part, NOTRANS, cp->n(), cp->items(), cp->mm, cp->nn, one.ptr(), raw, ldr, zero.ptr(), vb, ldp, 1,
                         st);
        return rc;
      }, {prev});
      prev = add_dist_entry_apply(P, C, e, vb, ldp, qp_slot(e.tt ? TT : TS, e), A.nb, qt, 0, b, prev);
      if (prev < -1) return false;
    }
  }
  return true;
}

}  // namespace

NatProgram* nat_geqrf_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx_dist(c, {A, TS, TT}, prec)) return fail(nullptr, "geqrf_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT)) return fail(nullptr, "geqrf_param: square tiles <= 256 and TS / TT of (IB x NB) tiles");
  if (!tree_fits(t, *A)) return fail(nullptr, "geqrf_param: a native tree built for A's tile rows and columns");
  NatProgram* P = new_program(c, "geqrf_param", true);
  int last = -1;
  if (!P->info || !(c->dist() ? dist_geqrf_param(*P, *t, *A, *TS, *TT) : add_geqrf_param(*P, *t, *A, *TS, *TT, false, last)))
    return fail(P, "geqrf_param: device allocation failed");
  return P;
}

NatProgram* nat_unmqr_param(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_qrtree_t* q,
                            dplasma_desc_t* dA, dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dC) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *C = dC ? dC->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx_dist(c, {A, TS, TT, C}, prec)) return fail(nullptr, "unmqr_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !tree_fits(t, *A)) return fail(nullptr, "unmqr_param: operands of geqrf_param");
  if ((side == LEFT && (C->m != A->m || C->mb != A->mb)) || (side == RIGHT && (C->n != A->m || C->nb != A->mb)))
    return fail(nullptr, "unmqr_param: C does not conform to Q");
  if (c->dist() && side != LEFT) return fail(nullptr, "unmqr_param: a multi-process context applies Q from the left");
  NatProgram* P = new_program(c, "unmqr_param", false);
  int last = -1;
  if (!(c->dist() ? dist_unmqr_param(*P, *t, trans, *A, *TS, *TT, *C) : add_unmqr_param(*P, *t, side, trans, *A, *TS, *TT, *C, last)))
    return fail(P, "unmqr_param: TS / TT must come from the native geqrf_param of A with this tree");
  return P;
}

NatProgram* nat_ungqr_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dQ) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *Q = dQ ? dQ->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx_dist(c, {A, TS, TT, Q}, prec)) return fail(nullptr, "ungqr_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !tree_fits(t, *A) || Q->m != A->m || Q->mb != A->mb || Q->n > A->m)
    return fail(nullptr, "ungqr_param: operands of geqrf_param, Q with A's rows");
  NatProgram* P = new_program(c, "ungqr_param", false);
  std::vector<TileItem> it;
  for (int i = 0; i < Q->mt; ++i)
    for (int j = 0; j < Q->nt; ++j)
      if (Q->local(i, j)) it.push_back(TileItem{Q->off(i, j), 0, Q->rows(i), Q->cols(j), i * Q->mb, j * Q->nb});
  auto d_it = dev_upload(it);
  if (!d_it) return fail(P, "ungqr_param: device allocation failed");
  P->keep.push_back(d_it);
  const int n = (int)it.size(), mb = Q->mb, nb = Q->nb, ldq = Q->lld;
  char* qd = Q->data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  int last = P->task(1, [=](hipStream_t s) {
    return n ? dpl_laset(prec, 0, n, d_it->p, mb, nb, zero.ptr(), one.ptr(), qd, ldq, s) : 0;
  }, {});
  if (!(c->dist() ? dist_unmqr_param(*P, *t, NOTRANS, *A, *TS, *TT, *Q) : add_unmqr_param(*P, *t, LEFT, NOTRANS, *A, *TS, *TT, *Q, last)))
    return fail(P, "ungqr_param: TS / TT must come from the native geqrf_param of A with this tree");
  return P;
}

NatProgram* nat_geqrs_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *B = dB ? dB->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx_dist(c, {A, TS, TT, B}, prec)) return fail(nullptr, "geqrs_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !tree_fits(t, *A) || A->m < A->n || B->m != A->m || B->mb != A->mb)
    return fail(nullptr, "geqrs_param: operands of geqrf_param of an M >= N matrix, B with A's rows");
  NatProgram* P = new_program(c, "geqrs_param", false);
  int last = -1;
  if (!(c->dist() ? dist_unmqr_param(*P, *t, CONJTRANS, *A, *TS, *TT, *B)
                  : add_unmqr_param(*P, *t, LEFT, CONJTRANS, *A, *TS, *TT, *B, last)))
    return fail(P, "geqrs_param: TS / TT must come from the native geqrf_param of A with this tree");
  if (c->dist()) {   // R X = (Q^H B)(0:N) on the grid
    auto dv = [](const NatDesc& D, int r, int cc) {
      auto v = std::make_shared<NatDesc>();
      v->ctx = D.ctx, v->prec = D.prec, v->es = D.es, v->mb = D.mb, v->nb = D.nb, v->m = r, v->n = cc;
      v->mt = (r + D.mb - 1) / D.mb, v->nt = (cc + D.nb - 1) / D.nb;
      v->P = D.P, v->Q = D.Q, v->myrow = D.myrow, v->mycol = D.mycol;
      v->lm = nat_numroc(r, D.mb, D.myrow, D.P), v->ln = nat_numroc(cc, D.nb, D.mycol, D.Q);
      v->lld = D.lld, v->data = D.data, v->owned = false;
      return v;
    };
    auto R = dv(*A, A->n, A->n), X = dv(*B, A->n, B->n);
    P->wdesc.push_back(R);
    P->wdesc.push_back(X);
    if (!nat_dist_trsm_into(*P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(prec, 1.0), *R, *X))
      return fail(P, "geqrs_param: device allocation failed");
    return P;
  }
  auto R = lead_view(*A, A->n, A->n), X = lead_view(*B, A->n, B->n);
  P->wdesc.push_back(R);
  P->wdesc.push_back(X);
  if (!add_trsm(*P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(prec, 1.0), *R, *X, 1, last))
    return fail(P, "geqrs_param: device allocation failed");
  return P;
}

// ---- LQ: the QR engine on W = A^H with the tree built for A^H (trans = ConjTrans: its rows are A's tile columns)
NatProgram* nat_gelqf_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, TS, TT}, prec)) return fail(nullptr, "gelqf_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT)) return fail(nullptr, "gelqf_param: square tiles <= 256 and TS / TT of (IB x NB) tiles");
  if (!t || t->mt != A->nt || t->nt != A->mt) return fail(nullptr, "gelqf_param: a native tree built with trans = ConjTrans");
  NatProgram* P = new_program(c, "gelqf_param", true);
  auto W = ctrans_desc(*P, *A);
  if (!W) return fail(P, "gelqf_param: device allocation failed");
  int last = add_ctrans(*P, *A, *W, -1);
  if (last < -1 || !P->info || !add_geqrf_param(*P, *t, *W, *TS, *TT, true, last))
    return fail(P, "gelqf_param: device allocation failed");
  if (add_ctrans(*P, *W, *A, last) < -1) return fail(P, "gelqf_param: device allocation failed");
  return P;
}

namespace {
bool add_unmlq_param(NatProgram& P, const nq::Tree& t, int side, int trans, NatDesc& A, NatDesc& TS, NatDesc& TT,
                     NatDesc& C, int& last) {
  auto W = ctrans_desc(P, A);
  if (!W) return false;
  last = add_ctrans(P, A, *W, last);
  if (last < -1) return false;
  return add_unmqr_param(P, t, side, trans == NOTRANS ? CONJTRANS : NOTRANS, *W, TS, TT, C, last);
}
}  // namespace

NatProgram* nat_unmlq_param(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_qrtree_t* q,
                            dplasma_desc_t* dA, dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dC) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *C = dC ? dC->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, TS, TT, C}, prec)) return fail(nullptr, "unmlq_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !t || t->mt != A->nt || t->nt != A->mt)
    return fail(nullptr, "unmlq_param: operands of gelqf_param");
  if ((side == LEFT && (C->m != A->n || C->mb != A->nb)) || (side == RIGHT && (C->n != A->n || C->nb != A->nb)))
    return fail(nullptr, "unmlq_param: C does not conform to Q");
  NatProgram* P = new_program(c, "unmlq_param", false);
  int last = -1;
  if (!add_unmlq_param(*P, *t, side, trans, *A, *TS, *TT, *C, last))
    return fail(P, "unmlq_param: TS / TT must come from the native gelqf_param of A with this tree");
  return P;
}

NatProgram* nat_unglq_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dQ) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *Q = dQ ? dQ->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, TS, TT, Q}, prec)) return fail(nullptr, "unglq_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !t || t->mt != A->nt || t->nt != A->mt || Q->n != A->n || Q->nb != A->nb ||
      Q->mb != A->mb || Q->m > A->n)
    return fail(nullptr, "unglq_param: operands of gelqf_param, Q with A's columns");
  NatProgram* P = new_program(c, "unglq_param", false);
  auto W = ctrans_desc(*P, *A), Qt = ctrans_desc(*P, *Q);
  if (!W || !Qt) return fail(P, "unglq_param: device allocation failed");
  std::vector<TileItem> it;
  for (int i = 0; i < Qt->mt; ++i)
    for (int j = 0; j < Qt->nt; ++j) it.push_back(TileItem{Qt->off(i, j), 0, Qt->rows(i), Qt->cols(j), i * Qt->mb, j * Qt->nb});
  auto d_it = dev_upload(it);
  if (!d_it) return fail(P, "unglq_param: device allocation failed");
  P->keep.push_back(d_it);
  const int n = (int)it.size(), mb = Qt->mb, nb = Qt->nb, ldq = Qt->lld;
  char* qd = Qt->data;
  const Scalar zero(prec, 0.0), one(prec, 1.0);
  int last = P->task(1, [=](hipStream_t s) { return dpl_laset(prec, 0, n, d_it->p, mb, nb, zero.ptr(), one.ptr(), qd, ldq, s); },
                     {});
  last = add_ctrans(*P, *A, *W, last);
  if (last < -1 || !add_unmqr_param(*P, *t, LEFT, NOTRANS, *W, *TS, *TT, *Qt, last))
    return fail(P, "unglq_param: TS / TT must come from the native gelqf_param of A with this tree");
  if (add_ctrans(*P, *Qt, *Q, last) < -1) return fail(P, "unglq_param: device allocation failed");
  return P;
}

NatProgram* nat_gelqs_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA,
                            dplasma_desc_t* dTS, dplasma_desc_t* dTT, dplasma_desc_t* dB) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr,
          *B = dB ? dB->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, TS, TT, B}, prec)) return fail(nullptr, "gelqs_param: descriptors of another context or precision");
  if (!param_conform(A, TS, TT) || !t || t->mt != A->nt || t->nt != A->mt || A->m > A->n || B->m < A->n ||
      B->mb != A->nb)
    return fail(nullptr, "gelqs_param: operands of gelqf_param of an M <= N matrix, B with N rows");
  NatProgram* P = new_program(c, "gelqs_param", false);
  auto L = lead_view(*A, A->m, A->m), Y = lead_view(*B, A->m, B->n);
  P->wdesc.push_back(L);
  P->wdesc.push_back(Y);
  int last = -1;
  if (!add_trsm(*P, LEFT, LOWER, NOTRANS, NONUNIT, Scalar(prec, 1.0), *L, *Y, 1, last))
    return fail(P, "gelqs_param: device allocation failed");
  last = last_on(*P, 1);
  if (A->n > A->m) {   // B(M:N) := 0
    std::vector<TileItem> it;
    for (int i = 0; i < B->mt; ++i) {
      const int top = i * B->mb, rows = B->rows(i);
      if (top + rows <= A->m) continue;
      const int skip = std::max(0, A->m - top);
      for (int j = 0; j < B->nt; ++j)
        it.push_back(TileItem{B->off(i, j) + skip, 0, rows - skip, B->cols(j), 0, 0});
    }
    if (!it.empty()) {
      auto d = dev_upload(it);
      if (!d) return fail(P, "gelqs_param: device allocation failed");
      P->keep.push_back(d);
      const int n = (int)it.size(), mb = B->mb, nb = B->nb, ldb = B->lld;
      char* bd = B->data;
      const Scalar zero(prec, 0.0);
      last = P->task(1, [=](hipStream_t s) { return dpl_laset(prec, 0, n, d->p, mb, nb, zero.ptr(), zero.ptr(), bd, ldb, s); },
                     {last});
    }
  }
  if (!add_unmlq_param(*P, *t, LEFT, CONJTRANS, *A, *TS, *TT, *B, last))
    return fail(P, "gelqs_param: TS / TT must come from the native gelqf_param of A with this tree");
  return P;
}

// ----------------------------------------------------------------------------- hybrid LU-QR (getrf_qrf, trsmpl_qrf)
// dplasma_zgetrf_qrf / ztrsmpl_qrf (reference src/zgetrf_qrf.jdf, ztrsmpl_qrf.jdf; models/lu_qr.py) on one
// process.  Step k: the diagonal domain -- panel tiles k, k+p, k+2p, ... (p = the grid rows) -- is stacked into a
// contiguous buffer and factored by the device partial-pivoting recursion (A untouched); a host DECIDE task
// (one stream synchronisation) evaluates the criterion from that LU and the off-domain tiles and records it in
// lu_tab[k]; both branches are in the program as predicated tasks (NatTask::guard): LU -- the stacked factors
// written back, IPIV(k, k) := the 1-based stack pivots, the domain rows of the trailing columns interchanged,
// TRSM of row k with L_kk and of the off-domain tiles with U_kk, one MFMA GEMM batch; QR -- the tree's step k
// (stacked TS-domain / TT panels, as geqrf_param).  Criteria as models/lu_qr.py (HIGHAM: alpha cond_1(U_kk) >
// sum ||A_ik||_1, SUM / MAX / MOY: alpha / ||(L U)_kk^-1||_1 against the sum / max / mean, MUMPS column maxima,
// LU_ONLY, QR_ONLY, RANDOM (balanced table), DEFAULT alternating); alpha = 0 forces QR, >= 9999999999 LU, a
// singular domain QR.  Norms are exact (the reference estimates them with trcon / gecon: a decision exactly at
// the estimate's margin is parity unpinned).
namespace {

enum { LQ_DEFAULT = 0, LQ_HIGHAM = 1, LQ_MUMPS = 2, LQ_LU_ONLY = 3, LQ_QR_ONLY = 4, LQ_RANDOM = 5, LQ_HSUM = 6,
       LQ_HMAX = 7, LQ_HMOY = 8 };

// balanced recursive split of nb_lu LU steps over [deb, fin] (dplasma_genrandom_lutab, models/lu_qr.py)
void genrandom_lutab(std::vector<int>& t, int deb, int fin, int nb_lu, int depth) {
  if (deb == fin) {
    t[deb] = nb_lu != 0;
    return;
  }
  const int n = fin - deb + 1;
  const int new_fin = n % 2 == 0 ? deb - 1 + n / 2 : deb - 1 + (fin - deb) / 2 + (depth % 2);
  const int new_nb = nb_lu % 2 == 0 ? nb_lu / 2 : (nb_lu - 1) / 2 + (depth % 2);
  genrandom_lutab(t, deb, new_fin, new_nb, depth + 1);
  genrandom_lutab(t, new_fin + 1, fin, nb_lu - new_nb, depth + 1);
}

using cplx = std::complex<double>;

// host copy of an r x c block (element ld) of a device matrix of precision prec, widened to complex<double>
bool host_block(int prec, const char* src, int ld, int r, int c, std::vector<cplx>& out) {
  const int es = esize(prec);
  std::vector<unsigned char> raw((size_t)r * c * es);
  if (r > 0 && c > 0 &&
      hipMemcpy2D(raw.data(), (size_t)r * es, src, (size_t)ld * es, (size_t)r * es, c, hipMemcpyDeviceToHost) != hipSuccess)
    return false;
  out.resize((size_t)r * c);
  for (size_t i = 0; i < out.size(); ++i) {
    const unsigned char* p = raw.data() + i * es;
    if (prec == P_S) out[i] = *(const float*)p;
    else if (prec == P_D) out[i] = *(const double*)p;
    else if (prec == P_C) out[i] = cplx(((const float*)p)[0], ((const float*)p)[1]);
    else out[i] = cplx(((const double*)p)[0], ((const double*)p)[1]);
  }
  return true;
}

// inverse of an n x n triangular matrix (column-major, ld n); unit: implicit unit diagonal
std::vector<cplx> tri_inverse(const std::vector<cplx>& T, int n, bool upper, bool unit) {
  std::vector<cplx> X((size_t)n * n, 0.0);
  for (int j = 0; j < n; ++j) {   // column j of X solves T x = e_j
    std::vector<cplx> x(n, 0.0);
    x[j] = 1.0;
    if (upper) {
      for (int i = n - 1; i >= 0; --i) {
        cplx s = x[i];
        for (int c = i + 1; c < n; ++c) s -= T[i + (size_t)c * n] * x[c];
        x[i] = unit ? s : s / T[i + (size_t)i * n];
      }
    } else {
      for (int i = 0; i < n; ++i) {
        cplx s = x[i];
        for (int c = 0; c < i; ++c) s -= T[i + (size_t)c * n] * x[c];
        x[i] = unit ? s : s / T[i + (size_t)i * n];
      }
    }
    for (int i = 0; i < n; ++i) X[i + (size_t)j * n] = x[i];
  }
  return X;
}

double norm1(const std::vector<cplx>& X, int r, int c, int ld) {
  double m = 0;
  for (int j = 0; j < c; ++j) {
    double s = 0;
    for (int i = 0; i < r; ++i) s += std::abs(X[i + (size_t)j * ld]);
    m = std::max(m, s);
  }
  return m;
}

struct LuqrState {
  std::vector<std::shared_ptr<int>> dec;   // per step: 1 LU, 0 QR (set by the DECIDE task)
  std::vector<int> table;                  // RANDOM criterion's lu_tab
};

bool luqr_conform(const NatDesc* A, const NatDesc* IP, const NatDesc* TS, const NatDesc* TT) {
  return A && IP && param_conform(A, TS, TT) && IP->prec == P_I && IP->mb == A->mb && IP->nb == 1 && IP->mt >= A->mt &&
         IP->nt >= std::min(A->mt, A->nt);
}

}  // namespace

NatProgram* nat_getrf_qrf(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA, dplasma_desc_t* dIP,
                          dplasma_desc_t* dTS, dplasma_desc_t* dTT, int criteria, double alpha, int* lu_tab, int* INFO) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr, *TS = dTS ? dTS->nat : nullptr,
          *TT = dTT ? dTT->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, TS, TT}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "getrf_qrf: descriptors of another context or precision");
  if (!luqr_conform(A, IP, TS, TT))
    return fail(nullptr, "getrf_qrf: square tiles <= 256, TS / TT of (IB x NB) tiles, IPIV of (MB x 1) int tiles");
  if (!tree_fits(t, *A)) return fail(nullptr, "getrf_qrf: a native tree built for A's tile rows and columns");
  if (criteria < LQ_DEFAULT || criteria > LQ_HMOY) return fail(nullptr, "getrf_qrf: unknown criterion");
  NatProgram* P = new_program(c, "getrf_qrf", true);
  // the domain period: the grid rows (DPLASMA_LUQR_P overrides it, as models/lu_qr.py's p argument)
  const int kt = std::min(A->mt, A->nt), mb = A->mb, nb = A->nb, es = A->es, ld = A->lld,
            pgrid = std::max(1, env_int("DPLASMA_LUQR_P", A->P));
  const auto ents = qp_entries(*t, *A);
  QpBufs qb;
  LuScratch S;
  if (!P->info || !qp_bufs(*P, *A, ents, (size_t)nb * std::max(1, A->n), qb) || !qp_slots(*P, *TS, *A, ents, false) ||
      !qp_slots(*P, *TT, *A, ents, true) || !lu_scratch(*P, *A, S))
    return fail(P, "getrf_qrf: device allocation failed");
  // the trailing domain rows during the interchanges (stack order), the domain LU's info
  DevPtr WT = dev_alloc((size_t)std::max(1, A->m) * std::max(1, A->n) * es, false);
  DevPtr DI = dev_alloc(sizeof(int), true);
  if (!WT || !DI) return fail(P, "getrf_qrf: device allocation failed");
  P->keep.push_back(WT);
  P->keep.push_back(DI);
  auto state = std::make_shared<LuqrState>();
  if (criteria == LQ_RANDOM) {
    state->table.assign(kt, 0);
    if (kt > 0) genrandom_lutab(state->table, 0, kt - 1, (int)std::lround(kt * alpha / 100.0), 0);
  }
  char* a = A->data;
  char* buf = (char*)S.pv->p;
  char* wt = (char*)WT->p;
  int* dinfo = (int*)DI->p;
  int* ipg = (int*)IP->data;
  const Scalar one(prec, 1.0), m_one(prec, -1.0), zero(prec, 0.0);
  int prev = P->task(1, [=](hipStream_t) {
    if (INFO) *INFO = 0;
    return 0;
  }, {});
  for (int k = 0; k < kt; ++k) {
    std::vector<int> dom, off;
    for (int m = k; m < A->mt; m += pgrid) dom.push_back(m);
    for (int m = k + 1; m < A->mt; ++m)
      if ((m - k) % pgrid) off.push_back(m);
    int M = 0;
    std::vector<int> soff;
    for (int m : dom) {
      soff.push_back(M);
      M += A->rows(m);
    }
    const int ncol = A->cols(k), kmax = std::min(M, ncol);
    // ---- domain LU on the stacked copy (A untouched)
    auto gat = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
    for (size_t i = 0; i < dom.size(); ++i) {
      gat->it.push_back(TileItem{A->off(dom[i], k), soff[i], A->rows(dom[i]), ncol, 0, 0});
      back->it.push_back(TileItem{soff[i], A->off(dom[i], k), A->rows(dom[i]), ncol, 0, 0});
      gat->mm = back->mm = std::max(gat->mm, A->rows(dom[i]));
    }
    gat->nn = back->nn = ncol;
    if (!gat->upload(*P) || !back->upload(*P)) return fail(P, "getrf_qrf: device allocation failed");
    prev = P->task(1, [=](hipStream_t s) {
      if (hipMemsetAsync(dinfo, 0, sizeof(int), s) != hipSuccess) return -1;
      return dpl_geadd(prec, 0, NOTRANS, gat->n(), gat->items(), gat->mm, gat->nn, one.ptr(), a, ld, zero.ptr(), buf, M, 1, s);
    }, {prev});
    prev = add_panel_lu(*P, prec, buf, M, M, 0, kmax, S, dinfo, 0, prev, true);
    if (prev < 0) return fail(P, "getrf_qrf: device allocation failed");
    const int* piv = (const int*)S.piv->p;
    if (ncol > kmax) {   // fewer domain rows than columns: the last columns take the swaps and L^-1
      prev = P->task(1, [=](hipStream_t s) { return dpl_laswp_panel(prec, buf, M, M, kmax, ncol, piv, 0, kmax, dinfo, s); },
                     {prev});
      auto tr = std::make_shared<Trsm1>();
      tr->tri = 0;
      tr->add((long long)kmax * M, kmax, ncol - kmax);
      if (!tr->upload(*P, prec, LEFT)) return fail(P, "getrf_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) { return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, buf, M, buf, M, s); },
                     {prev});
    }
    // ---- DECIDE (host, one synchronisation): the criterion from the domain LU and the untouched column k
    auto dec = std::make_shared<int>(0);
    state->dec.push_back(dec);
    const int r0 = k * mb, mrows = A->m - r0;
    const std::vector<int> off_c = off, dom_c = dom;
    prev = P->task(1, [=](hipStream_t s) {
      if (hipStreamSynchronize(s) != hipSuccess) return -1;
      int bad = 0;
      if (hipMemcpy(&bad, dinfo, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
      std::vector<cplx> col, lu;
      const bool need_col = criteria == LQ_MUMPS || criteria == LQ_HIGHAM || criteria == LQ_HSUM ||
                            criteria == LQ_HMAX || criteria == LQ_HMOY;
      if (need_col && !host_block(prec, a + A->off(k, k) * es, ld, mrows, ncol, col)) return -1;
      double w0 = 0.0, offsum = 0.0, offmax = 0.0;
      std::vector<double> cm_off(ncol, 0.0), cm_diag(ncol, 0.0);
      if (need_col) {
        for (int m : off_c) {   // 1-norms / column maxima of the off-domain tiles of column k
          const int rr = A->rows(m), base = (m - k) * mb;
          double tn = 0;
          for (int j = 0; j < ncol; ++j) {
            double sj = 0, mj = 0;
            for (int i = 0; i < rr; ++i) {
              const double v = std::abs(col[base + i + (size_t)j * mrows]);
              sj += v;
              mj = std::max(mj, v);
            }
            tn = std::max(tn, sj);
            cm_off[j] = std::max(cm_off[j], mj);
          }
          offsum += tn;
          offmax = std::max(offmax, tn);
        }
        for (int j = 0; j < ncol; ++j)
          for (int i = 0; i < std::min(ncol, A->rows(k)); ++i) cm_diag[j] = std::max(cm_diag[j], std::abs(col[i + (size_t)j * mrows]));
      }
      if (!bad && (criteria == LQ_HIGHAM || criteria == LQ_HSUM || criteria == LQ_HMAX || criteria == LQ_HMOY)) {
        const int n = kmax;
        if (!host_block(prec, buf, M, n, n, lu)) return -1;
        std::vector<cplx> U((size_t)n * n, 0.0), L((size_t)n * n, 0.0);
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < n; ++i) {
            if (i <= j) U[i + (size_t)j * n] = lu[i + (size_t)j * n];
            if (i > j) L[i + (size_t)j * n] = lu[i + (size_t)j * n];
          }
        const std::vector<cplx> Ui = tri_inverse(U, n, true, false);
        if (criteria == LQ_HIGHAM) {
          w0 = norm1(U, n, n, n) * norm1(Ui, n, n, n);
        } else {   // 1 / ||U^-1 L^-1||_1
          const std::vector<cplx> Li = tri_inverse(L, n, false, true);
          std::vector<cplx> X((size_t)n * n, 0.0);
          for (int j = 0; j < n; ++j)
            for (int l = j; l < n; ++l) {   // Li is unit lower: column j nonzero from row j
              const cplx x = Li[l + (size_t)j * n];
              if (x == 0.0) continue;
              for (int i = 0; i <= l; ++i) X[i + (size_t)j * n] += Ui[i + (size_t)l * n] * x;
            }
          w0 = 1.0 / norm1(X, n, n, n);
        }
      }
      int cond;
      if (bad) cond = 0;
      else if (criteria == LQ_HIGHAM || criteria == LQ_HSUM) cond = alpha * w0 > offsum;
      else if (criteria == LQ_HMAX) cond = alpha * w0 > offmax;
      else if (criteria == LQ_HMOY) {
        const int ntk = A->mt - k, nout = ntk - (ntk + pgrid - 1) / pgrid;
        cond = nout ? alpha * w0 > offsum / nout : 0;   // 0 / 0: the reference's NaN comparison
      } else if (criteria == LQ_MUMPS) {
        cond = 1;
        for (int j = 0; j < ncol; ++j)
          if (!(alpha * cm_diag[j] >= cm_off[j])) cond = 0;
      } else if (criteria == LQ_LU_ONLY) cond = 1;
      else if (criteria == LQ_QR_ONLY) cond = 0;
      else if (criteria == LQ_RANDOM) cond = state->table[k];
      else cond = k % 2;
      if (!bad) {
        if (alpha == 0) cond = 0;
        if (alpha >= 9999999999.0) cond = 1;
      }
      *dec = cond;
      if (lu_tab) lu_tab[k] = cond;
      return 0;
    }, {prev});
    // ---- LU branch (predicated on *dec == 1)
    P->cur_guard = dec;
    P->cur_want = 1;
    prev = P->task(1, [=](hipStream_t s) {
      return dpl_geadd(prec, 0, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), buf, M, zero.ptr(), a, ld, 1, s);
    }, {prev});
    int* ipk = ipg + IP->off(k, k);
    const int rk = A->rows(k);
    prev = P->task(1, [=](hipStream_t s) {
      if (hipMemsetAsync(ipk, 0, sizeof(int) * rk, s) != hipSuccess) return -1;
      return dpl_ipiv_shift(piv, ipk, kmax, 1, s);
    }, {prev});
    // interchanges inside the domain stack of the trailing columns: gather, laswp, scatter
    const int ntc = A->n - (k + 1) * nb;
    if (ntc > 0) {
      auto tg = std::make_shared<MapBatch>(), ts = std::make_shared<MapBatch>();
      for (size_t i = 0; i < dom.size(); ++i)
        for (int n = k + 1; n < A->nt; ++n) {
          const long long so = soff[i] + (long long)(n - k - 1) * nb * M;
          tg->it.push_back(TileItem{A->off(dom[i], n), so, A->rows(dom[i]), A->cols(n), 0, 0});
          ts->it.push_back(TileItem{so, A->off(dom[i], n), A->rows(dom[i]), A->cols(n), 0, 0});
        }
      tg->mm = ts->mm = mb;
      tg->nn = ts->nn = nb;
      if (!tg->upload(*P) || !ts->upload(*P)) return fail(P, "getrf_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) {
        int rc = dpl_geadd(prec, 0, NOTRANS, tg->n(), tg->items(), tg->mm, tg->nn, one.ptr(), a, ld, zero.ptr(), wt, M, 1, s);
        if (rc == 0) rc = dpl_laswp_panel(prec, wt, M, M, 0, ntc, piv, 0, kmax, dinfo, s);
        if (rc == 0)
          rc = dpl_geadd(prec, 0, NOTRANS, ts->n(), ts->items(), ts->mm, ts->nn, one.ptr(), wt, M, zero.ptr(), a, ld, 1, s);
        return rc;
      }, {prev});
      // U row: A(k, n) := L_kk^-1 A(k, n)
      auto tr = std::make_shared<Trsm1>();
      tr->tri = A->off(k, k);
      for (int n = k + 1; n < A->nt; ++n) tr->add(A->off(k, n), kmax, A->cols(n));
      if (!tr->upload(*P, prec, LEFT)) return fail(P, "getrf_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) { return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, a, ld, a, ld, s); },
                     {prev});
    }
    if (!off.empty()) {   // off-domain tiles: A(m, k) := A(m, k) U_kk^-1
      auto tr = std::make_shared<Trsm1>();
      tr->tri = A->off(k, k);
      for (int m : off) tr->add(A->off(m, k), A->rows(m), ncol);
      if (!tr->upload(*P, prec, RIGHT)) return fail(P, "getrf_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) { return tr->launch(prec, RIGHT, UPPER, NOTRANS, NONUNIT, one, a, ld, a, ld, s); },
                     {prev});
    }
    if (k + 1 < A->mt && k + 1 < A->nt) {
      auto g = std::make_shared<Gemm>();
      for (int n = k + 1; n < A->nt; ++n)
        for (int m = k + 1; m < A->mt; ++m) g->add(A->off(m, n), A->rows(m), A->cols(n), {KPair{A->off(m, k), A->off(k, n), kmax, 0}}, 0);
      if (!g->upload(*P)) return fail(P, "getrf_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) { return g->launch(prec, NOTRANS, NOTRANS, m_one, a, ld, a, ld, one, a, ld, s); },
                     {prev});
    }
    // ---- QR branch (predicated on *dec == 0): the tree's step k
    P->cur_want = 0;
    prev = P->task(1, [=](hipStream_t s) { return (int)hipMemsetAsync(ipk, 0, sizeof(int) * rk, s); }, {prev});
    for (const QpEntry& e : ents[k]) {
      prev = add_qp_factor_entry(*P, *A, *TS, *TT, e, qb, false, 1, prev);
      if (prev < -1) return fail(P, "getrf_qrf: device allocation failed");
    }
    P->cur_guard.reset();
    P->cur_want = 1;
  }
  return P;
}

// B := the hybrid factorization's L_k^-1 P_k / Q_k^H applied in step order (lu_tab from getrf_qrf); the solve
// x = U^-1 (that B) is the caller's trsm with A's upper triangle (tests/testing_zgetrf_qrf.c)
NatProgram* nat_trsmpl_qrf(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* dA, dplasma_desc_t* dIP,
                           dplasma_desc_t* dB, dplasma_desc_t* dTS, dplasma_desc_t* dTT, int* lu_tab) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *IP = dIP ? dIP->nat : nullptr, *B = dB ? dB->nat : nullptr,
          *TS = dTS ? dTS->nat : nullptr, *TT = dTT ? dTT->nat : nullptr;
  const nq::Tree* t = nat_qrtree(q);
  if (!same_ctx(c, {A, B, TS, TT}, prec) || !IP || IP->ctx != c)
    return fail(nullptr, "trsmpl_qrf: descriptors of another context or precision");
  if (!luqr_conform(A, IP, TS, TT) || !tree_fits(t, *A) || !lu_tab || B->m != A->m || B->mb != A->mb)
    return fail(nullptr, "trsmpl_qrf: operands of getrf_qrf (with its lu_tab), B with A's rows");
  const auto ents = qp_entries(*t, *A);
  if (!tree_T_ok(*TS, *A, ents, false) || !tree_T_ok(*TT, *A, ents, true))
    return fail(nullptr, "trsmpl_qrf: TS / TT must come from the native getrf_qrf of A with this tree");
  NatProgram* P = new_program(c, "trsmpl_qrf", true);
  const int kt = std::min(A->mt, A->nt), mb = A->mb, es = A->es, pgrid = std::max(1, env_int("DPLASMA_LUQR_P", A->P));
  QpBufs qb;
  if (!qp_bufs(*P, *A, ents, (size_t)A->nb * std::max(1, B->n), qb)) return fail(P, "trsmpl_qrf: device allocation failed");
  DevPtr WT = dev_alloc((size_t)std::max(1, A->m) * std::max(1, B->n) * es, false);
  DevPtr PV = dev_alloc(sizeof(int) * (mb + 16), true);
  if (!WT || !PV) return fail(P, "trsmpl_qrf: device allocation failed");
  P->keep.push_back(WT);
  P->keep.push_back(PV);
  char *a = A->data, *b = B->data, *wt = (char*)WT->p;
  int* pv = (int*)PV->p;
  int* info = (int*)P->info->p;
  const int lda = A->lld, ldb = B->lld;
  const Scalar one(prec, 1.0), m_one(prec, -1.0), zero(prec, 0.0);
  int prev = -1;
  for (int k = 0; k < kt; ++k) {
    if (!lu_tab[k]) {
      for (const QpEntry& e : ents[k]) {
        prev = add_entry_v(*P, *A, e, (char*)qb.V->p, qb.ld, 1, prev);
        if (prev < -1) return fail(P, "trsmpl_qrf: device allocation failed");
        std::vector<int> cols;
        for (int j = 0; j < B->nt; ++j) cols.push_back(j);
        int out = prev;
        if (!add_left_apply_rows(*P, prec, *B, e.rows, e.voff, e.kf, (char*)qb.V->p, qb.ld, qp_slot(e.tt ? *TT : *TS, e),
                                 A->nb, true, (char*)qb.W->p, (char*)qb.W2->p, cols, 1, prev, out))
          return fail(P, "trsmpl_qrf: device allocation failed");
        prev = out;
      }
      continue;
    }
    std::vector<int> dom;
    std::vector<long long> soff;
    int M = 0;
    for (int m = k; m < A->mt; m += pgrid) {
      dom.push_back(m);
      soff.push_back(M);
      M += A->rows(m);
    }
    const int kmax = std::min(M, A->cols(k));
    const int* ipk = (const int*)IP->data + IP->off(k, k);
    auto tg = std::make_shared<MapBatch>(), ts = std::make_shared<MapBatch>();
    for (size_t i = 0; i < dom.size(); ++i)
      for (int n = 0; n < B->nt; ++n) {
        const long long so = soff[i] + (long long)n * B->nb * M;
        tg->it.push_back(TileItem{B->off(dom[i], n), so, B->rows(dom[i]), B->cols(n), 0, 0});
        ts->it.push_back(TileItem{so, B->off(dom[i], n), B->rows(dom[i]), B->cols(n), 0, 0});
      }
    tg->mm = ts->mm = mb;
    tg->nn = ts->nn = B->nb;
    if (!tg->upload(*P) || !ts->upload(*P)) return fail(P, "trsmpl_qrf: device allocation failed");
    const int bn = B->n;
    prev = P->task(1, [=](hipStream_t s) {   // the domain rows of B interchanged with the step's 1-based stack pivots
      int rc = dpl_ipiv_shift(ipk, pv, kmax, -1, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, NOTRANS, tg->n(), tg->items(), tg->mm, tg->nn, one.ptr(), b, ldb, zero.ptr(), wt, M, 1, s);
      if (rc == 0) rc = dpl_laswp_panel(prec, wt, M, M, 0, bn, pv, 0, kmax, info, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, NOTRANS, ts->n(), ts->items(), ts->mm, ts->nn, one.ptr(), wt, M, zero.ptr(), b, ldb, 1, s);
      return rc;
    }, {prev});
    auto tr = std::make_shared<Trsm1>();
    tr->tri = A->off(k, k);
    for (int n = 0; n < B->nt; ++n) tr->add(B->off(k, n), kmax, B->cols(n));
    if (!tr->upload(*P, prec, LEFT)) return fail(P, "trsmpl_qrf: device allocation failed");
    prev = P->task(1, [=](hipStream_t s) { return tr->launch(prec, LEFT, LOWER, NOTRANS, UNIT, one, a, lda, b, ldb, s); },
                   {prev});
    if (k + 1 < B->mt) {
      auto g = std::make_shared<Gemm>();
      for (int n = 0; n < B->nt; ++n)
        for (int m = k + 1; m < B->mt; ++m) g->add(B->off(m, n), B->rows(m), B->cols(n), {KPair{A->off(m, k), B->off(k, n), kmax, 0}}, 0);
      if (!g->upload(*P)) return fail(P, "trsmpl_qrf: device allocation failed");
      prev = P->task(1, [=](hipStream_t s) { return g->launch(prec, NOTRANS, NOTRANS, m_one, a, lda, b, ldb, one, b, ldb, s); },
                     {prev});
    }
  }
  return P;
}

// ----------------------------------------------------------------------------- eigenvalues (herbt, hbrdt, heev)
// dplasma_zherbt / zhbrdt / zheev (reference src/zherbt_L.jdf, zhbrdt.jdf, zheev_wrapper.c; models/eigen.py) on one
// process.  herbt: the uplo triangle mirrored into full Hermitian storage, then per panel k the tile column k below
// the diagonal block (rows k+1..) factored in place as one Householder panel (dpl_qr_panel) and applied from both
// sides to the trailing block A(k+1:, k+1:) -- Q^H from the left (columns k+1..), Q from the right (rows k+1..) --
// with the batched MFMA GEMM engine; T's IB x IB diagonal blocks into tile T(k+1, k); Upper: the band mirrored
// back.  hbrdt: the Hermitian band -> real tridiagonal bulge chase of csrc/runtime/band_core.h on the host;
// eigenvalues of the tridiagonal by implicit QL with Wilkinson-type shifts (the role of LAPACK dsterf).
namespace {

// dst := the conjugate transpose of the uplo triangle (full Hermitian storage); band_only: the first
// sub/super-diagonal tiles only.  Stream 1 after prev.
int add_mirror(NatProgram& P, NatDesc& A, int uplo, bool band_only, int prev) {
  auto off = std::make_shared<MapBatch>(), dia = std::make_shared<MapBatch>();
  for (int n = 0; n < A.nt; ++n) {
    const int mend = band_only ? std::min(A.mt, n + 2) : A.mt;
    for (int m = n + 1; m < mend; ++m) {
      if (uplo == LOWER) off->it.push_back(TileItem{A.off(m, n), A.off(n, m), A.rows(n), A.cols(m), 0, 0});
      else off->it.push_back(TileItem{A.off(n, m), A.off(m, n), A.rows(m), A.cols(n), 0, 0});
    }
    if (n < A.mt) dia->it.push_back(TileItem{A.off(n, n), A.off(n, n), A.rows(n), A.cols(n), 0, 0});
  }
  for (auto* b : {off.get(), dia.get()}) {
    for (const TileItem& x : b->it) {
      b->mm = std::max(b->mm, x.m);
      b->nn = std::max(b->nn, x.n);
    }
  }
  if (!off->upload(P) || !dia->upload(P)) return -2;
  const int prec = A.prec, ld = A.lld, dpart = uplo == LOWER ? 4 : 3;   // the other triangle of the diagonal tiles
  char* a = A.data;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  return P.task(1, [=](hipStream_t s) {
    int rc = off->n() ? dpl_geadd(prec, 0, CONJTRANS, off->n(), off->items(), off->mm, off->nn, one.ptr(), a, ld, zero.ptr(),
                                  a, ld, 1, s) : 0;
    if (rc == 0 && dia->n())
      rc = dpl_geadd(prec, dpart, CONJTRANS, dia->n(), dia->items(), dia->mm, dia->nn, one.ptr(), a, ld, zero.ptr(), a, ld, 1, s);
    return rc;
  }, {prev});
}

bool add_herbt(NatProgram& P, int uplo, NatDesc& A, NatDesc& T, int& last) {
  const int prec = A.prec, nb = A.nb, es = A.es, ld = A.lld, mb = A.mb;
  int prev = add_mirror(P, A, uplo, false, last);
  if (prev < -1) return false;
  if (A.mt > 1) {
    const int ldv = std::max(16, (A.m + 15) / 16 * 16);
    DevPtr V = dev_alloc((size_t)ldv * nb * es, true), Tk = dev_alloc((size_t)nb * nb * es, true);
    DevPtr W = dev_alloc((size_t)std::max(ldv, nb * std::max(1, A.nt)) * nb * es, false);
    DevPtr W2 = dev_alloc((size_t)std::max(ldv, nb * std::max(1, A.nt)) * nb * es, false);
    DevPtr ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(prec, nb, nb) + 256, true);
    for (const DevPtr& d : {V, Tk, W, W2, ws}) {
      if (!d) return false;
      P.keep.push_back(d);
    }
    char *a = A.data, *v = (char*)V->p, *tk = (char*)Tk->p, *w = (char*)W->p, *w2 = (char*)W2->p, *wsp = (char*)ws->p;
    int* info = (int*)P.info->p;
    const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
    for (int k = 0; k + 1 < A.mt && k < A.nt; ++k) {
      const int r0 = k + 1, M = A.m - r0 * mb, kb = A.cols(k), kf = std::min(M, kb);
      char* pk = a + A.off(r0, k) * es;
      prev = P.task(1, [=](hipStream_t s) { return dpl_qr_panel(prec, pk, ld, 0, 0, M, kb, kf, v, ldv, tk, nb, wsp, info, s); },
                    {prev});
      if (r0 < T.mt && k < T.nt) {   // reference layout: T's IB x IB diagonal blocks into tile T(k+1, k)
        const int ib = T.mb;
        std::vector<TileItem> it;
        for (int b0 = 0; b0 < kf; b0 += ib) {
          const int bs = std::min(ib, kf - b0);
          it.push_back(TileItem{b0 + (long long)b0 * nb, T.off(r0, k) + (long long)b0 * T.lld, bs, bs, 0, 0});
        }
        auto d = dev_upload(it);
        if (!d) return false;
        P.keep.push_back(d);
        const int n = (int)it.size(), ldT = T.lld;
        char* td = T.data;
        prev = P.task(1, [=](hipStream_t s) {
          return dpl_geadd(prec, 0, NOTRANS, n, d->p, ib, ib, one.ptr(), tk, nb, zero.ptr(), td, ldT, 1, s);
        }, {prev});
      }
      // left: A(k+1:, k+1:) := Q^H A(k+1:, k+1:)
      std::vector<int> cols;
      for (int j = r0; j < A.nt; ++j) cols.push_back(j);
      int out = prev;
      if (!add_left_apply(P, prec, A, r0, M, kf, v, ldv, tk, nb, true, w, w2, cols, 1, prev, out)) return false;
      prev = out;
      // right: A(k+1:, k+1:) := A(k+1:, k+1:) Q  (W = C V, W2 = W T, C -= W2 V^H; rows k+1.. only)
      auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
      const int ldw = ldv;
      for (int i = r0; i < A.mt; ++i) {
        const long long wo = (long long)(i - r0) * mb;
        std::vector<KPair> kp;
        for (int j = r0; j < A.nt; ++j) kp.push_back(KPair{A.off(i, j), (long long)(j - r0) * mb, A.cols(j), 0});
        g1->add(wo, A.rows(i), kf, kp, 0);
        g2->add(wo, A.rows(i), kf, {KPair{wo, 0, kf, 0}}, 0);
        for (int j = r0; j < A.nt; ++j) g3->add(A.off(i, j), A.rows(i), A.cols(j), {KPair{wo, (long long)(j - r0) * mb, kf, 0}}, 0);
      }
      if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return false;
      prev = P.task(1, [=](hipStream_t s) {
        int rc = g1->launch(prec, NOTRANS, NOTRANS, one, a, ld, v, ldv, zero, w, ldw, s);
        if (rc == 0) rc = g2->launch(prec, NOTRANS, NOTRANS, one, w, ldw, tk, nb, zero, w2, ldw, s);
        if (rc == 0) rc = g3->launch(prec, NOTRANS, CONJTRANS, m_one, w2, ldw, v, ldv, one, a, ld, s);
        return rc;
      }, {prev});
    }
  }
  if (uplo == UPPER) {   // the reduced band back into the upper triangle
    prev = add_mirror(P, A, LOWER, true, prev);
    if (prev < -1) return false;
  }
  last = prev;
  return true;
}

// eigenvalues (ascending) of the symmetric tridiagonal (d, e) by implicit QL: false if an eigenvalue took more
// than 64 sweeps
bool tridiag_eigenvalues(std::vector<double>& d, std::vector<double> e) {
  const int n = (int)d.size();
  e.resize(std::max(n, 1), 0.0);
  if (n > 0) e[n - 1] = 0.0;
  const double eps = std::numeric_limits<double>::epsilon();
  for (int l = 0; l < n; ++l) {
    int iter = 0, m;
    do {
      for (m = l; m < n - 1; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd) break;
      }
      if (m != l) {
        if (iter++ == 64) return false;
        double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
        double r = std::hypot(g, 1.0);
        g = d[m] - d[l] + e[l] / (g + (g >= 0 ? std::fabs(r) : -std::fabs(r)));
        double s = 1.0, c = 1.0, p = 0.0;
        bool deflated = false;
        for (int i = m - 1; i >= l; --i) {
          double f = s * e[i];
          const double b = c * e[i];
          r = std::hypot(f, g);
          e[i + 1] = r;
          if (r == 0.0) {   // underflow: split here and restart the sweep
            d[i + 1] -= p;
            e[m] = 0.0;
            deflated = true;
            break;
          }
          s = f / r;
          c = g / r;
          g = d[i + 1] - p;
          r = (d[i] - g) * s + 2.0 * c * b;
          p = s * r;
          d[i + 1] = g + p;
          g = c * r - b;
        }
        if (deflated) continue;
        d[l] -= p;
        e[l] = g;
        e[m] = 0.0;
      }
    } while (m != l);
  }
  std::sort(d.begin(), d.end());
  return true;
}

template <typename TT>
void band_chase(const std::vector<unsigned char>& raw, int ldab, int n, int b, std::vector<double>& d, std::vector<double>& e) {
  using R = typename dpl_band::real_of<TT>::type;
  std::vector<R> dr(n), er(std::max(n - 1, 0));
  int nth = env_int("OMP_NUM_THREADS", 0);
  if (nth <= 0) nth = (int)std::thread::hardware_concurrency();
  nth = std::max(1, std::min(nth, 16));
  dpl_band::hbrdt_core<TT>((const TT*)raw.data(), ldab, n, b, nth, dr.data(), er.data());
  d.assign(dr.begin(), dr.end());
  e.assign(er.begin(), er.end());
}

// the lower nb-band of A (after herbt) in LAPACK band storage AB(i - j, j), ldab = nb + 1, on the host
bool host_lower_band(const NatDesc& A, std::vector<unsigned char>& ab) {
  const int nb = A.nb, N = std::min(A.m, A.n), es = A.es, ldab = nb + 1;
  ab.assign((size_t)ldab * std::max(N, 1) * es, 0);
  std::vector<unsigned char> col((size_t)2 * nb * es);
  for (int j = 0; j < N; ++j) {
    const int rows = std::min(nb + 1, N - j);
    if (hipMemcpy(col.data(), A.data + ((size_t)j * A.lld + j) * es, (size_t)rows * es, hipMemcpyDeviceToHost) != hipSuccess)
      return false;
    std::memcpy(ab.data() + (size_t)j * ldab * es, col.data(), (size_t)rows * es);
  }
  return true;
}

bool chase_and_solve(int prec, const std::vector<unsigned char>& ab, int ldab, int n, int b, std::vector<double>& w,
                     std::vector<double>* e_out = nullptr) {
  std::vector<double> d, e;
  switch (prec) {
    case P_S: band_chase<float>(ab, ldab, n, b, d, e); break;
    case P_D: band_chase<double>(ab, ldab, n, b, d, e); break;
    case P_C: band_chase<std::complex<float>>(ab, ldab, n, b, d, e); break;
    default: band_chase<std::complex<double>>(ab, ldab, n, b, d, e); break;
  }
  if (e_out) {
    w = d;
    *e_out = e;
    return true;
  }
  w = d;
  return tridiag_eigenvalues(w, e);
}

}  // namespace

NatProgram* nat_herbt(dplasma_context_t* ctx, int prec, int uplo, int ib, dplasma_desc_t* dA, dplasma_desc_t* dT) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *T = dT ? dT->nat : nullptr;
  if (!same_ctx(c, {A, T}, prec)) return fail(nullptr, "herbt: descriptors of another context or precision");
  if (A->m != A->n || A->mb != A->nb || A->nb > 256 || T->mb != ib || T->nb != A->nb || T->mt < A->mt || T->nt < A->nt)
    return fail(nullptr, "herbt: square A of square tiles <= 256, T of mt x nt tiles of ib x nb");
  if (uplo != LOWER && uplo != UPPER) return fail(nullptr, "herbt: illegal uplo");
  NatProgram* P = new_program(c, "herbt", true);
  int last = -1;
  if (!P->info || !add_herbt(*P, uplo, *A, *T, last)) return fail(P, "herbt: device allocation failed");
  return P;
}

// band -> tridiagonal in place on a band descriptor ((nb+1) x N, LAPACK lower band storage): on exit row 0 holds d,
// row 1 holds e, the rest is zero (models/eigen.py hetrd_b2s); one host task
NatProgram* nat_hbrdt(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA) {
  NatCtx* c = ctx->nat;
  NatDesc* B = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {B}, prec)) return fail(nullptr, "hbrdt: a descriptor of this context and precision");
  if (B->m < 2) return fail(nullptr, "hbrdt: a band of at least 2 rows");
  NatProgram* P = new_program(c, "hbrdt", false);
  NatDesc* Bp = B;
  P->task(1, [=](hipStream_t s) {
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    const int es = Bp->es, ldab = Bp->m, n = Bp->n;
    std::vector<unsigned char> ab((size_t)ldab * std::max(n, 1) * es);
    if (hipMemcpy2D(ab.data(), (size_t)ldab * es, Bp->data, (size_t)Bp->lld * es, (size_t)ldab * es, n,
                    hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    std::vector<double> d, e;
    chase_and_solve(prec, ab, ldab, n, ldab - 1, d, &e);
    std::vector<unsigned char> out(ab.size(), 0);
    auto put = [&](int r, int j, double v) {
      unsigned char* p = out.data() + ((size_t)j * ldab + r) * es;
      if (prec == P_S || prec == P_C) {
        const float f = (float)v;
        std::memcpy(p, &f, sizeof f);
      } else {
        std::memcpy(p, &v, sizeof v);
      }
    };
    for (int j = 0; j < n; ++j) put(0, j, d[j]);
    for (int j = 0; j + 1 < n; ++j) put(1, j, e[j]);
    return hipMemcpy2D(Bp->data, (size_t)Bp->lld * es, out.data(), (size_t)ldab * es, (size_t)ldab * es, n,
                       hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
  }, {});
  return P;
}

// eigenvalues of Hermitian A (NoVec, as the reference): herbt, then one host task -- the band to the host, the chase,
// QL; W (N x 1, A's precision or its real counterpart) receives them in ascending order
NatProgram* nat_heev(dplasma_context_t* ctx, int prec, int jobz, int uplo, dplasma_desc_t* dA, dplasma_desc_t* dW,
                     dplasma_desc_t*) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *W = dW ? dW->nat : nullptr;
  if (jobz != 301 /* NoVec */) return fail(nullptr, "heev: only jobz = NoVec (as the reference)");
  if (!same_ctx(c, {A}, prec) || !W || W->ctx != c) return fail(nullptr, "heev: descriptors of this context");
  const int rprec = prec == P_C ? P_S : (prec == P_Z ? P_D : prec);
  if (W->prec != prec && W->prec != rprec) return fail(nullptr, "heev: W of A's precision or its real counterpart");
  if (W->m < A->n || A->m != A->n || A->mb != A->nb || A->nb > 256) return fail(nullptr, "heev: square A of square tiles <= 256, W with N rows");
  const int ib = std::min(32, A->nb);
  auto T = std::make_shared<NatDesc>();   // block-reflector scratch (mt x nt tiles of ib x nb)
  T->ctx = c, T->prec = prec, T->es = A->es, T->mb = ib, T->nb = A->nb, T->m = A->mt * ib, T->n = A->n;
  T->mt = A->mt, T->nt = A->nt, T->lm = T->m, T->ln = T->n, T->lld = std::max(16, (T->m + 15) / 16 * 16);
  void* tp = nullptr;
  if (hipMalloc(&tp, (size_t)T->lld * std::max(1, T->n) * A->es) != hipSuccess) return fail(nullptr, "heev: device allocation failed");
  T->data = (char*)tp;
  T->owned = true;
  NatProgram* P = new_program(c, "heev", true);
  P->wdesc.push_back(T);
  int last = -1;
  if (!P->info || !add_herbt(*P, uplo, *A, *T, last)) return fail(P, "heev: device allocation failed");
  NatDesc* Ap = A;
  NatDesc* Wp = W;
  P->task(1, [=](hipStream_t s) {
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    std::vector<unsigned char> ab;
    if (!host_lower_band(*Ap, ab)) return -1;
    std::vector<double> w;
    if (!chase_and_solve(prec, ab, Ap->nb + 1, Ap->n, Ap->nb, w)) return -3;   // QL did not converge
    const int wes = Wp->es;
    std::vector<unsigned char> wv((size_t)Ap->n * wes, 0);
    for (int i = 0; i < Ap->n; ++i) {
      unsigned char* p = wv.data() + (size_t)i * wes;
      if (Wp->prec == P_S || Wp->prec == P_C) {
        const float f = (float)w[i];
        std::memcpy(p, &f, sizeof f);
      } else {
        std::memcpy(p, &w[i], sizeof(double));
      }
    }
    return hipMemcpy(Wp->data, wv.data(), wv.size(), hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
  }, {last});
  return P;
}

// ----------------------------------------------------------------------------- general -> band bidiagonal (ge2gb)
// dplasma_zgebrd_ge2gb / ge2gbx (reference src/zgebrd_ge2gb.jdf; models/eigen.py gebrd_ge2gbx_New) on one process,
// flat trees: per k a QR step (tile column k, rows k.., one in-place Householder panel, Q^H applied to columns
// k+1..) and, for k < nt - 1, an LQ step on tile row k, columns k+1.. (its conjugate transpose factored as one panel
// in a scratch buffer and written back -- L in A(k, k+1), the conj(V) rows beside it, LAPACK's LQ layout -- then Q
// applied from the right to rows k+1..).  Band: (nb + 1) x N upper band storage AB(nb + i - j, j).
namespace {

struct Ge2gbBufs {
  DevPtr V, Tk, W, W2, ws, Bt;
  int ldv = 0, ldb = 0;
};

// C(i0.., j0..) := C(i0.., j0..) op(H), H = I - V T V^H, V rows <-> C columns from j0 (nb each)
int add_right_from(NatProgram& P, NatDesc& A, int i0, int j0, int kf, char* V, int ldv, char* Tk, bool qt, char* W, char* W2,
                   int ldw, int prev) {
  if (i0 >= A.mt || j0 >= A.nt || kf <= 0) return prev;
  const int prec = A.prec, mb = A.mb, nb = A.nb, ld = A.lld;
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  for (int i = i0; i < A.mt; ++i) {
    const long long wo = (long long)(i - i0) * mb;
    std::vector<KPair> kp;
    for (int j = j0; j < A.nt; ++j) kp.push_back(KPair{A.off(i, j), (long long)(j - j0) * nb, A.cols(j), 0});
    g1->add(wo, A.rows(i), kf, kp, 0);
    g2->add(wo, A.rows(i), kf, {KPair{wo, 0, kf, 0}}, 0);
    for (int j = j0; j < A.nt; ++j) g3->add(A.off(i, j), A.rows(i), A.cols(j), {KPair{wo, (long long)(j - j0) * nb, kf, 0}}, 0);
  }
  if (!g1->upload(P) || !g2->upload(P) || !g3->upload(P)) return -2;
  char* a = A.data;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  return P.task(1, [=](hipStream_t s) {
    int rc = g1->launch(prec, NOTRANS, NOTRANS, one, a, ld, V, ldv, zero, W, ldw, s);
    if (rc == 0) rc = g2->launch(prec, NOTRANS, qt ? CONJTRANS : NOTRANS, one, W, ldw, Tk, nb, zero, W2, ldw, s);
    if (rc == 0) rc = g3->launch(prec, NOTRANS, CONJTRANS, m_one, W2, ldw, V, ldv, one, a, ld, s);
    return rc;
  }, {prev});
}

// IB x IB diagonal blocks of the nb x nb T (ld nb) into tile (ti, tj) of Td
int add_T_blocks(NatProgram& P, const NatDesc& Td, int ti, int tj, int kf, char* Tk, int nb, int prev) {
  if (ti >= Td.mt || tj >= Td.nt) return prev;
  const int ib = Td.mb, prec = Td.prec;
  std::vector<TileItem> it;
  for (int b0 = 0; b0 < kf; b0 += ib) {
    const int bs = std::min(ib, kf - b0);
    it.push_back(TileItem{b0 + (long long)b0 * nb, Td.off(ti, tj) + (long long)b0 * Td.lld, bs, bs, 0, 0});
  }
  auto d = dev_upload(it);
  if (!d) return -2;
  P.keep.push_back(d);
  const int n = (int)it.size(), ldT = Td.lld;
  char* td = Td.data;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  return P.task(1, [=](hipStream_t s) {
    return dpl_geadd(prec, 0, NOTRANS, n, d->p, ib, ib, one.ptr(), Tk, nb, zero.ptr(), td, ldT, 1, s);
  }, {prev});
}

bool add_ge2gb(NatProgram& P, NatDesc& A, const NatDesc* TSq, const NatDesc* TSl, NatDesc* Band, int& last) {
  const int prec = A.prec, nb = A.nb, mb = A.mb, es = A.es, ld = A.lld;
  Ge2gbBufs b;
  b.ldv = std::max(16, (std::max(A.m, A.n) + 15) / 16 * 16);
  b.ldb = std::max(16, (A.n + 15) / 16 * 16);
  b.V = dev_alloc((size_t)b.ldv * nb * es, true);
  b.Tk = dev_alloc((size_t)nb * nb * es, true);
  const size_t wl = (size_t)std::max(b.ldv, nb * std::max(1, A.nt)) * nb;
  b.W = dev_alloc(wl * es, false);
  b.W2 = dev_alloc(wl * es, false);
  b.ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(prec, nb, nb) + 256, true);
  b.Bt = dev_alloc((size_t)b.ldb * nb * es, true);
  for (const DevPtr& d : {b.V, b.Tk, b.W, b.W2, b.ws, b.Bt}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  char *a = A.data, *v = (char*)b.V->p, *tk = (char*)b.Tk->p, *w = (char*)b.W->p, *w2 = (char*)b.W2->p;
  char *ws = (char*)b.ws->p, *bt = (char*)b.Bt->p;
  const int ldv = b.ldv, ldb = b.ldb;
  int* info = (int*)P.info->p;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  int prev = last;
  for (int k = 0; k < A.nt; ++k) {
    // ---- QR step: column k, rows k..
    const int M = A.m - k * mb, kb = A.cols(k), kf = std::min(M, kb);
    char* pk = a + A.off(k, k) * es;
    prev = P.task(1, [=](hipStream_t s) { return dpl_qr_panel(prec, pk, ld, 0, 0, M, kb, kf, v, ldv, tk, nb, ws, info, s); },
                  {prev});
    if (TSq) prev = add_T_blocks(P, *TSq, k, k, kf, tk, nb, prev);
    if (prev < -1) return false;
    std::vector<int> cols;
    for (int j = k + 1; j < A.nt; ++j) cols.push_back(j);
    int out = prev;
    if (!add_left_apply(P, prec, A, k, M, kf, v, ldv, tk, nb, true, w, w2, cols, 1, prev, out)) return false;
    prev = out;
    if (k + 1 >= A.nt) break;
    // ---- LQ step: row k, columns k+1.. (its conjugate transpose as one panel)
    const int Nl = A.n - (k + 1) * nb, rk = A.rows(k), kfl = std::min(Nl, rk);
    auto to = std::make_shared<MapBatch>(), fro = std::make_shared<MapBatch>();
    for (int j = k + 1; j < A.nt; ++j) {
      const long long bo = (long long)(j - k - 1) * nb;
      to->it.push_back(TileItem{A.off(k, j), bo, A.cols(j), rk, 0, 0});     // Bt(j-block) := A(k, j)^H
      fro->it.push_back(TileItem{bo, A.off(k, j), rk, A.cols(j), 0, 0});    // A(k, j) := Bt(j-block)^H
    }
    to->mm = nb, to->nn = rk;
    fro->mm = rk, fro->nn = nb;
    if (!to->upload(P) || !fro->upload(P)) return false;
    prev = P.task(1, [=](hipStream_t s) {
      int rc = dpl_geadd(prec, 0, CONJTRANS, to->n(), to->items(), to->mm, to->nn, one.ptr(), a, ld, zero.ptr(), bt, ldb, 1, s);
      if (rc == 0) rc = dpl_qr_panel(prec, bt, ldb, 0, 0, Nl, rk, kfl, v, ldv, tk, nb, ws, info, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, CONJTRANS, fro->n(), fro->items(), fro->mm, fro->nn, one.ptr(), bt, ldb, zero.ptr(), a, ld, 1, s);
      return rc;
    }, {prev});
    if (TSl) prev = add_T_blocks(P, *TSl, k, k + 1, kfl, tk, nb, prev);
    if (prev < -1) return false;
    // rows k+1.. of columns k+1..: C := C Q_r (A(k, k+1:) = R^H Q_r^H)
    prev = add_right_from(P, A, k + 1, k + 1, kfl, v, ldv, tk, false, w, w2, ldv, prev);
    if (prev < -1) return false;
  }
  if (Band) {   // upper band storage: Band(nb + i - j, j) = A(i, j), max(0, j - nb) <= i <= j
    const int N = std::min(A.m, A.n), ldB = Band->lld;
    char* bd = Band->data;
    prev = P.task(1, [=](hipStream_t s) {
      if (hipMemsetAsync(bd, 0, (size_t)ldB * std::max(1, Band->n) * es, s) != hipSuccess) return -1;
      for (int j = 0; j < std::min(N, nb); ++j)
        if (hipMemcpyAsync(bd + ((size_t)j * ldB + (nb - j)) * es, a + (size_t)j * ld * es, (size_t)(j + 1) * es,
                           hipMemcpyDeviceToDevice, s) != hipSuccess)
          return -1;
      if (N > nb &&
          hipMemcpy2DAsync(bd + (size_t)nb * ldB * es, (size_t)ldB * es, a + ((size_t)nb * ld) * es, (size_t)(ld + 1) * es,
                           (size_t)(nb + 1) * es, N - nb, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return -1;
      return 0;
    }, {prev});
  }
  last = prev;
  return true;
}

bool tree_is_flat(const nq::Tree* t) {
  if (!t) return true;
  for (int k = 0; k < std::min(t->mt, t->nt); ++k) {
    std::vector<int> h;
    std::vector<nq::Kill> kl;
    t->plan(k, h, kl);
    if (h.size() != 1 || h[0] != k) return false;
    for (const nq::Kill& x : kl)
      if (x.piv != k || x.type != nq::KILLED_BY_TS) return false;
  }
  return true;
}

bool band_ok(const NatDesc* A, const NatDesc* Band) {
  return !Band || (Band->m >= A->nb + 1 && Band->n >= std::min(A->m, A->n) && Band->prec == A->prec);
}

}  // namespace

NatProgram* nat_gebrd_ge2gb(dplasma_context_t* ctx, int prec, int ib, dplasma_desc_t* dA, dplasma_desc_t* dBand) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *Band = dBand ? dBand->nat : nullptr;
  if (!same_ctx(c, {A}, prec) || (Band && Band->ctx != c)) return fail(nullptr, "gebrd_ge2gb: descriptors of this context");
  if (A->m < A->n || A->mb != A->nb || A->nb > 256 || ib <= 0 || !band_ok(A, Band))
    return fail(nullptr, "gebrd_ge2gb: M >= N, square tiles <= 256, Band of (nb + 1) x N");
  NatProgram* P = new_program(c, "gebrd_ge2gb", true);
  int last = -1;
  if (!P->info || !add_ge2gb(*P, *A, nullptr, nullptr, Band, last)) return fail(P, "gebrd_ge2gb: device allocation failed");
  return P;
}

// ge2gbx: the trees must be flat (every panel one TS domain: the engine above); TS0 receives the QR steps' T blocks
// (tile (k, k)), TS the LQ steps' (tile (k, k + 1)); TT0 / TT stay untouched (no TT kills in a flat tree)
NatProgram* nat_gebrd_ge2gbx(dplasma_context_t* ctx, int prec, int ib, dplasma_qrtree_t* qt0, dplasma_qrtree_t* qt,
                             dplasma_qrtree_t* lqt, dplasma_desc_t* dA, dplasma_desc_t* dTS0, dplasma_desc_t*,
                             dplasma_desc_t* dTS, dplasma_desc_t*, dplasma_desc_t* dBand) {
  NatCtx* c = ctx->nat;
  NatDesc *A = dA ? dA->nat : nullptr, *Band = dBand ? dBand->nat : nullptr;
  NatDesc *TS0 = dTS0 ? dTS0->nat : nullptr, *TS = dTS ? dTS->nat : nullptr;
  if (!same_ctx(c, {A}, prec) || (Band && Band->ctx != c)) return fail(nullptr, "gebrd_ge2gbx: descriptors of this context");
  const nq::Tree* tq = nat_qrtree(qt ? qt : qt0);
  const nq::Tree* tl = nat_qrtree(lqt);
  if ((qt || qt0) && !tq) return fail(nullptr, "gebrd_ge2gbx: native trees (dplasma_hqr_init on a native descriptor)");
  if (!tree_is_flat(tq) || !tree_is_flat(tl))
    return fail(nullptr, "gebrd_ge2gbx: the native engine reduces with flat trees (one TS domain per panel)");
  if (A->m < A->n || A->mb != A->nb || A->nb > 256 || ib <= 0 || !band_ok(A, Band))
    return fail(nullptr, "gebrd_ge2gbx: M >= N, square tiles <= 256, Band of (nb + 1) x N");
  NatProgram* P = new_program(c, "gebrd_ge2gbx", true);
  int last = -1;
  if (!P->info || !add_ge2gb(*P, *A, TS0, TS, Band, last)) return fail(P, "gebrd_ge2gbx: device allocation failed");
  return P;
}

// tau_j = T_k(j, j) of a native geqrf's T (the compact-WY diagonal: LAPACK's tau), j < k, to host memory
int nat_qr_tau(dplasma_desc_t* dT, void* tau, int k) {
  NatDesc* T = dT ? dT->nat : nullptr;
  if (!T || !T->fullT || k <= 0) return -1;
  const int nb = T->fullT_nb, es = T->es;
  if ((k + nb - 1) / nb > T->fullT_kt) return -1;
  for (int p = 0; p * nb < k; ++p) {
    const int c = std::min(nb, k - p * nb);
    if (hipMemcpy2D((char*)tau + (size_t)p * nb * es, es, (const char*)T->fullT->p + (size_t)p * nb * nb * es,
                    (size_t)(nb + 1) * es, es, c, hipMemcpyDefault) != hipSuccess)
      return -1;
  }
  return 0;
}

// ||A||_2 estimate by power iteration on A^H A (dplasma_zlanm2, src/zlanm2.jdf; the same loop as
// models/aux.lanm2): x = n^-1/2 (1, .., 1); y = A x; x = A^H y; e = ||x|| / ||y||; x /= ||x||, until e moves by
// less than 1e-10 relatively (at most 500 products).  *info: the iteration count, negative if not converged.
// dplasma_zpltmg (models/generators.py pltmg; reference src/cores/core_zpltmg.c): the closed-form LAWN-263
// types, evaluated per tile on the host from GLOBAL indices (identical for any tiling) and copied into the tile;
// Random is the native plrnt; the random-vector types (house, circul, hankel, compan, fiedler, toeppd, condex,
// demmel, langou: core_zpltmg_{circul,condex,fiedler,hankel,toeppd}.c, zpltmg_*.jdf) build their O(n) vectors
// once from the same 64-bit LCG stream as plrnt (PltmgVec below); the types the reference lacks return -2.
static bool pltmg_value(int t, long long I, long long J, long long gM, long long gN, double& v) {
  const double If = (double)I, Jf = (double)J, Ii = If + 1.0, Ji = Jf + 1.0;
  switch (t) {
    case 1: {   // hadamard
      long long x = I & J;
      int pc = 0;
      while (x > 0) pc += (int)(x & 1), x >>= 1;
      v = 1.0 - 2.0 * (pc % 2);
      return true;
    }
    case 3: v = 1.0 / (If - Jf + 0.5); return true;                          // parter
    case 4: v = 0.5 / ((double)gM - If - Jf - 0.5); return true;             // ris
    case 5: v = std::pow(0.5, std::fabs(If - Jf)); return true;              // kms
    case 8: v = I == J ? If + 1.0 : std::min(If, Jf) - 1.0; return true;     // moler
    case 18: v = (J + 2) % (I + 2) == 0 ? (double)(I + 1) : -1.0; return true;   // riemann
    case 22: v = Jf >= If ? Ii / Ji : Ji / Ii; return true;                  // lehmer
    case 24: v = std::min(Ii, Ji); return true;                              // minij
    case 31: v = Ji <= Ii ? Ji : -Ii; return true;                           // invhess
    case 34: v = 1.0 / (Ii + Ji); return true;                               // cauchy
    case 35: v = 1.0 / (If + Jf + 1.0); return true;                         // hilb
    case 36: v = I == 0 ? 1.0 : 1.0 / (If + Jf + 1.0); return true;          // lotkin
    case 38: {                                                               // orthog
      const double sc = M_PI / ((double)gN + 1.0);
      v = std::sqrt(2.0 / ((double)gN + 1.0)) * std::sin(Ii * Ji * sc);
      return true;
    }
    case 39: {                                                               // wilkinson
      const double dist = (double)std::min(gN - 1 - I, I);
      v = I == J ? ((double)gN - 2.0 * dist - 1.0) / 2.0 : (std::llabs(I - J) == 1 ? 1.0 : 0.0);
      return true;
    }
    case 40: {                                                               // foster (k = h = c = 1)
      const double k = 1.0, h = 1.0, c = 1.0;
      if (I == J) v = J == 0 ? 1.0 : J == gN - 1 ? 1 - 1 / c - k * h / 2 : 1 - k * h / 2;
      else v = J == 0 ? -k * h / 2 : J == gN - 1 ? -1 / c : I > J ? -k * h : 0.0;
      return true;
    }
    case 41: {                                                               // wright
      v = I == J ? 1.0 : 0.0;
      const bool even = J % 2 == 0;
      if (I == J + 2) v = even ? -0.9048 : -0.8270;
      if (I == J + 3) v = even ? -1.2092 : -1.3499;
      if (J == gM - 2 && I == 0) v = 1.0;
      if (J == gM - 1 && I == 1) v = 1.0;
      return true;
    }
    case 28: {                                                               // dorr
      const double theta = 0.01, h = 1.0 / ((double)gN + 1.0), term = theta / (h * h);
      const long long half = (gN + 1) / 2;
      const bool lo = J < half;
      if (I == J) v = lo ? 2 * term + (0.5 - (Jf + 1) * h) / h : 2 * term - (0.5 - (Jf + 1) * h) / h;
      else if (I == J - 1) v = (lo || J == half) ? -term - (0.5 - Jf * h) / h : -term;
      else if (I == J + 1) v = lo ? (J + 1 == half ? -term + (0.5 - (Jf + 2) * h) / h : -term)
                                  : -term + (0.5 - (Jf + 2) * h) / h;
      else v = 0.0;
      return true;
    }
    case 30: {                                                               // chebvand
      const double p = Jf * (gN > 1 ? 1.0 / ((double)gN - 1.0) : 0.0);
      double T0 = 1.0, T1 = p;
      if (I == 0) { v = T0; return true; }
      for (long long k = 2; k <= I; ++k) {
        const double T2 = 2 * p * T1 - T0;
        T0 = T1, T1 = T2;
      }
      v = T1;
      return true;
    }
    default: return false;
  }
}

// the plrnt stream on the host (csrc/kernels/aux.hip, utils/lcg.py): element (I, J) of a gM-row matrix is the
// LCG state after I + J gM (complex: 2 (I + J gM)) steps from the seed, value 0.5f - ran * 2^-64 in float
static unsigned long long lcg_jump(unsigned long long n, unsigned long long seed) {
  unsigned long long a = 6364136223846793005ULL, c = 1ULL, ran = seed;
  while (n) {
    if (n & 1ULL) ran = a * ran + c;
    c *= a + 1ULL;
    a *= a;
    n >>= 1;
  }
  return ran;
}
static double lcg_val(unsigned long long ran) { return (double)(0.5f - (float)ran * 5.4210108624275222e-20f); }
static std::complex<double> plrnt_at(unsigned long long idx, unsigned long long seed, bool cplx) {
  if (!cplx) return lcg_val(lcg_jump(idx, seed));
  const unsigned long long r = lcg_jump(2ULL * idx, seed);
  return {lcg_val(r), lcg_val(6364136223846793005ULL * r + 1ULL)};
}

// per-call state of the random-vector types (models/generators.py _formula, the same definitions)
struct PltmgVec {
  int t = 0;
  long long gM = 0, gN = 0;
  bool cplx = false;
  double eps = 0, tau = 0;
  unsigned long long seed = 0;
  std::vector<std::complex<double>> v;   // the random vector (circul / fiedler / hankel / house / compan)
  std::vector<double> tv;                // toeppd: t(d), d = -(n-1) .. n-1
  long long z = 0;
  std::vector<std::complex<double>> Q;   // condex: orthonormal basis (gM x 3, column-major)

  bool init(int type, long long m, long long n, int prec, unsigned long long sd) {
    t = type, gM = m, gN = n, seed = sd;
    cplx = prec == P_C || prec == P_Z;
    eps = (prec == P_S || prec == P_C) ? 1.1920928955078125e-07 : 2.220446049250313e-16;
    auto rv = [&](long long len) {            // the first column of a len-row plrnt matrix
      v.resize((size_t)len);
      for (long long i = 0; i < len; ++i) v[(size_t)i] = plrnt_at((unsigned long long)i, seed, cplx);
    };
    switch (t) {
      case 9: rv(gN); return true;                          // circul
      case 27: rv(std::max(gM, gN)); return true;           // fiedler
      case 12: rv(gM + gN); return true;                    // hankel
      case 2: {                                             // house: I - tau v v^H, tau = 2 / ||v||^2
        rv(gM);
        double s2 = 0;
        for (auto& x : v) s2 += std::norm(x);
        tau = 2.0 / s2;
        return true;
      }
      case 14: {                                            // compan: first row r / r(0)
        rv(gN);
        const std::complex<double> v0 = v[0];
        for (auto& x : v) x /= v0;
        return true;
      }
      case 23: {                                            // toeppd: t(d) = sum_k w_k cos(theta_k d)
        std::vector<double> w((size_t)gM), th((size_t)gM);
        for (long long k = 0; k < gM; ++k) {                // a 2-row plrnt matrix: row 0 -> w, row 1 -> theta
          w[(size_t)k] = plrnt_at((unsigned long long)(2 * k), seed, cplx).real() + 0.5;
          th[(size_t)k] = 2.0 * M_PI * (plrnt_at((unsigned long long)(1 + 2 * k), seed, cplx).real() + 0.5);
        }
        const long long nn = std::max(gM, gN);
        z = nn - 1;
        tv.assign((size_t)(2 * nn - 1), 0.0);
        for (long long d = 0; d < nn; ++d) {
          double acc = 0;
          for (long long k = 0; k < gM; ++k) acc += w[(size_t)k] * std::cos(th[(size_t)k] * (double)d);
          tv[(size_t)(z + d)] = tv[(size_t)(z - d)] = acc;   // cos is even
        }
        return true;
      }
      case 7: {                                             // condex: Q = orth([1, e_1, x]), x_i = (-1)^i (1 + i/(n-1))
        const long long n_ = gM;
        Q.assign((size_t)(3 * n_), 0.0);
        for (long long i = 0; i < n_; ++i) {
          Q[(size_t)i] = 1.0;
          Q[(size_t)(2 * n_ + i)] = ((i & 1) ? -1.0 : 1.0) * (1.0 + (double)i / (double)std::max<long long>(gN - 1, 1));
        }
        Q[(size_t)n_] = 1.0;
        for (int c = 0; c < 3; ++c)                          // modified Gram-Schmidt, twice: the projector
          for (int pass = 0; pass < 2; ++pass) {             // Q Q^H is what the formula uses (sign-free)
            std::complex<double>* qc = &Q[(size_t)c * n_];
            for (int b = 0; b < c; ++b) {
              const std::complex<double>* qb = &Q[(size_t)b * n_];
              std::complex<double> d = 0;
              for (long long i = 0; i < n_; ++i) d += std::conj(qb[i]) * qc[i];
              for (long long i = 0; i < n_; ++i) qc[i] -= d * qb[i];
            }
            double nr = 0;
            for (long long i = 0; i < n_; ++i) nr += std::norm(qc[i]);
            nr = std::sqrt(nr);
            if (!(nr > 0)) return false;
            for (long long i = 0; i < n_; ++i) qc[i] /= nr;
          }
        return true;
      }
      case 29: case 42: return true;                        // demmel, langou: the plrnt base per element
      default: return false;
    }
  }

  std::complex<double> at(long long I, long long J) const {
    switch (t) {
      case 9: return v[(size_t)(((J - I) % gN + gN) % gN)];
      case 27: return std::abs(v[(size_t)I] - v[(size_t)J]);
      case 12: return v[(size_t)(I + J)];
      case 2: return (I == J ? 1.0 : 0.0) - tau * v[(size_t)I] * std::conj(v[(size_t)J]);
      case 14:
        if (I == 0) return J == 0 ? std::complex<double>(0.0) : v[(size_t)std::min(J, gN - 1)];
        return I == J + 1 ? 1.0 : 0.0;
      case 23: return tv[(size_t)(I - J + z)];
      case 7: {
        const double theta = 100.0;
        std::complex<double> s = 0;
        for (int c = 0; c < 3; ++c) s += Q[(size_t)c * gM + I] * std::conj(Q[(size_t)c * gM + J]);
        return (I == J ? 1.0 + theta : 0.0) - theta * s;
      }
      case 29: {
        const std::complex<double> b = plrnt_at((unsigned long long)(I + J * gM), seed, cplx);
        return b * (std::pow(10.0, 14.0 * (double)I / (double)gM) * (I == J ? 1.0 : 1e-7));
      }
      case 42: {
        const std::complex<double> b = plrnt_at((unsigned long long)(I + J * gM), seed, cplx);
        const long long mn = std::min(gM, gN);
        return (J >= mn / 4 && J < mn / 2 && I >= J) ? b * eps : b;
      }
      default: return 0.0;
    }
  }
};

int nat_pltmg(dplasma_context_t* ctx, int prec, int mtxtype, dplasma_desc_t* dA, unsigned long long seed) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return (fail(nullptr, "pltmg: a descriptor of another context or precision"), -1);
  if (mtxtype == 0) return nat_execute(ctx, nat_plrnt(ctx, prec, 0, dA, seed));
  double probe;
  PltmgVec pv;
  const bool closed = pltmg_value(mtxtype, 0, 0, std::max(A->m, 1), std::max(A->n, 1), probe);
  if (!closed && !(A->m > 0 && A->n > 0 && pv.init(mtxtype, A->m, A->n, prec, seed)))
    return (fail(nullptr, "pltmg: matrix type not available (the reference lacks it)"), -2);
  if (mtxtype == 1 && (A->m != A->n || (A->m & (A->m - 1)))) return -2;   // hadamard: n a power of two
  for (int q = 0; q < NAT_NSTREAM; ++q)
    if (hipStreamSynchronize(c->st[q]) != hipSuccess) return -1;
  std::vector<char> h((size_t)A->mb * A->nb * A->es);
  for (int j = 0; j < A->nt; ++j)
    for (int i = 0; i < A->mt; ++i) {
      if (!A->local(i, j)) continue;
      const int r = A->rows(i), cc = A->cols(j);
      std::fill(h.begin(), h.end(), 0);
      for (int jj = 0; jj < cc; ++jj)
        for (int ii = 0; ii < r; ++ii) {
          const long long I = (long long)i * A->mb + ii, J = (long long)j * A->nb + jj;
          std::complex<double> z = 0.0;
          if (closed) {
            double v = 0.0;
            pltmg_value(mtxtype, I, J, A->m, A->n, v);
            z = v;
          } else {
            z = pv.at(I, J);
          }
          char* e = &h[((size_t)ii + (size_t)jj * r) * A->es];
          if (prec == P_S || prec == P_C) {
            const float f[2] = {(float)z.real(), (float)z.imag()};
            std::memcpy(e, f, (prec == P_C ? 2 : 1) * sizeof(float));
          } else {
            const double d[2] = {z.real(), z.imag()};
            std::memcpy(e, d, (prec == P_Z ? 2 : 1) * sizeof(double));
          }
        }
      if (hipMemcpy2D(A->data + A->off(i, j) * A->es, (size_t)A->lld * A->es, h.data(), (size_t)r * A->es,
                      (size_t)r * A->es, cc, hipMemcpyHostToDevice) != hipSuccess)
        return (fail(nullptr, "pltmg: copy to the device failed"), -1);
    }
  return 0;
}

// dplasma_zlatms (models/generators.py latms): singular values D(i) = 1 - i/(N-1) (1 - 1/cond) (D(0) = 1) on
// the diagonal, then A = Q1 D Q2 (General) or Q D Q^H (symmetric / Hermitian) with the random unitary factors of
// native geqrf's of plrnt matrices (seeds seed, seed + 1), applied by native unmqr.  One process.
int nat_latms(dplasma_context_t* ctx, int prec, int mtxtype, double cond, dplasma_desc_t* dA, unsigned long long seed) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx(c, {A}, prec)) return (fail(nullptr, "latms: a descriptor of another context (one process)"), -1);
  if (A->mb != A->nb || A->nb > 256 || !(cond > 0.0))
    return (fail(nullptr, "latms: square tiles <= 256 (the native geqrf) and cond > 0"), -1);
  const int n = A->n;
  const double tmp = 1.0 / cond, alp = n > 1 ? (1.0 - tmp) / (n - 1) : 0.0;
  double z2[2] = {0.0, 0.0};
  float zf[2] = {0.0f, 0.0f};
  const void* zero = (prec == P_D || prec == P_Z) ? (const void*)z2 : (const void*)zf;
  int rc = nat_execute(ctx, nat_laset(ctx, prec, UPPERLOWER, zero, zero, dA));
  if (rc != 0) return rc;
  // the diagonal: one strided host-to-device copy per diagonal tile (pitch lld + 1 elements)
  const int kd = std::min(A->m, A->n);
  std::vector<char> hd((size_t)std::max(kd, 1) * A->es, 0);
  for (int i = 0; i < kd; ++i) {
    const double d = i == 0 ? 1.0 : (n - i - 1) * alp + tmp;
    if (prec == P_S || prec == P_C) {
      const float f = (float)d;
      std::memcpy(&hd[(size_t)i * A->es], &f, sizeof f);
    } else {
      std::memcpy(&hd[(size_t)i * A->es], &d, sizeof d);
    }
  }
  for (int k = 0; k * A->mb < kd; ++k) {
    const int len = std::min(A->mb, kd - k * A->mb);
    if (hipMemcpy2D(A->data + A->off(k, k) * A->es, (size_t)(A->lld + 1) * A->es, &hd[(size_t)k * A->mb * A->es], A->es,
                    A->es, len, hipMemcpyHostToDevice) != hipSuccess)
      return (fail(nullptr, "latms: diagonal copy failed"), -1);
  }
  const int ib = std::min(32, A->nb);
  auto qfactor = [&](int rows, unsigned long long sd, dplasma_desc_t*& Q, dplasma_desc_t*& T) {
    Q = nat_desc(ctx, prec, A->nb, A->nb, rows, rows, 1, 1, nullptr, 0, 1);
    const int mt = (rows + A->nb - 1) / A->nb;
    T = nat_desc(ctx, prec, ib, A->nb, mt * ib, rows, 1, 1, nullptr, 0, 1);
    if (!Q || !T) return -1;
    int e = nat_execute(ctx, nat_plrnt(ctx, prec, 0, Q, sd));
    return e ? e : nat_execute(ctx, nat_geqrf(ctx, prec, Q, T));
  };
  dplasma_desc_t *Q1 = nullptr, *T1 = nullptr, *Q2 = nullptr, *T2 = nullptr;
  rc = qfactor(A->m, seed, Q1, T1);
  if (rc == 0) rc = nat_execute(ctx, nat_unmqr(ctx, prec, LEFT, NOTRANS, Q1, T1, dA));
  if (rc == 0) {
    if (mtxtype == 231 /* dplasmaGeneral */) {
      rc = qfactor(A->n, seed + 1, Q2, T2);
      if (rc == 0) rc = nat_execute(ctx, nat_unmqr(ctx, prec, RIGHT, NOTRANS, Q2, T2, dA));
    } else {
      rc = nat_execute(ctx, nat_unmqr(ctx, prec, RIGHT, (prec == P_C || prec == P_Z) ? CONJTRANS : TRANS, Q1, T1, dA));
    }
  }
  for (dplasma_desc_t* d : {Q1, T1, Q2, T2})
    if (d) nat_desc_free(d), delete d;
  return rc;
}

double nat_lanm2(dplasma_context_t* ctx, int prec, dplasma_desc_t* dA, int* info) {
  NatCtx* c = ctx->nat;
  NatDesc* A = dA ? dA->nat : nullptr;
  if (!same_ctx_dist(c, {A}, prec)) return (fail(nullptr, "lanm2: descriptor of another context or precision"), NAN);
  if (c->dist()) return (fail(nullptr, "lanm2: one process only on a native context"), NAN);
  dplasma_desc_t* X = nat_desc(ctx, prec, A->nb, A->nb, A->n, 1, 1, 1, nullptr, 0, 1);
  dplasma_desc_t* Y = nat_desc(ctx, prec, A->mb, A->nb, A->m, 1, 1, 1, nullptr, 0, 1);
  if (!X || !Y) {
    if (X) nat_desc_free(X), delete X;
    if (Y) nat_desc_free(Y), delete Y;
    return (fail(nullptr, "lanm2: device allocation failed"), NAN);
  }
  const bool cplx = prec == P_C || prec == P_Z;
  auto scal = [&](double v, double buf[2], float fbuf[2]) -> const void* {
    buf[0] = v, buf[1] = 0.0, fbuf[0] = (float)v, fbuf[1] = 0.0f;
    return (prec == P_D || prec == P_Z) ? (const void*)buf : (const void*)fbuf;
  };
  double b1[2], b0[2], bs[2];
  float f1[2], f0[2], fs[2];
  const void* one = scal(1.0, b1, f1);
  const void* zero = scal(0.0, b0, f0);
  const double x0 = 1.0 / std::sqrt((double)std::max(A->n, 1));
  double bx[2];
  float fx[2];
  const void* xv = scal(x0, bx, fx);
  int rc = nat_execute(ctx, nat_laset(ctx, prec, UPPERLOWER, xv, xv, X));
  if (rc == 0) rc = nat_execute(ctx, nat_laset(ctx, prec, UPPERLOWER, zero, zero, Y));
  double e = 0.0, e0 = -1.0;
  int it = 0;
  bool ok = rc == 0;
  while (ok && it < 500 && std::fabs(e - e0) > 1e-10 * std::max(e, 1e-300)) {
    e0 = e;
    ok = nat_execute(ctx, nat_gemm(ctx, prec, NOTRANS, NOTRANS, one, dA, X, zero, Y)) == 0 &&
         nat_execute(ctx, nat_gemm(ctx, prec, cplx ? CONJTRANS : TRANS, NOTRANS, one, dA, Y, zero, X)) == 0;
    if (!ok) break;
    const double nx = nat_lange(ctx, prec, 174 /* Frobenius */, X), ny = nat_lange(ctx, prec, 174, Y);
    if (!(nx > 0.0) || !(ny > 0.0)) {
      e = 0.0;
      break;
    }
    e = nx / ny;
    ok = nat_execute(ctx, nat_lascal(ctx, prec, UPPERLOWER, scal(1.0 / nx, bs, fs), X)) == 0;
    ++it;
  }
  nat_desc_free(X), delete X;
  nat_desc_free(Y), delete Y;
  if (!ok) return NAN;
  if (info) *info = std::fabs(e - e0) <= 1e-10 * std::max(e, 1e-300) ? it : -it;
  return e;
}
