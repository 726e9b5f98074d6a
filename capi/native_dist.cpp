// Multi-process native engine: Cholesky and SUMMA GEMM over a P x Q grid of ranks (one process per
// GPU), compiled in C++ into stream programs exactly like the one-process engine (native.cpp), with the
// tile traffic as grouped point-to-point exchanges on the context's communication stream
// (native_comm.h).  No Python anywhere: this is the C library a ScaLAPACK program links against.
//
// POTRF (reference: src/zpotrf_L.jdf / zpotrf_U.jdf -- POTRF(k) -> TRSM(m,k) -> HERK/GEMM(m,n,k)
// with the tiles travelling along the JDF's remote edges):
//   step k:  POTRF(k) on the owner of the diagonal tile (panel stream)
//            -> DIAG exchange: the factor to the ranks holding panel tiles (communication stream)
//            -> TRSM of this rank's panel tiles, one batched launch; pack them into the panel slots
//            -> PANEL exchange: every panel tile to exactly the ranks whose trailing tiles read it
//            -> NEXT (the trailing tiles of column k+1, panel stream) and REST (all others, update
//               stream): one MFMA GEMM launch each, A and B operands read from the panel slots.
//   Look-ahead 1: POTRF(k+1) needs NEXT(k) and REST(k-1) only, so step k+1's panel, its exchanges and
//   its TRSM run beside REST(k) -- the critical-path role of the reference's high_priority POTRF /
//   TRSM classes.  Panel slots are double-buffered by step parity.
// GEMM (reference: src/zgemm_NN_summa.jdf and the SUMMA variants): per chunk of kc k-steps, the owners
//   pack their op(A)(m, k) / op(B)(k, n) tiles, one exchange sends each to the ranks holding a C tile of
//   its block row / column, and one GEMM launch covers every local C tile with k-runs over the chunk;
//   chunk c+1's pack and exchange overlap chunk c's GEMM (double-buffered).
#include <algorithm>
#include <cstring>
#include <set>

#include "native_comm.h"
#include "native_internal.h"

namespace {

struct CopyBatch {   // packs local tiles into contiguous slots: one dpl_geadd (copy) launch
  std::vector<TileItem> it;
  int mm = 0, nn = 0;
  DevPtr d;
  void add(long long src, long long dst, int m, int n) {
    it.push_back(TileItem{src, dst, m, n, 0, 0});
    mm = std::max(mm, m);
    nn = std::max(nn, n);
  }
  bool upload(NatProgram& P) {
    if (it.empty()) return true;
    d = dev_upload(it);
    if (!d) return false;
    P.keep.push_back(d);
    return true;
  }
  int launch(int prec, const char* A, int lda, char* B, int ldb, hipStream_t s) const {
    if (it.empty()) return 0;
    const Scalar one(prec, 1.0), zero(prec, 0.0);
    return dpl_geadd(prec, 0, NOTRANS, (int)it.size(), d->p, mm, nn, one.ptr(), A, lda, zero.ptr(), B, ldb, 1, s);
  }
};

// one exchange task: the messages are fixed when the program is built
int add_exchange(NatProgram& Pr, std::vector<NatMsg> sends, std::vector<NatMsg> recvs, std::initializer_list<int> deps) {
  if (sends.empty() && recvs.empty()) return -1;
  NatComm* comm = Pr.ctx->comm;
  auto s = std::make_shared<std::vector<NatMsg>>(std::move(sends));
  auto r = std::make_shared<std::vector<NatMsg>>(std::move(recvs));
  return Pr.task(2, [=](hipStream_t st) { return comm->exchange(*s, *r, st); }, deps);
}

int either(int a, int b) { return a >= 0 ? a : b; }

int last_task_on(const NatProgram& P, int stream) {
  for (int i = (int)P.tasks.size() - 1; i >= 0; --i)
    if (P.tasks[i].stream == stream) return i;
  return -1;
}

}  // namespace

// ---------------------------------------------------------------------------------------------- POTRF
// The schedule of models/potrf_dist.py (the one tools/replay_potrf.py chose: profiles/r3_replay_*), in C++:
// panels in blocks of D (DPLASMA_POTRF_DEFER, default 2; D = 1 once fewer than 24 columns remain), and
// per panel k of block b = [c0, c1):
//   POTRF(k) on the diagonal owner (panel stream 0)
//   -> DIAG exchange: the factor to the other ranks holding panel tiles (communication stream 2)
//   -> TRSM of this rank's panel tiles (one launch), packed into panel k's slab
//   -> PANEL exchange: each tile from its owner straight to the ranks whose trailing tiles read it
//   -> NEAR(k): the rest of block b's columns (panel stream)
// and per block b, with every panel of the block in the k-runs (GEMM K = D x NB):
//   NEXT(b)  the columns of block b+1 (panel stream: the critical path),
//   NEXT2(b) the columns of block b+2 and REST2(b) everything beyond (update stream 1)
// -- look-ahead 2: block b+1's panels run beside REST2(b-1) / NEXT2(b), the role of the reference's
// high_priority POTRF / TRSM classes (src/zpotrf_L.jdf:58-69).  Panel slabs rotate over 3 blocks.
NatProgram* nat_dist_potrf(NatCtx* c, int uplo, NatDesc& A) {
  const int prec = A.prec, nt = A.nt, mb = A.mb, es = A.es, me = c->rank, Pg = A.P, Qg = A.Q;
  const bool lower = uplo == LOWER;
  NatProgram* Pr = new_program(c, "potrf", true);
  if (!Pr->info) return fail(Pr, "potrf: device allocation failed");
  const int D = std::max(1, env_int("DPLASMA_POTRF_DEFER", 2)), min_tiles = env_int("DPLASMA_POTRF_DEFER_MIN_TILES", 24);
  std::vector<std::pair<int, int>> blocks;
  for (int c0 = 0; c0 < nt;) {
    const int d = nt - c0 >= min_tiles ? D : 1;
    blocks.push_back({c0, std::min(nt, c0 + d)});
    c0 += d;
  }
  const int NSLAB = 3;
  const size_t slot_elems = (size_t)mb * mb, slab_elems = (size_t)D * std::max(1, nt) * slot_elems;
  DevPtr W = dev_alloc(NSLAB * slab_elems * es, false);
  if (!W) return fail(Pr, "potrf: panel slabs: device allocation failed");
  Pr->keep.push_back(W);
  // loopback (NatCtx::loop): the owner stages what it sends to itself in LB (laid out like W)
  const bool loop = c->loop;
  DevPtr LBw;
  if (loop) {
    LBw = dev_alloc(NSLAB * slab_elems * es, false);
    if (!LBw) return fail(Pr, "potrf: loopback slabs: device allocation failed");
    Pr->keep.push_back(LBw);
  }
  // panel k's slab: (block parity, position in the block); tile i of the panel at slot i of it
  auto slab = [&](char* base, int b, int k) {
    return base + ((size_t)(b % NSLAB) * D + (k - blocks[b].first)) * std::max(1, nt) * slot_elems * es;
  };
  auto slot = [&](int i) { return (long long)i * (long long)slot_elems; };
  auto tc = [&](int i, int k) { return lower ? std::make_pair(i, k) : std::make_pair(k, i); };
  auto own = [&](int i, int k) { const auto t = tc(i, k); return A.owner(t.first, t.second); };
  // trailing tiles of step k: lower {(m, n): k < n <= m}, upper {(m, n): k < m <= n}; C(m, n) reads
  // panel tiles m and n, so panel tile i goes to the owners of row i and column i of that set
  auto consumers = [&](int k, int i) {
    std::set<int> s;
    const int a0 = lower ? k + 1 : i, a1 = lower ? i + 1 : nt;     // C(i, n), n in [a0, a1)
    const int b0 = lower ? i : k + 1, b1 = lower ? nt : i + 1;     // C(m, i), m in [b0, b1)
    for (int n = a0; n < std::min(a1, a0 + Qg); ++n) s.insert(A.owner(i, n));
    for (int m = b0; m < std::min(b1, b0 + Pg); ++m) s.insert(A.owner(m, i));
    return s;
  };
  const int tA = lower ? NOTRANS : CONJTRANS, tB = lower ? CONJTRANS : NOTRANS;
  const int side = lower ? RIGHT : LEFT, tri_mask = lower ? 1 : 2;
  const Scalar one(prec, 1.0), m_one(prec, -1.0);
  char* base = A.data;
  char* wbase = (char*)W->p;
  char* lbase = loop ? (char*)LBw->p : nullptr;
  const int ld = A.lld;
  int* info = (int*)Pr->info->p;
  const size_t sbytes = slot_elems * es;
  const bool rb = prec == P_D && A.mb == A.nb && A.mb <= 512 && env_int("DPLASMA_NATIVE_RB", 1) == 1;
  const int zsz = rb ? dpl_potrf_zbuf_size() : 0;
  DevPtr zb;
  if (rb) {
    zb = dev_alloc((size_t)2 * zsz * sizeof(double), false);
    if (!zb) return fail(Pr, "potrf: device allocation failed");
    Pr->keep.push_back(zb);
  }
  // GEMM batch of the trailing tiles in columns [n0, n1) (local), k-runs over panels ks (their slabs)
  auto upd = [&](int b, const std::vector<int>& ks, int n0, int n1) {
    auto g = std::make_shared<Gemm>();
    for (int n_ = n0; n_ < n1; ++n_)
      for (int m_ = n_; m_ < nt; ++m_) {
        const int m = lower ? m_ : n_, n = lower ? n_ : m_;
        if (!A.local(m, n)) continue;
        std::vector<KPair> kp;
        for (int k : ks) {
          const long long so = (long long)(slab(wbase, b, k) - wbase) / es;
          kp.push_back(KPair{so + slot(m), so + slot(n), A.rows(k), 0});
        }
        g->add(A.off(m, n), A.rows(m), A.cols(n), kp, m == n ? tri_mask : 0);
      }
    return g;
  };
  auto gemm_task = [&](int stream, std::shared_ptr<Gemm> g, std::initializer_list<int> deps) {
    if (g->empty()) return -1;
    if (!g->upload(*Pr)) return -2;
    return Pr->task(stream, [=](hipStream_t s) {
      return g->launch(prec, tA, tB, m_one, wbase, mb, wbase, mb, one, base, ld, s);
    }, deps);
  };
  const int nbk = (int)blocks.size();
  std::vector<int> next_of(nbk, -1), nxt2_of(nbk, -1), rest_of(nbk, -1), last_xch_of(nbk, -1), last0_of(nbk, -1);
  int xch_prev = -1;   // the latest communication-stream task
  for (int b = 0; b < nbk; ++b) {
    const int c0 = blocks[b].first, c1 = blocks[b].second;
    // every update of block b's columns from earlier blocks: NEXT(b-1) (panel stream, in order), NEXT2(b-2)
    // and REST2(<= b-3) (update stream: REST2(b-3) precedes NEXT2(b-2) there)
    const int upd_in = b >= 2 ? nxt2_of[b - 2] : -1;
    // the slabs of block b were last read by block b-3's updates and sent by its exchanges
    const int slab_free = b >= NSLAB ? rest_of[b - NSLAB] : -1;
    const int slab_sent = b >= NSLAB ? last_xch_of[b - NSLAB] : -1;
    // ... and by its panel-stream tasks (NEAR / NEXT of block b-3 read the same slabs): a rank with no panel or
    // diagonal tile in blocks b-2 and b-1 has no other ordering between those reads and a write into the slab
    const int slab_read = b >= NSLAB ? last0_of[b - NSLAB] : -1;
    for (int k = c0; k < c1; ++k) {
      const int kb = A.rows(k), own_k = A.owner(k, k);
      char* wb = slab(wbase, b, k);
      char* sb = loop ? slab(lbase, b, k) : wb;   // where this rank's outgoing panel data is staged
      int t_diag = -1;
      if (me == own_k) {
        const long long dk = A.off(k, k);
        double* zk = rb ? (double*)zb->p + (size_t)(k % 2) * zsz : nullptr;
        const int t_potrf = Pr->task(0, [=](hipStream_t s) {
          return rb ? dpl_potrf_tile_rbz(uplo, kb, (double*)base + dk, ld, info, k * mb, zk, s)
                    : dpl_potrf_tile(prec, uplo, kb, base, dk, ld, info, k * mb, s);
        }, {upd_in});
        char* dst = sb + slot(k) * es;
        t_diag = Pr->task(0, [=](hipStream_t s) {
          return hipMemcpy2DAsync(dst, (size_t)mb * es, base + dk * es, (size_t)ld * es, (size_t)kb * es, kb,
                                  hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : -1;
        }, {t_potrf, slab_free, slab_sent, slab_read});
      }
      // DIAG exchange: the factor to every other rank holding a panel tile of step k
      std::set<int> drc;
      for (int i = k + 1; i < std::min(nt, k + 1 + (lower ? Pg : Qg)); ++i) drc.insert(own(i, k));
      if (!loop) drc.erase(own_k);
      std::vector<NatMsg> ds, dr;
      if (me == own_k)
        for (int r : drc) ds.push_back(NatMsg{r, sb + slot(k) * es, sbytes});
      if (drc.count(me)) dr.push_back(NatMsg{own_k, wb + slot(k) * es, sbytes});
      const int t_xd = add_exchange(*Pr, ds, dr, {t_diag, slab_free, slab_sent, slab_read, xch_prev});
      if (t_xd >= 0) xch_prev = t_xd;
      // TRSM of this rank's panel tiles against the factor, then pack them into their slots
      auto tr = std::make_shared<Trsm1>();
      auto pk = std::make_shared<CopyBatch>();
      tr->tri = slot(k);
      for (int i = k + 1; i < nt; ++i) {
        const auto t = tc(i, k);
        if (!A.local(t.first, t.second)) continue;
        tr->add(A.off(t.first, t.second), A.rows(t.first), A.cols(t.second));
        pk->add(A.off(t.first, t.second), slot(i), A.rows(t.first), A.cols(t.second));
      }
      int t_pack = -1;
      if (!tr->it.empty() && rb) {
        std::vector<RbItem> strips;   // 16-row strips of this rank's panel tiles
        for (int i = k + 1; i < nt; ++i) {
          const auto t = tc(i, k);
          if (!A.local(t.first, t.second)) continue;
          const int ext = lower ? A.rows(i) : A.cols(i);
          for (int r0 = 0; r0 < ext; r0 += 16)
            strips.push_back(RbItem{A.off(t.first, t.second) + (lower ? r0 : (long long)r0 * ld), std::min(16, ext - r0), 0});
        }
        DevPtr d = dev_upload(strips);
        if (!d || !pk->upload(*Pr)) return fail(Pr, "potrf: device allocation failed");
        Pr->keep.push_back(d);
        const int nrb = (int)strips.size();
        double* zk = (double*)zb->p + (size_t)(k % 2) * zsz;
        const bool ownf = me == own_k && !loop;
        const double* L = ownf ? (const double*)base + A.off(k, k) : (const double*)(wb + slot(k) * es);
        const int ldl = ownf ? ld : mb;
        const int t_trsm = Pr->task(0, [=](hipStream_t s) {
          if (!ownf) {   // the factor came by exchange: invert its 32-blocks here
            const int rc = dpl_trsm_rb_prep(uplo, kb, L, ldl, zk, s);
            if (rc) return rc;
          }
          return dpl_trsm_rb(uplo, kb, L, ldl, zk, nrb, d->p, (double*)base, ld, s);
        }, {either(t_xd, t_diag), upd_in});
        t_pack = Pr->task(0, [=](hipStream_t s) { return pk->launch(prec, base, ld, sb, mb, s); },
                          {t_trsm, slab_free, slab_sent, slab_read});
      } else if (!tr->it.empty()) {
        // the factor from the slab (the owner's copy or the received one), offset relative to the slabs' base
        const long long to = (long long)((wb - wbase) / es) + slot(k);
        for (TileItem& x : tr->it) x.a_off = to;
        tr->tri = to;
        if (!tr->upload(*Pr, prec, side) || !pk->upload(*Pr)) return fail(Pr, "potrf: device allocation failed");
        const int t_trsm = Pr->task(0, [=](hipStream_t s) {
          return tr->launch(prec, side, uplo, CONJTRANS, NONUNIT, one, wbase, mb, base, ld, s);
        }, {either(t_xd, t_diag), upd_in});
        t_pack = Pr->task(0, [=](hipStream_t s) { return pk->launch(prec, base, ld, sb, mb, s); },
                          {t_trsm, slab_free, slab_sent, slab_read});
      }
      // PANEL exchange: tile i from its owner to the ranks whose trailing tiles read it (ascending i:
      // both sides of a pair enumerate their messages in the same order)
      std::vector<NatMsg> ps, pr;
      for (int i = k + 1; i < nt; ++i) {
        const int src = own(i, k);
        std::set<int> cs = consumers(k, i);
        if (!loop) cs.erase(src);
        if (src == me)
          for (int r : cs) ps.push_back(NatMsg{r, sb + slot(i) * es, sbytes});
        if (cs.count(me) && (src != me || loop)) pr.push_back(NatMsg{src, wb + slot(i) * es, sbytes});
      }
      const int t_xp = add_exchange(*Pr, ps, pr, {t_pack, t_xd, slab_free, slab_sent, slab_read, xch_prev});
      if (t_xp >= 0) xch_prev = t_xp;
      last_xch_of[b] = xch_prev;
      // NEAR(k): the rest of this block with panel k (panel stream)
      const int t_in = either(t_xp, either(t_pack, t_xd));
      const int t_near = gemm_task(0, upd(b, {k}, k + 1, c1), {t_in});
      if (t_near == -2) return fail(Pr, "potrf: device allocation failed");
    }
    if (c1 >= nt) break;
    std::vector<int> ks;
    for (int k = c0; k < c1; ++k) ks.push_back(k);
    const int n1 = blocks[b + 1].second, n2 = b + 2 < nbk ? blocks[b + 2].second : nt;
    const int t_in = xch_prev;
    // NEXT(b) (critical): block b+1's columns; they are also written by NEXT2(b-1) and REST2(b-2)
    next_of[b] = gemm_task(0, upd(b, ks, c1, n1), {t_in, b >= 1 ? nxt2_of[b - 1] : -1, b >= 2 ? rest_of[b - 2] : -1});
    if (next_of[b] == -2) return fail(Pr, "potrf: device allocation failed");
    last0_of[b] = last_task_on(*Pr, 0);   // the last panel-stream reader of block b's slabs
    nxt2_of[b] = gemm_task(1, upd(b, ks, n1, n2), {t_in});
    if (nxt2_of[b] == -2) return fail(Pr, "potrf: device allocation failed");
    rest_of[b] = gemm_task(1, upd(b, ks, n2, nt), {t_in});
    if (rest_of[b] == -2) return fail(Pr, "potrf: device allocation failed");
    // (an empty NEXT2 / REST2: the latest update-stream task stands for it)
    const int last1 = last_task_on(*Pr, 1);
    if (nxt2_of[b] < 0) nxt2_of[b] = last1;
    if (rest_of[b] < 0) rest_of[b] = last1;
  }
  return Pr;
}

// ----------------------------------------------------------------------------------------------- GEMM
NatProgram* nat_dist_gemm(NatCtx* c, int prec, int tA, int tB, const Scalar& alpha, NatDesc& A, NatDesc& B,
                          const Scalar& beta, NatDesc& C) {
  NatProgram* Pr = new_program(c, "gemm", false);
  if (!nat_dist_gemm_into(*Pr, prec, tA, tB, alpha, A, B, beta, C, UPPERLOWER))
    return fail(Pr, "gemm: device allocation failed");
  return Pr;
}

// appended to Pr after everything already in it
// tri: UPPERLOWER (every C tile) or LOWER / UPPER (C's triangle only, diagonal tiles masked -- herk / syrk)
bool nat_dist_gemm_into(NatProgram& PrR, int prec, int tA, int tB, const Scalar& alpha, NatDesc& A, NatDesc& B,
                        const Scalar& beta, NatDesc& C, int tri) {
  NatProgram* Pr = &PrR;
  NatCtx* c = Pr->ctx;
  const int es = C.es, me = c->rank;
  const bool an = tA == NOTRANS, bn = tB == NOTRANS;
  const int kt = an ? A.nt : A.mt;
  if (kt == 0)   // C := beta C (restricted to C's triangle when tri says so); no exchange at all
    return nat_add_lascal(*Pr, tri, beta, C);
  const int j0 = last_task_on(*Pr, 0), j1 = last_task_on(*Pr, 1), j2 = last_task_on(*Pr, 2);
  const int kc = std::max(1, std::min(kt, env_int("DPLASMA_NATIVE_SUMMA_K", 4)));
  const size_t sa = (size_t)A.mb * A.nb, sb = (size_t)B.mb * B.nb;   // slots: stored tiles, ld mb
  DevPtr WA = dev_alloc(2 * (size_t)kc * C.mt * sa * es, false), WB = dev_alloc(2 * (size_t)kc * C.nt * sb * es, false);
  if (!WA || !WB) return false;
  Pr->keep.push_back(WA);
  Pr->keep.push_back(WB);
  // loopback (NatCtx::loop): owners pack into LA / LB and send to themselves into WA / WB
  const bool loop = c->loop;
  DevPtr LA, LB;
  if (loop) {
    LA = dev_alloc(2 * (size_t)kc * C.mt * sa * es, false);
    LB = dev_alloc(2 * (size_t)kc * C.nt * sb * es, false);
    if (!LA || !LB) return false;
    Pr->keep.push_back(LA);
    Pr->keep.push_back(LB);
  }
  auto aslot = [&](int kk, int m) { return ((long long)kk * C.mt + m) * (long long)sa; };
  auto bslot = [&](int kk, int n) { return ((long long)kk * C.nt + n) * (long long)sb; };
  // ranks holding a C tile of block row m / block column n
  std::set<int> qs, ps;
  for (int n = 0; n < std::min(C.nt, C.Q); ++n) qs.insert(n % C.Q);
  for (int m = 0; m < std::min(C.mt, C.P); ++m) ps.insert(m % C.P);
  const Scalar one(prec, 1.0);
  const int nch = (kt + kc - 1) / kc;
  std::vector<int> gem(nch, -1), xch(nch, -1);
  for (int ch = 0; ch < nch; ++ch) {
    const int k0 = ch * kc, k1 = std::min(kt, k0 + kc), b = ch % 2;
    char* wa = (char*)WA->p + (size_t)b * kc * C.mt * sa * es;
    char* wb = (char*)WB->p + (size_t)b * kc * C.nt * sb * es;
    char* pa_dst = loop ? (char*)LA->p + (size_t)b * kc * C.mt * sa * es : wa;   // packing targets
    char* pb_dst = loop ? (char*)LB->p + (size_t)b * kc * C.nt * sb * es : wb;
    const int g2 = ch >= 2 ? gem[ch - 2] : -1, x2 = ch >= 2 ? xch[ch - 2] : -1;
    auto pa = std::make_shared<CopyBatch>(), pb = std::make_shared<CopyBatch>();
    std::vector<NatMsg> snd, rcv;
    for (int k = k0; k < k1; ++k)
      for (int m = 0; m < C.mt; ++m) {   // op(A)(m, k): stored tile (m, k) or (k, m)
        const int si = an ? m : k, sj = an ? k : m, src = A.owner(si, sj);
        void* p = wa + aslot(k - k0, m) * es;
        if (src == me) {
          pa->add(A.off(si, sj), aslot(k - k0, m), A.rows(si), A.cols(sj));
          for (int q : qs) {
            const int r = (m % C.P) * C.Q + q;
            if (r != me || loop) snd.push_back(NatMsg{r, pa_dst + aslot(k - k0, m) * es, sa * es});
          }
        }
        if ((src != me || loop) && m % C.P == C.myrow && qs.count(C.mycol)) rcv.push_back(NatMsg{src, p, sa * es});
      }
    for (int k = k0; k < k1; ++k)
      for (int n = 0; n < C.nt; ++n) {   // op(B)(k, n): stored tile (k, n) or (n, k)
        const int si = bn ? k : n, sj = bn ? n : k, src = B.owner(si, sj);
        void* p = wb + bslot(k - k0, n) * es;
        if (src == me) {
          pb->add(B.off(si, sj), bslot(k - k0, n), B.rows(si), B.cols(sj));
          for (int pr : ps) {
            const int r = pr * C.Q + n % C.Q;
            if (r != me || loop) snd.push_back(NatMsg{r, pb_dst + bslot(k - k0, n) * es, sb * es});
          }
        }
        if ((src != me || loop) && n % C.Q == C.mycol && ps.count(C.myrow)) rcv.push_back(NatMsg{src, p, sb * es});
      }
    if (!pa->upload(*Pr) || !pb->upload(*Pr)) return false;
    const char *a = A.data, *bb = B.data;
    const int lda = A.lld, ldb = B.lld, amb = A.mb, bmb = B.mb;
    int t_pack = -1;
    if (!pa->it.empty() || !pb->it.empty())
      t_pack = Pr->task(0, [=](hipStream_t s) {
        const int rc = pa->launch(prec, a, lda, pa_dst, amb, s);
        return rc ? rc : pb->launch(prec, bb, ldb, pb_dst, bmb, s);
      }, {g2, x2, j0, j1, j2});
    const int t_x = add_exchange(*Pr, snd, rcv, {t_pack, g2, j0, j1, j2});
    xch[ch] = either(t_x, ch >= 1 ? xch[ch - 1] : -1);
    auto g = std::make_shared<Gemm>();
    for (int n = C.mycol; n < C.nt; n += C.Q)
      for (int m = C.myrow; m < C.mt; m += C.P) {
        if ((tri == LOWER && m < n) || (tri == UPPER && m > n)) continue;
        std::vector<KPair> kp;
        for (int k = k0; k < k1; ++k) kp.push_back(KPair{aslot(k - k0, m), bslot(k - k0, n), an ? A.cols(k) : A.rows(k), 0});
        g->add(C.off(m, n), C.rows(m), C.cols(n), kp, m == n && tri != UPPERLOWER ? (tri == LOWER ? 1 : 2) : 0);
      }
    if (g->empty()) continue;
    if (!g->upload(*Pr)) return false;
    const Scalar be = ch == 0 ? beta : one;
    char* cc = C.data;
    const int ldc = C.lld;
    gem[ch] = Pr->task(1, [=](hipStream_t s) {
      return g->launch(prec, tA, tB, alpha, wa, amb, wb, bmb, be, cc, ldc, s);
    }, {either(t_x, t_pack), j0, j1, j2});
  }
  return true;
}

// ----------------------------------------------------------------------------------------------- TRSM
// op(A) X = alpha B (left) / X op(A) = alpha B (right) on the grid (reference: src/ztrsm_LLN.jdf and the
// other seven variants): per step k of the solve order, the diagonal tile goes to the ranks holding block
// row (left) / column (right) k of B, they solve it (alpha folded in at the first step) and pack it, one
// exchange sends the solved tiles and op(A)'s panel tiles to the ranks whose remaining B tiles read them,
// and one MFMA GEMM launch updates every remaining local tile (beta = the step's alpha, as the
// one-process engine).  Slots are double-buffered by step parity.  Appended to Pr after everything
// already in it (posv / potrs).
bool nat_dist_trsm_into(NatProgram& Pr, int side, int uplo, int trans, int diag, const Scalar& alpha, NatDesc& A,
                        NatDesc& B) {
  NatCtx* c = Pr.ctx;
  const int prec = B.prec, es = B.es, me = c->rank;
  const bool left = side == LEFT, notrans = trans == NOTRANS;
  const int nk = left ? B.mt : B.nt;
  const bool forward = left ? ((uplo == LOWER) == notrans) : ((uplo == UPPER) == notrans);
  const size_t sa = (size_t)A.mb * A.nb, sbt = (size_t)B.mb * B.nb;
  const int ns = std::max(B.mt, B.nt);
  DevPtr W = dev_alloc(2 * (sa + ns * sa + ns * sbt) * es, false);
  if (!W) return false;
  Pr.keep.push_back(W);
  auto dslot = [&](int par) { return (char*)W->p + (size_t)par * (sa + ns * sa + ns * sbt) * es; };
  auto aoff = [&](int i) { return (long long)(sa + (size_t)i * sa); };                 // elements from dslot
  auto xoff = [&](int i) { return (long long)(sa + (size_t)ns * sa + (size_t)i * sbt); };
  // ranks holding B tiles of block row i / block column j
  std::set<int> bq, bp;
  for (int j = 0; j < std::min(B.nt, B.Q); ++j) bq.insert(j % B.Q);
  for (int i = 0; i < std::min(B.mt, B.P); ++i) bp.insert(i % B.P);
  const Scalar one(prec, 1.0), m_one(prec, -1.0);
  char* bb = B.data;
  const int ldb = B.lld, amb = A.mb, bmb = B.mb;
  // the solve follows everything already in the program (a factorisation, an earlier solve)
  int j0 = -1, j1 = -1, j2 = -1;
  for (int i = (int)Pr.tasks.size() - 1; i >= 0; --i) {
    const int s = Pr.tasks[i].stream;
    if (s == 0 && j0 < 0) j0 = i;
    if (s == 1 && j1 < 0) j1 = i;
    if (s == 2 && j2 < 0) j2 = i;
  }
  std::vector<int> gem(nk, -1), xch(nk, -1);
  int prev_g = -1;
  for (int s = 0; s < nk; ++s) {
    const int k = forward ? s : nk - 1 - s, par = s % 2;
    char* ws = dslot(par);
    const Scalar ak = s == 0 ? alpha : one;
    const int g2 = s >= 2 ? gem[s - 2] : -1, x2 = s >= 2 ? xch[s - 2] : -1;
    const int base_deps[4] = {prev_g, j0, j1, j2};
    // remaining indices of the solve order after k
    std::vector<int> rem;
    for (int r = s + 1; r < nk; ++r) rem.push_back(forward ? r : nk - 1 - r);
    // diagonal tile -> the ranks holding B's block row / column k
    std::set<int> drc;
    if (left) for (int q : bq) drc.insert((k % B.P) * B.Q + q);
    else for (int p : bp) drc.insert(p * B.Q + k % B.Q);
    const int od = A.owner(k, k);
    int t_d = -1;
    if (me == od && !drc.empty()) {
      char* dst = ws;
      const char* src = A.data + A.off(k, k) * es;
      const int lda = A.lld, rk = A.rows(k), ck = A.cols(k);
      t_d = Pr.task(0, [=](hipStream_t st) {
        return hipMemcpy2DAsync(dst, (size_t)amb * es, src, (size_t)lda * es, (size_t)rk * es, ck,
                                hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : -1;
      }, {base_deps[0], base_deps[1], base_deps[2], base_deps[3], g2, x2});
    }
    std::vector<NatMsg> ds, dr;
    if (me == od)
      for (int r : drc)
        if (r != me) ds.push_back(NatMsg{r, ws, sa * es});
    if (me != od && drc.count(me)) dr.push_back(NatMsg{od, ws, sa * es});
    const int t_xd = add_exchange(Pr, ds, dr, {t_d, base_deps[0], base_deps[1], base_deps[2], base_deps[3], g2, x2});
    // solve this rank's tiles of block row / column k, pack them into the X slots
    auto tr = std::make_shared<Trsm1>();
    auto pk = std::make_shared<CopyBatch>();
    tr->tri = 0;
    const int nn = left ? B.nt : B.mt;
    for (int t = 0; t < nn; ++t) {
      const int bi = left ? k : t, bj = left ? t : k;
      if (!B.local(bi, bj)) continue;
      tr->add(B.off(bi, bj), B.rows(bi), B.cols(bj));
      pk->add(B.off(bi, bj), xoff(t), B.rows(bi), B.cols(bj));
    }
    int t_pack = -1;
    if (!tr->it.empty()) {
      if (!tr->upload(Pr, prec, side) || !pk->upload(Pr)) return false;
      const int t_s = Pr.task(0, [=](hipStream_t st) {
        return tr->launch(prec, side, uplo, trans, diag, ak, ws, amb, bb, ldb, st);
      }, {either(t_xd, t_d), base_deps[0], base_deps[1], base_deps[2], base_deps[3]});
      t_pack = Pr.task(0, [=](hipStream_t st) { return pk->launch(prec, bb, ldb, ws, bmb, st); }, {t_s, g2, x2});
    }
    if (rem.empty()) {
      gem[s] = either(t_pack, prev_g);
      prev_g = gem[s];
      xch[s] = either(t_xd, s >= 1 ? xch[s - 1] : -1);
      continue;
    }
    // exchange: solved tiles X(t) and op(A)'s panel tiles (index i in rem) to the ranks that read them
    std::vector<NatMsg> ps, pr;
    std::set<int> remset(rem.begin(), rem.end());
    for (int t = 0; t < nn; ++t) {   // X tile t: left X(k, t) -> ranks (i % P, t % Q), i in rem
      const int bi = left ? k : t, bj = left ? t : k;
      const int src = B.owner(bi, bj);
      std::set<int> cs;
      for (size_t u = 0; u < rem.size() && u < (size_t)(left ? B.P : B.Q); ++u) {
        const int i = rem[u];
        cs.insert(left ? B.owner(i, t) : B.owner(t, i));
      }
      cs.erase(src);
      void* p = ws + xoff(t) * es;
      if (src == me)
        for (int r : cs) ps.push_back(NatMsg{r, p, sbt * es});
      else if (cs.count(me))
        pr.push_back(NatMsg{src, p, sbt * es});
    }
    for (int i : rem) {   // op(A) tile: left op(A)(i, k) -> ranks (i % P, q); right op(A)(k, i) -> ranks (p, i % Q)
      const int si = left ? (notrans ? i : k) : (notrans ? k : i), sj = left ? (notrans ? k : i) : (notrans ? i : k);
      const int src = A.owner(si, sj);
      std::set<int> cs;
      if (left) for (int q : bq) cs.insert((i % B.P) * B.Q + q);
      else for (int p : bp) cs.insert(p * B.Q + i % B.Q);
      void* p = ws + aoff(i) * es;
      const bool need = cs.count(me) > 0;
      cs.erase(src);
      if (src == me) {
        for (int r : cs) ps.push_back(NatMsg{r, p, sa * es});   // (packed below with the other local tiles)
      } else if (need) {
        pr.push_back(NatMsg{src, p, sa * es});
      }
    }
    // pack this rank's op(A) panel tiles that anybody reads
    auto pa = std::make_shared<CopyBatch>();
    for (int i : rem) {
      const int si = left ? (notrans ? i : k) : (notrans ? k : i), sj = left ? (notrans ? k : i) : (notrans ? i : k);
      if (A.owner(si, sj) == me) pa->add(A.off(si, sj), aoff(i), A.rows(si), A.cols(sj));
    }
    int t_pa = -1;
    if (!pa->it.empty()) {
      if (!pa->upload(Pr)) return false;
      const char* ad = A.data;
      const int lda = A.lld;
      t_pa = Pr.task(0, [=](hipStream_t st) { return pa->launch(prec, ad, lda, ws, amb, st); }, {g2, x2, t_pack});
    }
    const int t_xp = add_exchange(Pr, ps, pr, {t_pack, t_pa, t_xd, g2, x2, base_deps[0], base_deps[1], base_deps[2],
                                               base_deps[3]});
    xch[s] = either(t_xp, either(t_xd, s >= 1 ? xch[s - 1] : -1));
    // update the remaining local tiles: left B(i, t) = ak B(i, t) - op(A)(i, k) X(k, t);
    // right B(t, i) = ak B(t, i) - X(t, k) op(A)(k, i)
    auto g = std::make_shared<Gemm>();
    for (int i : rem)
      for (int t = 0; t < nn; ++t) {
        const int bi = left ? i : t, bj = left ? t : i;
        if (!B.local(bi, bj)) continue;
        if (left)
          g->add(B.off(bi, bj), B.rows(bi), B.cols(bj), {KPair{aoff(i), xoff(t), A.rows(k), 0}}, 0);
        else
          g->add(B.off(bi, bj), B.rows(bi), B.cols(bj), {KPair{xoff(t), aoff(i), A.rows(k), 0}}, 0);
      }
    const int t_in = either(t_xp, either(t_pa, either(t_pack, t_xd)));
    if (!g->empty()) {
      if (!g->upload(Pr)) return false;
      const int ta = left ? (notrans ? NOTRANS : trans) : NOTRANS, tb = left ? NOTRANS : (notrans ? NOTRANS : trans);
      // both operands live in this parity's slots (offsets from ws): A slots have ld amb, X slots bmb
      gem[s] = Pr.task(1, [=](hipStream_t st) {
        return left ? g->launch(prec, ta, tb, m_one, ws, amb, ws, bmb, ak, bb, ldb, st)
                    : g->launch(prec, ta, tb, m_one, ws, bmb, ws, amb, ak, bb, ldb, st);
      }, {t_in, prev_g, t_pack});
    } else {
      gem[s] = either(t_in, prev_g);
    }
    prev_g = gem[s];
  }
  return true;
}

// ------------------------------------------------------------------------------------- mirror (symm)
// W(m, n) := op(A(n, m)) for the strict triangle opposite A's stored uplo (op: TRANS / CONJTRANS) -- or for
// every tile with uplo = UPPERLOWER (a distributed transpose: geadd / tradd with op(A)) -- on the
// grid: tiles whose mirror lives on another rank travel in one exchange (every rank walks the stored
// triangle in the same order, so pairs match), then one transposing copy launch per source buffer.
bool nat_dist_mirror_into(NatProgram& Pr, const NatDesc& A, int uplo, int mtrans, NatDesc& W) {
  NatCtx* c = Pr.ctx;
  const int prec = A.prec, es = A.es, me = c->rank;
  const size_t st = (size_t)A.mb * A.nb;
  std::vector<std::pair<int, int>> srcs;   // stored strict-triangle tiles (n, m) in canonical order
  for (int n = 0; n < A.mt; ++n)
    for (int m = 0; m < A.nt; ++m)
      if ((uplo == LOWER && n > m) || (uplo == UPPER && n < m) || uplo == UPPERLOWER) srcs.emplace_back(n, m);
  int nsend = 0, nrecv = 0;
  for (auto [n, m] : srcs) {
    const int so = A.owner(n, m), dt = W.owner(m, n);
    if (so == dt) continue;
    if (so == me) ++nsend;
    if (dt == me) ++nrecv;
  }
  DevPtr S = dev_alloc((size_t)std::max(1, nsend + nrecv) * st * es, false);
  if (!S) return false;
  Pr.keep.push_back(S);
  char* sb = (char*)S->p;
  auto pk = std::make_shared<CopyBatch>(), loc = std::make_shared<CopyBatch>(), rc = std::make_shared<CopyBatch>();
  std::vector<NatMsg> sends, recvs;
  int is = 0, ir = nsend;
  for (auto [n, m] : srcs) {
    const int so = A.owner(n, m), dt = W.owner(m, n);
    if (so == me && dt == me) {
      loc->add(A.off(n, m), W.off(m, n), W.rows(m), W.cols(n));   // (transposing copy: dest-sized item)
    } else if (so == me) {
      pk->add(A.off(n, m), (long long)is * st, A.rows(n), A.cols(m));
      sends.push_back(NatMsg{dt, sb + (size_t)is * st * es, st * es});
      ++is;
    } else if (dt == me) {
      rc->add((long long)ir * st, W.off(m, n), W.rows(m), W.cols(n));
      recvs.push_back(NatMsg{so, sb + (size_t)ir * st * es, st * es});
      ++ir;
    }
  }
  if (!pk->upload(Pr) || !loc->upload(Pr) || !rc->upload(Pr)) return false;
  const int j0 = last_task_on(Pr, 0), j1 = last_task_on(Pr, 1), j2 = last_task_on(Pr, 2);
  const char* a = A.data;
  char* w = W.data;
  const int lda = A.lld, ldw = W.lld, mb = A.mb;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  auto tcopy = [=](std::shared_ptr<CopyBatch> b, const char* src, int lds) {
    return [=](hipStream_t s) {
      if (b->it.empty()) return 0;
      return dpl_geadd(prec, 0, mtrans, (int)b->it.size(), b->d->p, b->mm, b->nn, one.ptr(), src, lds, zero.ptr(), w,
                       ldw, 1, s);
    };
  };
  int t_pk = -1;
  if (!pk->it.empty())
    t_pk = Pr.task(0, [=](hipStream_t s) { return pk->launch(prec, a, lda, sb, mb, s); }, {j0, j1, j2});
  const int t_x = add_exchange(Pr, sends, recvs, {t_pk, j0, j1, j2});
  int last = Pr.task(1, tcopy(loc, a, lda), {j0, j1, j2});
  if (!rc->it.empty()) last = Pr.task(1, tcopy(rc, sb, mb), {last, t_x});
  return true;
}

// ----------------------------------------------------------------------------- F77 redistribution
// A ScaLAPACK operand that does not start at IA = JA = 1 of a matrix distributed from process (0, 0)
// is not a tile-aligned block-cyclic matrix: the reference wrappers redistribute it into an aligned copy
// before running and back afterwards (src/scalapack_wrappers/common.c:27-128).  Same here, between HOST
// local arrays: global rows (columns) of the operand split into runs on which both the source block and
// the aligned copy's block are constant; the message from rank s to rank d is every (column run, column,
// row run) piece owned by s and destined to d, enumerated in the same order on both sides, packed on the
// host, moved in ONE exchange of the context's transport and unpacked (own pieces are copied directly).
namespace {
struct RdRun { int sp, sl, dp, dl, len; };

// runs of global indices [i0, i0 + n) (0-based): source blocks of nbk from process src, aligned copy
// blocks of nbk from process 0, over np processes
std::vector<RdRun> rd_runs(int i0, int n, int nbk, int src, int np) {
  std::vector<RdRun> r;
  int I = i0;
  while (I < i0 + n) {
    const int i = I - i0;
    const int len = std::min({nbk - I % nbk, nbk - i % nbk, i0 + n - I});
    const int bs = I / nbk, bd = i / nbk;
    r.push_back(RdRun{(src + bs) % np, (bs / np) * nbk + I % nbk, bd % np, (bd / np) * nbk + i % nbk, len});
    I += len;
  }
  return r;
}
}  // namespace

int nat_redistribute(dplasma_context_t* ctx, int es, char* src, int slld, int mb, int nb, int rsrc, int csrc, int ia,
                     int ja, int m, int n, char* dst, int dlld, bool to_aligned) {
  NatCtx* c = ctx ? ctx->nat : nullptr;
  if (!c || m <= 0 || n <= 0) return 0;
  const int P = c->P, Q = c->Q, me = c->rank, myrow = c->myrow, mycol = c->mycol;
  const std::vector<RdRun> rr = rd_runs(ia - 1, m, mb, rsrc, P), cr = rd_runs(ja - 1, n, nb, csrc, Q);
  // the orientation of this call: data flows from "from" layout to "to" layout
  auto from_row = [&](const RdRun& x) { return to_aligned ? x.sp : x.dp; };
  auto to_row = [&](const RdRun& x) { return to_aligned ? x.dp : x.sp; };
  auto from_l = [&](const RdRun& x) { return to_aligned ? x.sl : x.dl; };
  auto to_l = [&](const RdRun& x) { return to_aligned ? x.dl : x.sl; };
  char* fbuf = to_aligned ? src : dst;
  char* tbuf = to_aligned ? dst : src;
  const int flld = to_aligned ? slld : dlld, tlld = to_aligned ? dlld : slld;
  // bytes of the message from (fr, fc) to (tr, tc)
  auto msg_elems = [&](int fr, int fc, int tr, int tc) {
    long long rows = 0, cols = 0;
    for (const RdRun& x : rr)
      if (from_row(x) == fr && to_row(x) == tr) rows += x.len;
    for (const RdRun& y : cr)
      if (from_row(y) == fc && to_row(y) == tc) cols += y.len;
    return rows * cols;
  };
  // walk the pieces of one message: f(from_offset, to_offset, len) in elements
  auto walk = [&](int fr, int fc, int tr, int tc, auto&& f) {
    for (const RdRun& y : cr) {
      if (from_row(y) != fc || to_row(y) != tc) continue;
      for (int jj = 0; jj < y.len; ++jj)
        for (const RdRun& x : rr) {
          if (from_row(x) != fr || to_row(x) != tr) continue;
          f((long long)from_l(x) + (long long)(from_l(y) + jj) * flld, (long long)to_l(x) + (long long)(to_l(y) + jj) * tlld,
            x.len);
        }
    }
  };
  std::vector<NatMsg> sends, recvs;
  std::vector<std::vector<char>> hs, hr;
  std::vector<int> speer, rpeer;
  for (int d = 0; d < P * Q; ++d) {
    const int dr = d / Q, dc = d % Q;
    if (d == me) {   // own pieces: direct host copies
      walk(myrow, mycol, myrow, mycol, [&](long long fo, long long to, int len) {
        std::memcpy(tbuf + to * es, fbuf + fo * es, (size_t)len * es);
      });
      continue;
    }
    const long long ns = msg_elems(myrow, mycol, dr, dc), nr = msg_elems(dr, dc, myrow, mycol);
    if (ns > 0) {
      std::vector<char> b((size_t)ns * es);
      size_t p = 0;
      walk(myrow, mycol, dr, dc, [&](long long fo, long long, int len) {
        std::memcpy(b.data() + p, fbuf + fo * es, (size_t)len * es);
        p += (size_t)len * es;
      });
      hs.push_back(std::move(b));
      speer.push_back(d);
    }
    if (nr > 0) {
      hr.emplace_back((size_t)nr * es);
      rpeer.push_back(d);
    }
  }
  std::vector<void*> dbufs;
  auto dev = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
    dbufs.push_back(p);
    return p;
  };
  int rc = 0;
  for (size_t q = 0; q < hs.size() && rc == 0; ++q) {
    void* p = dev(hs[q].size());
    if (!p || hipMemcpy(p, hs[q].data(), hs[q].size(), hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    else sends.push_back(NatMsg{speer[q], p, hs[q].size()});
  }
  for (size_t q = 0; q < hr.size() && rc == 0; ++q) {
    void* p = dev(hr[q].size());
    if (!p) rc = -1;
    else recvs.push_back(NatMsg{rpeer[q], p, hr[q].size()});
  }
  hipStream_t st = c->st[0];
  if (rc == 0 && (!sends.empty() || !recvs.empty())) rc = c->comm->exchange(sends, recvs, st);
  if (rc == 0 && hipStreamSynchronize(st) != hipSuccess) rc = -1;
  for (size_t q = 0; q < hr.size() && rc == 0; ++q) {
    if (hipMemcpy(hr[q].data(), recvs[q].buf, hr[q].size(), hipMemcpyDeviceToHost) != hipSuccess) { rc = -1; break; }
    const int s = rpeer[q];
    size_t p = 0;
    walk(s / Q, s % Q, myrow, mycol, [&](long long, long long to, int len) {
      std::memcpy(tbuf + to * es, hr[q].data() + p, (size_t)len * es);
      p += (size_t)len * es;
    });
  }
  for (void* p : dbufs) (void)hipFree(p);
  return rc;
}

// ------------------------------------------------------------------------------------------------- QR
// Flat-tree Householder QR, Q application and least squares on the grid (reference: src/zgeqrf.jdf,
// zunmqr_LC.jdf and zgels_wrapper.c on a P x Q process grid; the data movement of ScaLAPACK's pdgeqrf:
// a panel factorisation, then the block reflector applied as C -= V T^H (V^H C) with V^H C summed over
// each process column).  Step k:
//   1. the panel (tile column k, rows k..) goes to every rank (owners pack, one exchange) and every rank
//      factors it redundantly with the persistent panel kernel (dpl_qr_panel: deterministic, so R, V and T
//      come out identical everywhere, the distributed LU's scheme) -- T_k is kept on every rank (fullT);
//   2. this rank's tiles of the factored panel go back into A (R above, V below the diagonal: LAPACK's
//      layout, tau_j = T_k(j, j)); T(k, k)'s owner stores the reference-layout IB x IB diagonal blocks;
//   3. this rank's rows of V are packed in local row order (Vloc); W = Vloc^H C_loc over its trailing tiles
//      (one MFMA GEMM), the partial W goes to the process column's other ranks (one exchange) and theirs
//      are added; C_loc -= Vloc (T^H W) (two GEMMs).
// unmqr (left): V_k of tile column k is rebuilt from A by the ranks of that process column and sent
// along the process rows; then step 3 on C's tiles.  gels: geqrf, Q^H B, R X = (Q^H B)(0:N).
namespace {

// a view of the leading r x c part of a distributed matrix (same storage)
std::shared_ptr<NatDesc> dist_view(const NatDesc& D, int r, int c) {
  auto v = std::make_shared<NatDesc>();
  v->ctx = D.ctx;
  v->prec = D.prec, v->es = D.es, v->mb = D.mb, v->nb = D.nb, v->m = r, v->n = c;
  v->mt = (r + D.mb - 1) / D.mb;
  v->nt = (c + D.nb - 1) / D.nb;
  v->P = D.P, v->Q = D.Q, v->myrow = D.myrow, v->mycol = D.mycol;
  auto loc = [](int n, int b, int p, int np) {   // numroc from process 0
    const int nbl = n / b, ext = nbl % np;
    int x = (nbl / np) * b;
    if (p < ext) x += b;
    else if (p == ext) x += n % b;
    return x;
  };
  v->lm = loc(r, D.mb, D.myrow, D.P);
  v->ln = loc(c, D.nb, D.mycol, D.Q);
  v->lld = D.lld;
  v->data = D.data;
  v->owned = false;
  return v;
}

// first local row (tile row) >= k and first local column (tile column) >= j0 of D on this rank
long long first_local_row(const NatDesc& D, int k) {
  for (int m = k; m < D.mt; ++m)
    if (m % D.P == D.myrow) return (long long)(m / D.P) * D.mb;
  return D.lm;
}
long long first_local_col(const NatDesc& D, int j0) {
  for (int n = j0; n < D.nt; ++n)
    if (n % D.Q == D.mycol) return (long long)(n / D.Q) * D.nb;
  return D.ln;
}

struct DistQrWork {
  DevPtr pan, V, ws, Vl, W, W2, Wr, slots;
  int ldv = 0, ldvl = 0, wcols = 0;
};

bool dist_qr_work(NatProgram& P, const NatDesc& A, const NatDesc& C, DistQrWork& w) {
  const int es = A.es, nb = A.nb;
  w.ldv = std::max(16, (A.m + 15) / 16 * 16);
  w.ldvl = std::max(16, (A.lm + 15) / 16 * 16);
  w.wcols = std::max(1, C.ln);
  w.pan = dev_alloc((size_t)w.ldv * nb * es, false);
  w.V = dev_alloc((size_t)w.ldv * nb * es, true);
  w.ws = dev_alloc((size_t)dpl_qr_panel_ws_bytes(A.prec, nb, nb) + 256, true);
  w.Vl = dev_alloc((size_t)w.ldvl * nb * es, true);
  w.W = dev_alloc((size_t)nb * w.wcols * es, true);
  w.W2 = dev_alloc((size_t)nb * w.wcols * es, true);
  w.Wr = dev_alloc((size_t)std::max(1, A.P - 1) * nb * w.wcols * es, true);
  w.slots = dev_alloc((size_t)std::max(1, A.mt) * A.mb * nb * es, false);
  for (const DevPtr& d : {w.pan, w.V, w.ws, w.Vl, w.W, w.W2, w.Wr, w.slots}) {
    if (!d) return false;
    P.keep.push_back(d);
  }
  return true;
}

// step 3: C_loc (tile rows >= k, local columns from lc0) := op(I - V T V^H) C_loc, V = Vloc (ldvl, rows in
// C's local row order starting at lr0); reduction over the process column.  Tasks on stream 1 after prev.
int add_dist_left_apply(NatProgram& P, NatDesc& C, const DistQrWork& w, long long lr0, long long lc0, int kf,
                        const char* Tk, int ldt, bool qt, int prev) {
  NatComm* comm = P.ctx->comm;
  const int prec = C.prec, es = C.es, ldc = C.lld, Pg = C.P, Q = C.Q, me = P.ctx->rank;
  const int rows = (int)(C.lm - lr0), cols = (int)(C.ln - lc0);
  if (cols <= 0 || kf <= 0) return prev;
  const Scalar one(prec, 1.0), zero(prec, 0.0), m_one(prec, -1.0);
  char *c = C.data, *vl = (char*)w.Vl->p, *W = (char*)w.W->p, *W2 = (char*)w.W2->p, *Wr = (char*)w.Wr->p;
  const int ldvl = w.ldvl;
  auto g1 = std::make_shared<Gemm>(), g2 = std::make_shared<Gemm>(), g3 = std::make_shared<Gemm>();
  // one item per local tile column (the engine's 128 x 128 sub-tiles), W column offset = local column
  for (long long j = lc0; j < C.ln; j += C.nb) {
    const int nj = (int)std::min<long long>(C.nb, C.ln - j);
    const long long wo = (j - lc0) * kf;
    if (rows > 0) g1->add(wo, kf, nj, {KPair{0, lr0 + j * ldc, rows, 0}}, 0);
    g2->add(wo, kf, nj, {KPair{0, wo, kf, 0}}, 0);
    if (rows > 0) g3->add(lr0 + j * ldc, rows, nj, {KPair{0, wo, kf, 0}}, 0);
  }
  if ((!g1->empty() && !g1->upload(P)) || !g2->upload(P) || (!g3->empty() && !g3->upload(P))) return -2;
  const size_t wbytes = (size_t)kf * cols * es;
  auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
  int slot = 0;
  for (int r = 0; r < Pg; ++r) {
    const int peer = r * Q + C.mycol;
    if (peer == me) continue;
    sends->push_back(NatMsg{peer, W, wbytes});
    recvs->push_back(NatMsg{peer, Wr + (size_t)slot * wbytes, wbytes});
    ++slot;
  }
  const int nsl = slot;
  std::vector<TileItem> sum_it{TileItem{0, 0, kf, cols, 0, 0}};
  DevPtr d_sum = dev_upload(sum_it);
  if (!d_sum) return -2;
  P.keep.push_back(d_sum);
  return P.task(1, [=](hipStream_t s) {
    int rc = 0;
    if (g1->empty()) rc = hipMemsetAsync(W, 0, wbytes, s) == hipSuccess ? 0 : -1;
    else rc = g1->launch(prec, CONJTRANS, NOTRANS, one, vl, ldvl, c, ldc, zero, W, kf, s);
    if (rc == 0 && nsl) rc = comm->exchange(*sends, *recvs, s);
    for (int q = 0; q < nsl && rc == 0; ++q)   // W += the column's other partials
      rc = dpl_geadd(prec, 0, NOTRANS, 1, d_sum->p, kf, cols, one.ptr(), Wr + (size_t)q * wbytes, kf, one.ptr(), W, kf,
                     0, s);
    if (rc == 0) rc = g2->launch(prec, qt ? CONJTRANS : NOTRANS, NOTRANS, one, Tk, ldt, W, kf, zero, W2, kf, s);
    if (rc == 0 && !g3->empty()) rc = g3->launch(prec, NOTRANS, NOTRANS, m_one, vl, ldvl, W2, kf, one, c, ldc, s);
    return rc;
  }, {prev});
}

}  // namespace

bool nat_dist_geqrf_into(NatProgram& P, NatDesc& A, NatDesc& T) {
  NatCtx* c = P.ctx;
  NatComm* comm = c->comm;
  const int prec = A.prec, mb = A.mb, nb = A.nb, ld = A.lld, es = A.es, me = c->rank;
  const int kt = std::min(A.mt, A.nt);
  DistQrWork w;
  if (!dist_qr_work(P, A, A, w)) return false;
  T.fullT = dev_alloc((size_t)std::max(1, kt) * nb * nb * es, true);
  if (!T.fullT) return false;
  T.fullT_nb = nb;
  T.fullT_kt = kt;
  P.keep.push_back(T.fullT);
  char *a = A.data, *pan = (char*)w.pan->p, *V = (char*)w.V->p, *ws = (char*)w.ws->p, *vl = (char*)w.Vl->p;
  char *tf = (char*)T.fullT->p, *sl = (char*)w.slots->p, *t = T.data;
  int* info = (int*)P.info->p;
  const int ldv = w.ldv, ldvl = w.ldvl, ldT = T.lld, ib = T.mb;
  const size_t st = (size_t)mb * nb;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  int prev = -1;
  for (int k = 0; k < kt; ++k) {
    const int M = A.m - k * mb, kb = A.cols(k), kf = std::min(M, kb);
    // ---- 1. the panel to every rank, packed tile by tile into the contiguous panel (ld ldv)
    auto pk = std::make_shared<MapBatch>(), sc = std::make_shared<MapBatch>(), back = std::make_shared<MapBatch>();
    auto vpk = std::make_shared<MapBatch>();
    auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
    long long vrow = 0;   // Vloc row of the next local tile
    for (int m = k; m < A.mt; ++m) {
      const int src = A.owner(m, k);
      char* slot = sl + (size_t)m * st * es;
      if (src == me) {
        pk->it.push_back(TileItem{A.off(m, k), (long long)m * (long long)st, A.rows(m), kb, 0, 0});
        back->it.push_back(TileItem{(long long)(m - k) * mb, A.off(m, k), A.rows(m), kb, 0, 0});
        for (int r = 0; r < c->world; ++r)
          if (r != me) sends->push_back(NatMsg{r, slot, st * es});
      } else {
        recvs->push_back(NatMsg{src, slot, st * es});
      }
      if (m % A.P == A.myrow) {   // my rows of V, local order
        vpk->it.push_back(TileItem{(long long)(m - k) * mb, vrow, A.rows(m), kf, 0, 0});
        vrow += A.rows(m);
        vpk->mm = std::max(vpk->mm, A.rows(m));
      }
      sc->it.push_back(TileItem{(long long)m * (long long)st, (long long)(m - k) * mb, A.rows(m), kb, 0, 0});
      pk->mm = sc->mm = back->mm = std::max(pk->mm, A.rows(m));
    }
    pk->nn = sc->nn = back->nn = kb;
    vpk->nn = kf;
    if (!pk->upload(P) || !sc->upload(P) || !back->upload(P) || !vpk->upload(P)) return false;
    char* Tk = tf + (size_t)k * nb * nb * es;
    prev = P.task(1, [=](hipStream_t s) {
      int rc = pk->n() ? dpl_geadd(prec, 0, NOTRANS, pk->n(), pk->items(), pk->mm, pk->nn, one.ptr(), a, ld, zero.ptr(),
                                   sl, mb, 1, s) : 0;
      if (rc == 0 && (!sends->empty() || !recvs->empty())) rc = comm->exchange(*sends, *recvs, s);
      if (rc == 0)
        rc = dpl_geadd(prec, 0, NOTRANS, sc->n(), sc->items(), sc->mm, sc->nn, one.ptr(), sl, mb, zero.ptr(), pan, ldv, 1, s);
      // ---- the factorisation, redundantly on every rank
      if (rc == 0) rc = dpl_qr_panel(prec, pan, ldv, 0, 0, M, kb, kf, V, ldv, Tk, nb, ws, info, s);
      // ---- 2. my tiles back; 3. my rows of V
      if (rc == 0 && back->n())
        rc = dpl_geadd(prec, 0, NOTRANS, back->n(), back->items(), back->mm, back->nn, one.ptr(), pan, ldv, zero.ptr(), a, ld,
                       1, s);
      if (rc == 0 && vpk->n())
        rc = dpl_geadd(prec, 0, NOTRANS, vpk->n(), vpk->items(), vpk->mm, vpk->nn, one.ptr(), V, ldv, zero.ptr(), vl, ldvl,
                       1, s);
      return rc;
    }, {prev});
    if (T.local(k, k)) {   // the reference layout: IB x IB diagonal blocks of T_k into tile T(k, k)
      std::vector<TileItem> ti;
      for (int b0 = 0; b0 < kf; b0 += ib) {
        const int bs = std::min(ib, kf - b0);
        ti.push_back(TileItem{(long long)k * nb * nb + b0 + (long long)b0 * nb, T.off(k, k) + (long long)b0 * ldT, bs, bs, 0, 0});
      }
      DevPtr d_ti = dev_upload(ti);
      if (!d_ti) return false;
      P.keep.push_back(d_ti);
      const int nti = (int)ti.size();
      prev = P.task(1, [=](hipStream_t s) {
        return dpl_geadd(prec, 0, NOTRANS, nti, d_ti->p, ib, ib, one.ptr(), tf, nb, zero.ptr(), t, ldT, 1, s);
      }, {prev});
    }
    if (k + 1 >= A.nt) continue;
    prev = add_dist_left_apply(P, A, w, first_local_row(A, k), first_local_col(A, k + 1), kf, Tk, nb, true, prev);
    if (prev < -1) return false;
  }
  return true;
}

// C := op(Q) C with Q from nat_dist_geqrf_into (left side; C distributed like A's rows)
bool nat_dist_unmqr_into(NatProgram& P, int trans, NatDesc& A, NatDesc& T, NatDesc& C) {
  NatCtx* c = P.ctx;
  NatComm* comm = c->comm;
  const int prec = A.prec, mb = A.mb, nb = A.nb, ld = A.lld, es = A.es, me = c->rank, Q = A.Q;
  const int kt = std::min(A.mt, A.nt);
  DistQrWork w;
  if (!dist_qr_work(P, A, C, w)) return false;
  const bool qt = trans != NOTRANS;
  char *a = A.data, *vl = (char*)w.Vl->p, *raw = (char*)w.pan->p, *tf = (char*)T.fullT->p;
  const int ldvl = w.ldvl;
  const Scalar one(prec, 1.0), zero(prec, 0.0);
  int prev = last_task_on(P, 1);
  for (int s = 0; s < kt; ++s) {
    const int k = qt ? s : kt - 1 - s;   // Q^H C: panel 0 first; Q C: the last first
    const int M = A.m - k * mb, kb = A.cols(k), kf = std::min(M, kb), pc = k % Q;
    const long long lr0 = first_local_row(A, k), rows = A.lm - lr0;
    // V_k rows of this process row: the column-k owner in my process row packs them (raw, ld ldvl) and
    // sends them along the row; every rank builds Vloc (unit diagonal, zeros above it) from raw
    auto sends = std::make_shared<std::vector<NatMsg>>(), recvs = std::make_shared<std::vector<NatMsg>>();
    const size_t rbytes = (size_t)ldvl * kb * es;
    if (rows > 0) {
      if (A.mycol == pc) {
        for (int q = 0; q < Q; ++q)
          if (q != A.mycol) sends->push_back(NatMsg{A.myrow * Q + q, raw, rbytes});
      } else {
        recvs->push_back(NatMsg{A.myrow * Q + pc, raw, rbytes});
      }
    }
    auto lt = std::make_shared<MapBatch>(), cp = std::make_shared<MapBatch>();
    long long vrow = 0;
    for (int m = k; m < A.mt; ++m) {
      if (m % A.P != A.myrow) continue;
      lt->it.push_back(TileItem{vrow, vrow, A.rows(m), kf, (m - k) * mb, 0});
      cp->it.push_back(TileItem{vrow, vrow, A.rows(m), kf, (m - k) * mb, 0});
      vrow += A.rows(m);
      lt->mm = cp->mm = std::max(lt->mm, A.rows(m));
    }
    lt->nn = cp->nn = kf;
    if (!lt->upload(P) || !cp->upload(P)) return false;
    const bool mine = A.mycol == pc && rows > 0;
    const long long coff = lr0 + (long long)(k / Q) * nb * ld;   // my column-k rows in A (when mine)
    prev = P.task(1, [=](hipStream_t st) {
      int rc = 0;
      if (mine && hipMemcpy2DAsync(raw, (size_t)ldvl * es, a + coff * es, (size_t)ld * es, (size_t)rows * es, kb,
                                   hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = -1;
      if (rc == 0 && (!sends->empty() || !recvs->empty())) rc = comm->exchange(*sends, *recvs, st);
      if (rc == 0 && lt->n()) rc = dpl_laset(prec, 0, lt->n(), lt->items(), lt->mm, lt->nn, zero.ptr(), one.ptr(), vl, ldvl, st);
      if (rc == 0 && cp->n())   // part 3: strictly below the panel's diagonal
        rc = dpl_geadd(prec, 3, NOTRANS, cp->n(), cp->items(), cp->mm, cp->nn, one.ptr(), raw, ldvl, zero.ptr(), vl, ldvl, 1, st);
      return rc;
    }, {prev});
    prev = add_dist_left_apply(P, C, w, first_local_row(C, k), 0, kf, tf + (size_t)k * nb * nb * es, nb, qt, prev);
    if (prev < -1) return false;
  }
  return true;
}

NatProgram* nat_dist_geqrf(NatCtx* c, NatDesc& A, NatDesc& T) {
  NatProgram* P = new_program(c, "geqrf", true);
  if (!P->info || !nat_dist_geqrf_into(*P, A, T)) return fail(P, "geqrf: device allocation failed");
  return P;
}

NatProgram* nat_dist_unmqr(NatCtx* c, int trans, NatDesc& A, NatDesc& T, NatDesc& C) {
  NatProgram* P = new_program(c, "unmqr", false);
  if (!nat_dist_unmqr_into(*P, trans, A, T, C)) return fail(P, "unmqr: device allocation failed");
  return P;
}

NatProgram* nat_dist_gels(NatCtx* c, NatDesc& A, NatDesc& T, NatDesc& B) {
  NatProgram* P = new_program(c, "gels", true);
  if (!P->info || !nat_dist_geqrf_into(*P, A, T) || !nat_dist_unmqr_into(*P, CONJTRANS, A, T, B))
    return fail(P, "gels: device allocation failed");
  auto R = dist_view(A, A.n, A.n), X = dist_view(B, A.n, B.n);
  P->wdesc.push_back(R);
  P->wdesc.push_back(X);
  if (!nat_dist_trsm_into(*P, LEFT, UPPER, NOTRANS, NONUNIT, Scalar(A.prec, 1.0), *R, *X))
    return fail(P, "gels: device allocation failed");
  return P;
}
