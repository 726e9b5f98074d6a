// Internal types of the interpreter-free engine (native.cpp, native_dist.cpp): kernel entry points,
// batch records, device buffers, contexts, descriptors and stream programs.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "capi_bridge.h"

extern "C" {  // csrc/kernels (libdplasma_kernels.so)
int dpl_gemm_batched(int prec, int transA, int transB, int nitems, const void* items, const void* kpairs, int max_m,
                     int max_n, const void* alpha, const void* A, int lda, const void* B, int ldb, const void* beta,
                     void* C, int ldc, int vec_ok, int force_generic, hipStream_t st);
int dpl_potrf_tile(int prec, int uplo, int n, void* A, long long a_off, int lda, int* info, int info_base,
                   hipStream_t st);
int dpl_potrf_tile_rbz(int uplo, int n, double* A, int lda, int* info, int info_base, double* zbuf, hipStream_t st);
int dpl_potrf_zbuf_size();
int dpl_trsm_rb_prep(int uplo, int n, const double* L, int ldl, double* zbuf, hipStream_t st);
int dpl_trsm_rb(int uplo, int n, const double* L, int ldl, const double* zbuf, int nrb, const void* items, double* B,
                int ldb, hipStream_t st);
int dpl_trsm_batched(int prec, int side, int uplo, int trans, int diag, int nitems, const void* items, int max_m,
                     int max_n, const void* alpha, const void* A, int lda, void* B, int ldb, int ntri,
                     const void* tri_off, void* work, hipStream_t st);
int dpl_generate(int prec, int kind, int nitems, const void* items, int mmax, int nmax, void* A, int lda,
                 long long gM, unsigned long long seed, const void* bump, hipStream_t st);
int dpl_laset(int prec, int part, int nitems, const void* items, int mmax, int nmax, const void* alpha,
              const void* beta, void* A, int lda, hipStream_t st);
int dpl_geadd(int prec, int part, int trans, int nitems, const void* items, int mmax, int nmax, const void* alpha,
              const void* A, int lda, const void* beta, void* B, int ldb, int copy, hipStream_t st);
int dpl_lascal(int prec, int part, int nitems, const void* items, int mmax, int nmax, const void* alpha, void* A,
               int lda, hipStream_t st);
int dpl_diag_scale(int prec, int part, int cols, int nitems, const void* items, int mmax, int nmax,
                   const void* D, int ldd, void* B, int ldb, hipStream_t st);
int dpl_tile_norm(int prec, int kind, int part, int unit, int nitems, const void* items, const void* A, int lda,
                  double* out, int ostride, hipStream_t st);
long long dpl_lu_block_ws_bytes(int m);
int dpl_getrf_tile(int prec, int nitems, const void* items, int* info, hipStream_t st);
int dpl_gessm(int prec, int nitems, const void* items, int max_n, hipStream_t st);
int dpl_ssssm(int prec, int nitems, const void* items, int max_n, int ib, int NB, hipStream_t st);
int dpl_tstrf(int prec, int nitems, const void* items, int ib, int NB, int max_m, int* info, hipStream_t st);
int dpl_lu_block(int prec, void* A, int ld, int m, int c0, int cend, int* ipiv, void* ws, int* cnt, int* info,
                 int info_base, int pivot, hipStream_t st);
int dpl_butterfly(int prec, int side, int trans, int m, int n, int size, const double* r, void* A, long long si,
                  long long sj, int mb, int nb, int ld, hipStream_t st);
int dpl_laswp_panel(int prec, void* A, int ld, int m, int ca, int cb, const int* ipiv, int i0, int i1, int* info,
                    hipStream_t st);
int dpl_piv_moves(const int* ipiv, int kb, int mrel, int* dst, int* src, int* cnt, int* info, hipStream_t st);
int dpl_rows_permute(int prec, void* A, int ld, int mb, int r0, const long long* rowoff, int nrt,
                     const long long* coloff, const int* ncols, int nct, int nb, const int* dst, const int* src,
                     const int* cnt, int maxcnt, int* info, hipStream_t st);
int dpl_ipiv_shift(const int* in, int* out, int n, int delta, hipStream_t st);
long long dpl_qr_panel_ws_bytes(int prec, int nc, int kf);
int dpl_qr_panel(int prec, void* P, int ldp, int rbl, long long rstride, int M, int nc, int kf, void* V, int ldv,
                 void* Tm, int ldt, void* ws, int* info, hipStream_t st);
}

namespace natk {

enum { NOTRANS = 111, TRANS = 112, CONJTRANS = 113, UPPER = 121, LOWER = 122, UPPERLOWER = 123, NONUNIT = 131,
       LEFT = 141, RIGHT = 142 };
enum { P_I = 1, P_S = 2, P_D = 3, P_C = 4, P_Z = 5 };   // P_I: int32 (pivot descriptors)

// kernel records (csrc/kernels/common.h, gemm.hip, potrf_rb.hip)
struct GemmItemK { long long c_off; int kt_beg, kt_cnt, m, n, flags, pad; };
struct KPair { long long a_off, b_off; int k, pad; };
struct TileItem { long long a_off, b_off; int m, n, gi, gj; };
struct RbItem { long long b_off; int rows, pad; };
static_assert(sizeof(GemmItemK) == 32 && sizeof(KPair) == 24 && sizeof(TileItem) == 32 && sizeof(RbItem) == 16,
              "kernel record layouts");

inline int esize(int prec) { return prec == P_S || prec == P_I ? 4 : prec == P_Z ? 16 : 8; }
inline bool prec_ok(int prec) { return prec >= P_S && prec <= P_Z; }

// one scalar of a precision (complex = two reals), as the kernels' host API takes it
struct Scalar {
  alignas(16) unsigned char b[16] = {};   // read as hipDoubleComplex (16-byte aligned loads)
  Scalar(int prec, double re, double im = 0.0) {
    if (prec == P_S || prec == P_C) {
      float v[2] = {(float)re, (float)im};
      std::memcpy(b, v, prec == P_S ? 4 : 8);
    } else {
      double v[2] = {re, im};
      std::memcpy(b, v, prec == P_D ? 8 : 16);
    }
  }
  Scalar(int prec, const void* p) { std::memcpy(b, p, esize(prec)); }
  const void* ptr() const { return b; }
};

struct DevMem {
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};
using DevPtr = std::shared_ptr<DevMem>;

// Zero device memory and return once the zeros have landed: a private non-blocking stream and
// hipStreamSynchronize, never the null stream (a rocprofv3 trace showed null-stream fills completing
// after a later kernel of a non-blocking stream had started, profiles/r4_potrf_rb_race.txt)
inline hipError_t nat_zero_sync(void* p, size_t bytes) {
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(p, 0, bytes, s);
  const hipError_t e2 = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  return e != hipSuccess ? e : e2;
}

inline DevPtr dev_alloc(size_t bytes, bool zero) {
  auto d = std::make_shared<DevMem>();
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&d->p, bytes) != hipSuccess) return nullptr;
  if (zero && nat_zero_sync(d->p, bytes) != hipSuccess) return nullptr;
  return d;
}

template <typename R>
DevPtr dev_upload(const std::vector<R>& v) {
  auto d = dev_alloc(v.size() * sizeof(R), false);
  if (d && !v.empty() && hipMemcpy(d->p, v.data(), v.size() * sizeof(R), hipMemcpyHostToDevice) != hipSuccess)
    return nullptr;
  return d;
}

}  // namespace natk
using namespace natk;

// ----------------------------------------------------------------------------- handles
class NatComm;                     // native_comm.h: tile transport of a multi-process context
// the smallest positive info of any rank (a failing column), or -1 if any rank failed (native_comm.cpp)
int nat_comm_reduce_info(NatComm* c, int& info);

NatComm* nat_comm_create(int rank, int world, int device, const char* rdv_dir, std::string& err);
void nat_comm_destroy(NatComm* c);
void nat_ctx_destroy(NatCtx* c);

// ScaLAPACK numroc: rows / columns of an n-long dimension (blocks of nb) kept by process iproc of np
inline int nat_numroc(int n, int nb, int iproc, int np) {
  const int nblocks = n / nb;
  int num = (nblocks / np) * nb;
  const int extra = nblocks % np;
  if (iproc < extra) num += nb;
  else if (iproc == extra) num += n % nb;
  return num;
}

constexpr int NAT_NSTREAM = 3;   // 0: panel (high priority), 1: update, 2: communication

struct NatCtx {
  int device = 0;
  hipStream_t st[NAT_NSTREAM] = {};
  hipEvent_t join[NAT_NSTREAM] = {};
  std::vector<NatProgram*> queue;
  // multi-process context (dplasma_init_native_dist): rank = myrow * Q + mycol on a P x Q grid
  int rank = 0, world = 1, P = 1, Q = 1, myrow = 0, mycol = 0;
  NatComm* comm = nullptr;
  // loopback rehearsal (DPLASMA_LOOPBACK=1 on a world-1 dist context): the grid builders run with the
  // rank as the peer of its own tile edges, so the transport (RCCL self send / receive) really executes
  bool loop = false;
  bool dist() const { return world > 1 || loop; }
};

struct NatDesc {
  NatCtx* ctx = nullptr;
  int prec = P_D, es = 8, mb = 0, nb = 0, m = 0, n = 0, mt = 0, nt = 0, lld = 0;
  // 2-D block-cyclic over the context's P x Q grid: this rank keeps the tiles (i, j) with i % P == myrow
  // and j % Q == mycol, in ScaLAPACK local layout (column-major, lld >= local rows)
  int P = 1, Q = 1, myrow = 0, mycol = 0, lm = 0, ln = 0;
  char* data = nullptr;
  bool owned = false;
  // a T descriptor written by the native geqrf: every panel's full nb x nb compact-WY T (ld nb), the
  // reference-layout IB x IB diagonal blocks being in the tiles themselves (unmqr / ungqr / gels read it)
  DevPtr fullT;
  int fullT_nb = 0, fullT_kt = 0;
  // written by the native tree-driven geqrf_param (TS: one slot per TS domain head, TT: one per TT-killed
  // row): slot of (row, k) at tidx[k * tidx_mt + row] (-1: none), each an nb x nb T in fullT
  std::vector<long long> tidx;
  int tidx_mt = 0;
  NatDesc() = default;
  NatDesc(const NatDesc&) = delete;             // owns its buffer: never copied (nor captured by value)
  NatDesc& operator=(const NatDesc&) = delete;
  // offset of tile (i, j) in the local storage (a tile of this rank: local(i, j))
  long long off(int i, int j) const { return (long long)(i / P) * mb + (long long)(j / Q) * nb * lld; }
  bool local(int i, int j) const { return i % P == myrow && j % Q == mycol; }
  int owner(int i, int j) const { return (i % P) * Q + j % Q; }
  bool dist() const { return P * Q > 1; }
  int rows(int i) const { return std::min(mb, m - i * mb); }
  int cols(int j) const { return std::min(nb, n - j * nb); }
  ~NatDesc() {
    if (owned && data) (void)hipFree(data);
  }
};

struct NatTask {
  int stream;
  std::vector<int> deps;
  std::function<int(hipStream_t)> fn;
  bool event = false;
  // predicated task (a data-dependent branch decided by an earlier task at enqueue time): fn runs only if
  // *guard == want; otherwise the task launches nothing (its event, if any, is still recorded)
  std::shared_ptr<int> guard;
  int want = 1;
};

struct NatProgram {
  NatCtx* ctx = nullptr;
  std::string name;
  std::vector<NatTask> tasks;
  std::vector<hipEvent_t> ev;
  std::vector<DevPtr> keep;      // batch records and scratch referenced by the tasks
  std::vector<std::shared_ptr<NatDesc>> wdesc;   // workspace matrices (trmm / symm / getrf panels)
  DevPtr info;                   // device int: first failing column (LAPACK info), 0 if none
  int result = 0;
  bool enqueued = false;
  // gate >= 0: tasks from index gate on are enqueued only if the factorisation before them left info == 0
  // (blocking posv: the reference's zposv_wrapper runs potrs only then); run() synchronises at the gate
  int gate = -1;

  // tasks added while cur_guard is set are predicated on *cur_guard == cur_want
  std::shared_ptr<int> cur_guard;
  int cur_want = 1;

  int task(int stream, std::function<int(hipStream_t)> fn, std::initializer_list<int> deps) {
    NatTask t;
    t.stream = stream;
    t.fn = std::move(fn);
    t.guard = cur_guard;
    t.want = cur_want;
    const int id = (int)tasks.size();
    for (int d : deps) {
      if (d < 0 || d >= id) continue;
      t.deps.push_back(d);
      if (tasks[d].stream != stream) tasks[d].event = true;
    }
    tasks.push_back(std::move(t));
    return id;
  }

  // enqueue every task (stream order + events for cross-stream edges); the program starts after
  // everything already queued on the context's streams (join events) -- programs compose in call order
  int run() {
    if (ev.empty()) {
      ev.assign(tasks.size(), nullptr);
      for (size_t i = 0; i < tasks.size(); ++i)
        if (tasks[i].event && hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return -1;
    }
    // info is cleared before the join, so a task on any stream that writes it (tile factorisations, row
    // moves reporting an out-of-range pivot) is ordered after the clear
    if (info && hipMemsetAsync(info->p, 0, sizeof(int), ctx->st[0]) != hipSuccess) return -1;
    for (int s = 0; s < NAT_NSTREAM; ++s)
      if (hipEventRecord(ctx->join[s], ctx->st[s]) != hipSuccess) return -1;
    for (int s = 0; s < NAT_NSTREAM; ++s)
      for (int o = 0; o < NAT_NSTREAM; ++o)
        if (o != s && hipStreamWaitEvent(ctx->st[s], ctx->join[o], 0) != hipSuccess) return -1;
    for (size_t i = 0; i < tasks.size(); ++i) {
      if (info && (int)i == gate) {
        int v = 0;
        for (int q = 0; q < NAT_NSTREAM; ++q)
          if (hipStreamSynchronize(ctx->st[q]) != hipSuccess) return -1;
        if (hipMemcpy(&v, info->p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        if (ctx->comm && nat_comm_reduce_info(ctx->comm, v) != 0) return -1;   // every rank takes the same branch
        if (v != 0) break;
      }
      NatTask& t = tasks[i];
      hipStream_t s = ctx->st[t.stream];
      for (int d : t.deps)
        if (tasks[d].stream != t.stream && hipStreamWaitEvent(s, ev[d], 0) != hipSuccess) return -1;
      const int rc = (t.guard && *t.guard != t.want) ? 0 : t.fn(s);
      if (rc != 0) {
        if (const char* e = std::getenv("DPLASMA_NATIVE_DEBUG"); e && *e == '1')
          std::fprintf(stderr, "[native] %s: task %zu of %zu (stream %d) failed: %d\n", name.c_str(), i, tasks.size(),
                       t.stream, rc);
        return rc;
      }
      if (t.event && hipEventRecord(ev[i], s) != hipSuccess) return -1;
    }
    enqueued = true;
    return 0;
  }

  int wait() {
    for (int s = 0; s < NAT_NSTREAM; ++s)
      if (hipStreamSynchronize(ctx->st[s]) != hipSuccess) return -1;
    result = 0;
    if (info && hipMemcpy(&result, info->p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    // a distributed factorisation's info is the same on every rank (the reference all-reduces it)
    if (info && ctx->comm && nat_comm_reduce_info(ctx->comm, result) != 0) return -1;
    enqueued = false;
    return 0;
  }

  ~NatProgram() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

namespace natk {

// tile-wise maps / copies: one item per tile of B (paired with op(A)'s source tile), one dpl_geadd / dpl_laset launch
struct MapBatch {
  std::vector<TileItem> it;
  int mm = 0, nn = 0;
  DevPtr d;
  // the tiles of B (optionally paired with op(A)'s source tile) touching the uplo part
  void build(const NatDesc& B, int uplo, const NatDesc* A, int trans) {
    for (int n = 0; n < B.nt; ++n)
      for (int m = 0; m < B.mt; ++m) {
        if ((uplo == LOWER && m < n) || (uplo == UPPER && m > n)) continue;
        if (!B.local(m, n)) continue;   // (a multi-process context: this rank's tiles)
        const long long ao = A ? (trans == NOTRANS ? A->off(m, n) : A->off(n, m)) : B.off(m, n);
        it.push_back(TileItem{A ? ao : B.off(m, n), B.off(m, n), B.rows(m), B.cols(n), m * B.mb, n * B.nb});
        mm = std::max(mm, B.rows(m));
        nn = std::max(nn, B.cols(n));
      }
  }
  bool upload(NatProgram& P) {
    if (it.empty()) return true;
    d = dev_upload(it);
    if (!d) return false;
    P.keep.push_back(d);
    return true;
  }
  int n() const { return (int)it.size(); }
  const void* items() const { return d ? d->p : nullptr; }
};

struct Gemm {
  std::vector<GemmItemK> it;
  std::vector<KPair> kp;
  int max_m = 0, max_n = 0;
  bool full = true;
  long long align = 0;
  DevPtr d_it, d_kp;

  void add(long long c, int m, int n, const std::vector<KPair>& pairs, int mask) {
    GemmItemK g{c, (int)kp.size(), (int)pairs.size(), m, n, mask, 0};
    for (const KPair& p : pairs) {
      kp.push_back(p);
      align |= p.a_off | p.b_off;
      if (p.k % 16) full = false;
    }
    if (m % 128 || n % 128) full = false;
    align |= c;
    it.push_back(g);
    max_m = std::max(max_m, m);
    max_n = std::max(max_n, n);
  }
  bool empty() const { return it.empty(); }
  bool upload(NatProgram& P) {
    if (kp.empty()) kp.push_back(KPair{0, 0, 0, 0});
    d_it = dev_upload(it);
    d_kp = dev_upload(kp);
    if (!d_it || !d_kp) return false;
    P.keep.push_back(d_it);
    P.keep.push_back(d_kp);
    return true;
  }
  int launch(int prec, int ta, int tb, const Scalar& alpha, const void* A, int lda, const void* B, int ldb,
             const Scalar& beta, void* C, int ldc, hipStream_t st) const {
    if (it.empty()) return 0;
    const int ve = std::max(1, 16 / esize(prec));
    int vec = (align % ve == 0 && lda % ve == 0 && ldb % ve == 0 && (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0)
                  ? 1 : 0;
    if (vec && full) vec |= 2;
    return dpl_gemm_batched(prec, ta, tb, (int)it.size(), d_it->p, d_kp->p, max_m, max_n, alpha.ptr(), A, lda, B,
                            ldb, beta.ptr(), C, ldc, vec, 0, st);
  }
};

// items sharing ONE triangular tile (dpl_trsm_batched with ntri = 1)
struct Trsm1 {
  std::vector<TileItem> it;
  int max_m = 0, max_n = 0, npos = 0;
  DevPtr d_it, d_tri, d_work;
  long long tri = 0;
  void add(long long b_off, int m, int n) {
    it.push_back(TileItem{tri, b_off, m, n, 0, 0});
    max_m = std::max(max_m, m);
    max_n = std::max(max_n, n);
  }
  bool upload(NatProgram& P, int prec, int side) {
    npos = side == LEFT ? max_m : max_n;
    d_it = dev_upload(it);
    d_tri = dev_upload(std::vector<long long>{tri});
    d_work = dev_alloc((size_t)((npos + 15) / 16) * 256 * esize(prec), false);
    if (!d_it || !d_tri || !d_work) return false;
    P.keep.push_back(d_it);
    P.keep.push_back(d_tri);
    P.keep.push_back(d_work);
    return true;
  }
  int launch(int prec, int side, int uplo, int trans, int diag, const Scalar& alpha, const void* A, int lda, void* B,
             int ldb, hipStream_t st) const {
    if (it.empty()) return 0;
    return dpl_trsm_batched(prec, side, uplo, trans, diag, (int)it.size(), d_it->p, max_m, max_n, alpha.ptr(), A, lda,
                            B, ldb, 1, d_tri->p, d_work->p, st);
  }
};

// set by same_ctx when it refuses a multi-process context: fail() then names that as the reason
inline thread_local bool nat_dist_refused = false;

inline NatProgram* fail(NatProgram* P, const std::string& msg) {
  delete P;
  if (nat_dist_refused) {
    nat_dist_refused = false;
    const std::string op = msg.substr(0, msg.find(':'));
    dpl_set_error((op + ": not available on a multi-process native context (potrf, potrs, posv, the level-3 BLAS, "
                        "the generators, the element-wise maps and the norms are)").c_str());
    return nullptr;
  }
  dpl_set_error(msg.c_str());
  return nullptr;
}

inline NatProgram* new_program(NatCtx* c, const char* name, bool with_info) {
  NatProgram* P = new NatProgram;
  P->ctx = c;
  P->name = name;
  if (with_info) P->info = dev_alloc(sizeof(int), true);
  return P;
}

inline int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

}  // namespace natk
using namespace natk;

// multi-process builders (native_dist.cpp)
NatProgram* nat_dist_potrf(NatCtx* c, int uplo, NatDesc& A);
NatProgram* nat_dist_gemm(NatCtx* c, int prec, int tA, int tB, const Scalar& alpha, NatDesc& A, NatDesc& B,
                          const Scalar& beta, NatDesc& C);
bool nat_dist_gemm_into(NatProgram& Pr, int prec, int tA, int tB, const Scalar& alpha, NatDesc& A, NatDesc& B,
                        const Scalar& beta, NatDesc& C, int tri = UPPERLOWER);
bool nat_dist_mirror_into(NatProgram& Pr, const NatDesc& A, int uplo, int mtrans, NatDesc& W);
bool nat_dist_trsm_into(NatProgram& Pr, int side, int uplo, int trans, int diag, const Scalar& alpha, NatDesc& A,
                        NatDesc& B);
bool nat_dist_geqrf_into(NatProgram& P, NatDesc& A, NatDesc& T);
bool nat_dist_unmqr_into(NatProgram& P, int trans, NatDesc& A, NatDesc& T, NatDesc& C);
NatProgram* nat_dist_geqrf(NatCtx* c, NatDesc& A, NatDesc& T);
NatProgram* nat_dist_unmqr(NatCtx* c, int trans, NatDesc& A, NatDesc& T, NatDesc& C);
NatProgram* nat_dist_gels(NatCtx* c, NatDesc& A, NatDesc& T, NatDesc& B);

// A := al A on this rank's tiles of the uplo part, appended after everything already in P (native.cpp)
bool nat_add_lascal(NatProgram& P, int uplo, const Scalar& al, NatDesc& A);
