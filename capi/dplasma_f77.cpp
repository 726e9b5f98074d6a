// ScaLAPACK-compatible Fortran-77 entry points of libdplasma.so.
//
// Reference: src/scalapack_wrappers/ (dplasma_wrapper_pd{gemm,potrf,getrf_1d,trsm,trmm,latsqr}.c,
// GENERATE_F77_BINDINGS in common.h:66-82, parsec_init_wrapper_ / parsec_fini_wrapper_ in
// dplasma_wrapper_parsec_init.c): a ScaLAPACK program links libdplasma instead of ScaLAPACK for
// these routines and keeps its own block-cyclic local arrays and 9-integer descriptors.
//
// Every argument arrives by reference (Fortran).  Local arrays may be host memory (copied to the
// GPU for the call and back) or device memory of the context's GPU (used in place); the Python
// side (dplasma_amd.capi.f77) tells them apart with hipPointerGetAttributes.  The BLACS context
// in DESC(2) is a handle made by blacs_gridinit_ below (or dplasma_blacs_gridinit from C) -- the
// weak BLACS / TOOLS symbols here let a standalone program run without a BLACS library, and yield
// to a real one when it is linked.
#include "capi_bridge.h"
#include "include/dplasma.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

PyObject* desc_list(const int* d) {
  PyObject* l = PyList_New(9);
  for (int i = 0; i < 9; ++i) PyList_SET_ITEM(l, i, PyLong_FromLong(d ? d[i] : 0));
  return l;
}
PyObject* chr(const char* c) { return dpl_arg_str(c, 1); }
PyObject* iv(const int* p) { return PyLong_FromLong(p ? *p : 0); }
PyObject* sc(const float* p) { return PyFloat_FromDouble(p ? *p : 0.0); }
PyObject* sc(const double* p) { return PyFloat_FromDouble(p ? *p : 0.0); }
PyObject* sc(const dplasma_complex32_t* p) { return p ? PyComplex_FromDoubles(__real__ *p, __imag__ *p) : PyComplex_FromDoubles(0, 0); }
PyObject* sc(const dplasma_complex64_t* p) { return p ? PyComplex_FromDoubles(__real__ *p, __imag__ *p) : PyComplex_FromDoubles(0, 0); }

// dplasma_amd.capi.f77(name, *args) -> int (info); -1 and the message kept on a Python error
int f77(const char* name, std::initializer_list<PyObject*> args) {
  DplGil g;
  PyObject* n = PyUnicode_FromString(name);
  PyObject* tup = PyTuple_New((Py_ssize_t)args.size() + 1);
  PyTuple_SET_ITEM(tup, 0, n);
  Py_ssize_t i = 1;
  for (PyObject* a : args) {
    if (!a) { a = Py_None; Py_INCREF(a); }
    PyTuple_SET_ITEM(tup, i++, a);
  }
  PyObject* r = dpl_call_fn("f77_tuple", {tup});
  int v = -1;
  if (r) v = (int)PyLong_AsLong(r);
  Py_XDECREF(r);
  return v;
}

// ---- interpreter-free path: a single-process run whose BLACS grid is 1 x 1 runs the ScaLAPACK calls on
// the native engine (capi/native.cpp), and so does a multi-process run (RANK / WORLD_SIZE, one process per
// GPU) given a rendezvous directory in DPLASMA_NATIVE_RDV: its nprow x npcol BLACS grid becomes a
// multi-process native context (capi/native_dist.cpp) and p?potrf_ / p?gemm_ run on the ranks' local
// arrays -- the reference wrappers' flow (dplasma_wrapper_pdpotrf.c:133-291: wrap the local array, run,
// hand it back) without Python.  DPLASMA_F77_PYTHON=1 forces the Python layer.
constexpr int NATIVE_CTXT = 1 << 20;    // BLACS handles of the native registry (Python's are small ints)

int env_i(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
int job_world() { return std::max(1, env_i("WORLD_SIZE", 1)); }
int job_rank() { return env_i("RANK", 0); }

// decided once, at the first F77 call: a GPU, no Python-backed dplasma context already created by the
// program (dplasma_init) -- a program that mixes the C API's Python contexts with the F77 layer keeps
// the Python layer -- and, for more than one process, a rendezvous directory
bool f77_native() {
  static int v = -1;
  if (v < 0) {
    const char* f = std::getenv("DPLASMA_F77_PYTHON");
    const char* rdv = std::getenv("DPLASMA_NATIVE_RDV");
    int nd = 0;
    const bool gpu = hipGetDeviceCount(&nd) == hipSuccess && nd > 0;
    if (!gpu) (void)hipGetLastError();
    v = (job_world() <= 1 || (rdv && *rdv)) && !(f && std::atoi(f) == 1) && gpu && !dplasma_python_active() ? 1 : 0;
  }
  return v == 1;
}

dplasma_context_t* g_nctx = nullptr;
int g_nprow = 1, g_npcol = 1;   // the native BLACS grid

dplasma_context_t* native_ctx() {
  if (!g_nctx && job_world() <= 1) g_nctx = dplasma_init_native(env_i("LOCAL_RANK", 0));
  return g_nctx;
}

dplasma_context_t* native_ctx_any() { return g_nctx; }

bool native_grid(const int* desc) { return f77_native() && desc && desc[1] == NATIVE_CTXT; }

bool on_device(const void* p) {
  hipPointerAttribute_t at;
  if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice;
}

// a native descriptor over the m x n submatrix at (ia, ja) (1-based) of a local array with leading
// dimension lld: zero copy for device memory, a device copy (written back by unwrap) for host memory
struct Wrapped {
  dplasma_desc_t* d = nullptr;
  char* host = nullptr;
  int lld = 0;
  bool copy = false;
  void* dev = nullptr;          // multi-process grids: device copy of a host local array (lm x ln, lld)
  int lm = 0, ln = 0, es = 0;
  // multi-process grids, an operand off (1, 1) or distributed from another process than (0, 0): the
  // aligned copy (host image + device matrix) and the source array's host image
  bool redist = false, src_dev = false;
  void* src = nullptr;
  std::vector<char> hsrc, hw;
  int slld = 0, mb = 0, nb = 0, rsrc = 0, csrc = 0, ia = 1, ja = 1, m = 0, n = 0, wlld = 0;
  size_t sbytes = 0;
};
constexpr int NAT_TILE = 256;

Wrapped wrap(int prec, int es, void* a, int ia, int ja, const int* desc, int m, int n) {
  Wrapped w;
  w.lld = desc[8];
  dplasma_context_t* c = native_ctx();
  if (!c || m <= 0 || n <= 0) return w;
  if (dplasma_context_world(c) > 1) {
    // P x Q grid: the local array IS this rank's tiles in ScaLAPACK local layout when the operand starts
    // at (1, 1) of a matrix distributed from process (0, 0) with mb x nb blocks (the tiles)
    const int mb = desc[4], nb = desc[5], me = dplasma_context_rank(c);
    const int myrow = me / g_npcol, mycol = me % g_npcol;
    int zero = 0;
    int mm = m, nn = n, mbv = mb, nbv = nb, pr = g_nprow, pc = g_npcol, r = myrow, q = mycol;
    const int lm = numroc_(&mm, &mbv, &r, &zero, &pr), ln = numroc_(&nn, &nbv, &q, &zero, &pc);
    if (ia != 1 || ja != 1 || desc[6] != 0 || desc[7] != 0) {
      // not tile aligned: redistribute into an aligned copy (reference scalapack_wrappers/common.c:27-128)
      w.redist = true;
      w.es = es;
      w.src = a;
      w.slld = w.lld, w.mb = mb, w.nb = nb, w.rsrc = desc[6], w.csrc = desc[7], w.ia = ia, w.ja = ja, w.m = m, w.n = n;
      int gm = desc[2], gn = desc[3], rs = desc[6], cs = desc[7];
      const int slm = numroc_(&gm, &mbv, &r, &rs, &pr), sln = numroc_(&gn, &nbv, &q, &cs, &pc);
      (void)slm;
      w.sbytes = (size_t)w.slld * std::max(0, sln) * es;
      w.src_dev = on_device(a);
      char* hs = (char*)a;
      if (w.src_dev) {
        w.hsrc.resize(std::max<size_t>(w.sbytes, 1));
        if (w.sbytes && hipMemcpy(w.hsrc.data(), a, w.sbytes, hipMemcpyDeviceToHost) != hipSuccess) return w;
        hs = w.hsrc.data();
      }
      w.wlld = std::max(1, lm);
      w.hw.assign((size_t)w.wlld * std::max(1, ln) * es, 0);
      if (nat_redistribute(c, es, hs, w.slld, mb, nb, desc[6], desc[7], ia, ja, m, n, w.hw.data(), w.wlld, true) != 0) {
        dpl_set_error("native multi-process F77: redistribution of an unaligned operand failed");
        return w;
      }
      void* d = nullptr;
      if (hipMalloc(&d, w.hw.size()) != hipSuccess) return w;
      if (hipMemcpy(d, w.hw.data(), w.hw.size(), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return w;
      }
      w.dev = d;
      w.d = dplasma_desc_block_cyclic_lapack(c, prec, mb, nb, m, n, 0, 0, 0, 0, d, w.wlld, 1);
      return w;
    }
    void* dev = a;
    if (!on_device(a)) {   // host local array: through a device copy, written back by unwrap
      dev = nullptr;
      const size_t bytes = (size_t)w.lld * std::max(1, ln) * es;
      if (hipMalloc(&dev, bytes) != hipSuccess) return w;
      if (lm > 0 && ln > 0 &&
          hipMemcpy2D(dev, (size_t)w.lld * es, a, (size_t)w.lld * es, (size_t)lm * es, ln, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dev);
        return w;
      }
      w.host = (char*)a;
      w.copy = true;
      w.dev = dev;
      w.lm = lm;
      w.ln = ln;
    }
    w.d = dplasma_desc_block_cyclic_lapack(c, prec, mb, nb, m, n, 0, 0, 0, 0, dev, w.lld, 1);
    w.es = es;
    return w;
  }
  char* sub = (char*)a + ((size_t)(ia - 1) + (size_t)(ja - 1) * w.lld) * es;
  if (on_device(a)) {
    w.d = dplasma_desc_block_cyclic_lapack(c, prec, NAT_TILE, NAT_TILE, m, n, 1, 1, 0, 0, sub, w.lld, 1);
  } else {
    w.d = dplasma_desc_block_cyclic(c, prec, NAT_TILE, NAT_TILE, m, n, 1, 1, 123);
    if (w.d && dplasma_desc_set_lapack(w.d, sub, w.lld) != 0) {
      dplasma_desc_destroy(w.d);
      w.d = nullptr;
    }
    w.host = sub;
    w.copy = true;
  }
  return w;
}

void unwrap(Wrapped& w, bool write_back) {
  if (w.redist) {   // aligned copy -> the caller's (unaligned) operand
    if (write_back && w.d && w.dev &&
        hipMemcpy(w.hw.data(), w.dev, w.hw.size(), hipMemcpyDeviceToHost) == hipSuccess) {
      char* hs = w.src_dev ? w.hsrc.data() : (char*)w.src;
      if (nat_redistribute(native_ctx_any(), w.es, hs, w.slld, w.mb, w.nb, w.rsrc, w.csrc, w.ia, w.ja, w.m, w.n,
                           w.hw.data(), w.wlld, false) == 0 &&
          w.src_dev && w.sbytes)
        (void)hipMemcpy(w.src, hs, w.sbytes, hipMemcpyHostToDevice);
    }
    if (w.d) dplasma_desc_destroy(w.d);
    if (w.dev) (void)hipFree(w.dev);
    w.d = nullptr;
    w.dev = nullptr;
    return;
  }
  if (w.dev) {   // multi-process host local array
    if (write_back && w.d && w.lm > 0 && w.ln > 0)
      (void)hipMemcpy2D(w.host, (size_t)w.lld * w.es, w.dev, (size_t)w.lld * w.es, (size_t)w.lm * w.es, w.ln,
                        hipMemcpyDeviceToHost);
    if (w.d) dplasma_desc_destroy(w.d);
    (void)hipFree(w.dev);
    w.d = nullptr;
    w.dev = nullptr;
    return;
  }
  if (!w.d) return;
  if (w.copy && write_back) (void)dplasma_desc_get_lapack(w.d, w.host, w.lld);
  dplasma_desc_destroy(w.d);
  w.d = nullptr;
}

// the Python layer's 1 x 1 BLACS grid (created on first use; the GIL is held by the caller)
int python_grid() {
  static int h = -1;
  if (h < 0) {
    int one = 1;
    h = f77("gridinit", {iv(&one), iv(&one)});
  }
  return h;
}

int native_trans(const char* t) { return (*t == 'N' || *t == 'n') ? 111 : (*t == 'T' || *t == 't') ? 112 : 113; }
int native_uplo(const char* u) { return (*u == 'U' || *u == 'u') ? 121 : 122; }
int native_side(const char* s_) { return (*s_ == 'L' || *s_ == 'l') ? 141 : 142; }
int native_diag(const char* d) { return (*d == 'U' || *d == 'u') ? 132 : 131; }

}  // namespace

extern "C" {

// ---- runtime (parsec_init_wrapper_ / parsec_fini_wrapper_)
DPL_CAPI void parsec_init_wrapper_(void) {
  if (f77_native()) {
    native_ctx();   // one process; a multi-process context is created by blacs_gridinit_ (it needs the grid)
    return;
  }
  DplGil g;
  f77("init", {});
}
DPL_CAPI void parsec_fini_wrapper_(void) {
  if (f77_native()) {
    if (g_nctx) dplasma_fini(g_nctx);
    g_nctx = nullptr;
    return;
  }
  DplGil g;
  f77("fini", {});
}

// ---- BLACS / TOOLS subset (weak: a real BLACS library takes precedence)
DPL_CAPI __attribute__((weak)) void blacs_pinfo_(int* mypnum, int* nprocs) {
  if (f77_native()) {
    *mypnum = job_rank();
    *nprocs = job_world();
    return;
  }
  DplGil g;
  PyObject* r = dpl_call_fn("blacs_pinfo", {});
  if (r && PyTuple_Check(r)) {
    *mypnum = (int)PyLong_AsLong(PyTuple_GetItem(r, 0));
    *nprocs = (int)PyLong_AsLong(PyTuple_GetItem(r, 1));
  }
  Py_XDECREF(r);
}
DPL_CAPI __attribute__((weak)) void blacs_get_(int* icontxt, int* what, int* val) {
  (void)icontxt;
  (void)what;
  *val = 0;  // the system context
}
DPL_CAPI __attribute__((weak)) void blacs_gridinit_(int* icontxt, const char* order, int* nprow, int* npcol) {
  (void)order;
  if (f77_native()) {   // the grid must hold every process of the job (one process: 1 x 1)
    const int world = job_world();
    if (*nprow < 1 || *npcol < 1 || *nprow * *npcol != world ||
        (g_nctx && world > 1 && (*nprow != g_nprow || *npcol != g_npcol))) {
      dpl_set_error("blacs_gridinit: the native grid is nprow x npcol = WORLD_SIZE processes (one grid per job)");
      *icontxt = -1;
      return;
    }
    if (world > 1 && !g_nctx) {
      g_nctx = dplasma_init_native_dist(env_i("LOCAL_RANK", 0), job_rank(), world, *nprow, nullptr);
      if (!g_nctx) { *icontxt = -1; return; }
    }
    g_nprow = *nprow;
    g_npcol = *npcol;
    *icontxt = NATIVE_CTXT;
    return;
  }
  DplGil g;  // the argument objects are built before f77() runs: hold the GIL here
  *icontxt = f77("gridinit", {iv(nprow), iv(npcol)});
}
DPL_CAPI __attribute__((weak)) void blacs_gridinfo_(int* icontxt, int* nprow, int* npcol, int* myrow, int* mycol) {
  if (f77_native()) {
    const bool ok = *icontxt == NATIVE_CTXT;
    const int me = job_world() > 1 ? job_rank() : 0;
    *nprow = ok ? g_nprow : -1;
    *npcol = ok ? g_npcol : -1;
    *myrow = ok ? me / g_npcol : -1;
    *mycol = ok ? me % g_npcol : -1;
    return;
  }
  DplGil g;
  PyObject* r = dpl_call_fn("blacs_gridinfo", {iv(icontxt)});
  if (r && PyTuple_Check(r)) {
    *nprow = (int)PyLong_AsLong(PyTuple_GetItem(r, 0));
    *npcol = (int)PyLong_AsLong(PyTuple_GetItem(r, 1));
    *myrow = (int)PyLong_AsLong(PyTuple_GetItem(r, 2));
    *mycol = (int)PyLong_AsLong(PyTuple_GetItem(r, 3));
  } else {
    *nprow = *npcol = *myrow = *mycol = -1;
  }
  Py_XDECREF(r);
}
DPL_CAPI __attribute__((weak)) void blacs_gridexit_(int* icontxt) { (void)icontxt; }
DPL_CAPI __attribute__((weak)) int numroc_(int* n, int* nb, int* iproc, int* isrcproc, int* nprocs) {
  const int mydist = (*nprocs + *iproc - *isrcproc) % *nprocs;
  const int nblocks = *n / *nb;
  int num = (nblocks / *nprocs) * *nb;
  const int extra = nblocks % *nprocs;
  if (mydist < extra) num += *nb;
  else if (mydist == extra) num += *n % *nb;
  return num;
}
DPL_CAPI __attribute__((weak)) void descinit_(int* desc, int* m, int* n, int* mb, int* nb, int* irsrc, int* icsrc,
                                              int* ictxt, int* lld, int* info) {
  desc[0] = 1; desc[1] = *ictxt; desc[2] = *m; desc[3] = *n; desc[4] = *mb; desc[5] = *nb;
  desc[6] = *irsrc; desc[7] = *icsrc; desc[8] = *lld;
  *info = 0;
}

// C helper: a BLACS handle onto an existing dplasma context (grid of the context)
DPL_CAPI int dplasma_blacs_gridinit(dplasma_context_t* ctx) {
  DplGil g;
  PyObject* r = dpl_call_fn("gridinit_ctx", {(Py_INCREF(ctx->obj), ctx->obj)});
  const int v = r ? (int)PyLong_AsLong(r) : -1;
  Py_XDECREF(r);
  return v;
}

// p?latsqr_ workspace size, as the reference wrapper reports it (dplasma_wrapper_pdlatsqr.c:257-258):
// NB_A * (mloc + nloc + NB_A), local extents from numroc over the BLACS grid of DESCA
static int latsqr_work(const int* desca) {
  int ctxt = desca[1], nprow = 1, npcol = 1, myrow = 0, mycol = 0;
  blacs_gridinfo_(&ctxt, &nprow, &npcol, &myrow, &mycol);
  if (nprow < 1 || npcol < 1 || myrow < 0 || mycol < 0) nprow = npcol = 1, myrow = mycol = 0;
  int gm = desca[2], gn = desca[3], mb = desca[4], nb = desca[5], rsrc = desca[6], csrc = desca[7];
  const int mloc = numroc_(&gm, &mb, &myrow, &rsrc, &nprow);
  const int nloc = numroc_(&gn, &nb, &mycol, &csrc, &npcol);
  return nb * (mloc + nloc + nb);
}

// ---- p?gemm_, p?potrf_, p?getrf_, p?trsm_, p?trmm_, p?latsqr_
// native bodies of the ScaLAPACK entry points (1 x 1 grid, see f77_native); C = prec code
#define DPL_F77_NATIVE(P, T, C)                                                                                   \
  static void nat_p##P##gemm(const char* ta, const char* tb, int m, int n, int k, T alpha, T* a, int ia, int ja,  \
                             const int* da, T* b, int ib, int jb, const int* db, T beta, T* c, int ic, int jc,    \
                             const int* dc) {                                                                     \
    const int tA = native_trans(ta), tB = native_trans(tb);                                                      \
    Wrapped A = wrap(C, sizeof(T), a, ia, ja, da, tA == 111 ? m : k, tA == 111 ? k : m);                         \
    Wrapped B = wrap(C, sizeof(T), b, ib, jb, db, tB == 111 ? k : n, tB == 111 ? n : k);                         \
    Wrapped X = wrap(C, sizeof(T), c, ic, jc, dc, m, n);                                                          \
    if (A.d && B.d && X.d) (void)dplasma_##P##gemm(native_ctx(), tA, tB, alpha, A.d, B.d, beta, X.d);             \
    unwrap(A, false), unwrap(B, false), unwrap(X, true);                                                          \
  }                                                                                                               \
  static int nat_p##P##potrf(const char* uplo, int n, T* a, int ia, int ja, const int* da) {                      \
    Wrapped A = wrap(C, sizeof(T), a, ia, ja, da, n, n);                                                          \
    int info = A.d ? dplasma_##P##potrf(native_ctx(), native_uplo(uplo), A.d) : -1;                               \
    unwrap(A, true);                                                                                              \
    return info;                                                                                                  \
  }                                                                                                               \
  static int nat_p##P##getrf(int m, int n, T* a, int ia, int ja, const int* da, int* ipiv) {                      \
    const int k = m < n ? m : n;                                                                                  \
    Wrapped A = wrap(C, sizeof(T), a, ia, ja, da, m, n);                                                          \
    dplasma_desc_t* IP = A.d ? dplasma_desc_ipiv(native_ctx(), 1, NAT_TILE, 1, k, 1, 1) : nullptr;               \
    int info = IP ? dplasma_##P##getrf_1d(native_ctx(), A.d, IP) : -1;                                           \
    if (IP && ipiv) {                                                                                             \
      std::vector<int> p(k);                                                                                      \
      if (dplasma_desc_get_lapack(IP, p.data(), 1) == 0) {                                                        \
        if (dplasma_context_world(native_ctx()) > 1) {   /* ScaLAPACK layout: the entries of my local rows */  \
          /* (local row li of the whole local array -> global row gi; rows ia-1 .. ia-1+k of the operand */     \
          /*  hold the operand's pivots, as global rows of the whole matrix) */                                 \
          const int mbv = da[4], me = dplasma_context_rank(native_ctx()), myrow = me / g_npcol;                  \
          int gm = da[2], mbb = mbv, r = myrow, rs = da[6], pr = g_nprow;                                         \
          const int lm = numroc_(&gm, &mbb, &r, &rs, &pr), d = (myrow - rs + g_nprow) % g_nprow;                  \
          for (int li = 0; li < lm; ++li) {                                                                       \
            const int gi = ((li / mbv) * g_nprow + d) * mbv + li % mbv - (ia - 1);                                \
            if (gi >= 0 && gi < k) ipiv[li] = p[gi] + ia - 1;                                                     \
          }                                                                                                       \
        } else {                                                                                                  \
          for (int i = 0; i < k; ++i) ipiv[i] = p[i] + ia - 1;   /* global row of the whole array */           \
        }                                                                                                         \
      }                                                                                                           \
    }                                                                                                             \
    if (IP) dplasma_desc_destroy(IP);                                                                             \
    unwrap(A, true);                                                                                              \
    return info;                                                                                                  \
  }                                                                                                               \
  static void nat_p##P##trxm(bool solve, const char* side, const char* uplo, const char* ta, const char* diag,    \
                             int m, int n, T alpha, T* a, int ia, int ja, const int* da, T* b, int ib, int jb,    \
                             const int* db) {                                                                     \
    const int sd = native_side(side), ka = sd == 141 ? m : n;                                                     \
    Wrapped A = wrap(C, sizeof(T), a, ia, ja, da, ka, ka);                                                        \
    Wrapped B = wrap(C, sizeof(T), b, ib, jb, db, m, n);                                                          \
    if (A.d && B.d) {                                                                                             \
      if (solve)                                                                                                  \
        (void)dplasma_##P##trsm(native_ctx(), sd, native_uplo(uplo), native_trans(ta), native_diag(diag), alpha,  \
                                A.d, B.d);                                                                        \
      else                                                                                                        \
        (void)dplasma_##P##trmm(native_ctx(), sd, native_uplo(uplo), native_trans(ta), native_diag(diag), alpha,  \
                                A.d, B.d);                                                                        \
    }                                                                                                             \
    unwrap(A, false), unwrap(B, true);                                                                            \
  }                                                                                                               \
  static int nat_p##P##latsqr(int m, int n, T* a, int ia, int ja, const int* da, T* tau) {                        \
    Wrapped A = wrap(C, sizeof(T), a, ia, ja, da, m, n);                                                          \
    if (!A.d) { unwrap(A, false); return -1; }                                                                    \
    const int nb = da[4], ib = nb < 32 ? nb : 32, mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;                \
    dplasma_desc_t* Td = dplasma_desc_block_cyclic(native_ctx(), C, ib, nb, mt * ib, nt * nb, 0, 0, 123);        \
    int info = Td ? dplasma_##P##geqrf(native_ctx(), A.d, Td) : -1;                                               \
    if (info == 0 && tau) info = nat_qr_tau(Td, tau, m < n ? m : n);                                              \
    if (Td) dplasma_desc_destroy(Td);                                                                             \
    unwrap(A, true);                                                                                              \
    return info;                                                                                                  \
  }

DPL_F77_NATIVE(s, float, 2)
DPL_F77_NATIVE(d, double, 3)
DPL_F77_NATIVE(c, dplasma_complex32_t, 4)
DPL_F77_NATIVE(z, dplasma_complex64_t, 5)

#define DPL_F77_PREC(P, T)                                                                                      \
  DPL_CAPI void p##P##gemm_(const char* transa, const char* transb, int* m, int* n, int* k, T* alpha, T* a,      \
                            int* ia, int* ja, int* desca, T* b, int* ib, int* jb, int* descb, T* beta, T* c,     \
                            int* ic, int* jc, int* descc) {                                                      \
    if (native_grid(desca)) {                                                                                    \
      nat_p##P##gemm(transa, transb, *m, *n, *k, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb, *beta, c, *ic,  \
                     *jc, descc);                                                                                \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    f77("p" #P "gemm_", {chr(transa), chr(transb), iv(m), iv(n), iv(k), sc(alpha), dpl_arg_ptr(a), iv(ia),       \
                         iv(ja), desc_list(desca), dpl_arg_ptr(b), iv(ib), iv(jb), desc_list(descb), sc(beta),   \
                         dpl_arg_ptr(c), iv(ic), iv(jc), desc_list(descc)});                                     \
  }                                                                                                              \
  DPL_CAPI void p##P##potrf_(const char* uplo, int* n, T* a, int* ia, int* ja, int* desca, int* info) {          \
    if (native_grid(desca)) {                                                                                    \
      *info = nat_p##P##potrf(uplo, *n, a, *ia, *ja, desca);                                                     \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    *info = f77("p" #P "potrf_", {chr(uplo), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(desca)});          \
  }                                                                                                              \
  DPL_CAPI void p##P##getrf_(int* m, int* n, T* a, int* ia, int* ja, int* desca, int* ipiv, int* info) {        \
    if (native_grid(desca)) {                                                                                    \
      *info = nat_p##P##getrf(*m, *n, a, *ia, *ja, desca, ipiv);                                                 \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    *info = f77("p" #P "getrf_",                                                                                 \
                {iv(m), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(desca), dpl_arg_ptr(ipiv)});            \
  }                                                                                                              \
  DPL_CAPI void p##P##trsm_(const char* side, const char* uplo, const char* transa, const char* diag, int* m,    \
                            int* n, T* alpha, T* a, int* ia, int* ja, int* desca, T* b, int* ib, int* jb,        \
                            int* descb) {                                                                        \
    if (native_grid(desca)) {                                                                                    \
      nat_p##P##trxm(true, side, uplo, transa, diag, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb);    \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    f77("p" #P "trsm_", {chr(side), chr(uplo), chr(transa), chr(diag), iv(m), iv(n), sc(alpha), dpl_arg_ptr(a),  \
                         iv(ia), iv(ja), desc_list(desca), dpl_arg_ptr(b), iv(ib), iv(jb), desc_list(descb)});   \
  }                                                                                                              \
  DPL_CAPI void p##P##trmm_(const char* side, const char* uplo, const char* transa, const char* diag, int* m,    \
                            int* n, T* alpha, T* a, int* ia, int* ja, int* desca, T* b, int* ib, int* jb,        \
                            int* descb) {                                                                        \
    if (native_grid(desca)) {                                                                                    \
      nat_p##P##trxm(false, side, uplo, transa, diag, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb);   \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    f77("p" #P "trmm_", {chr(side), chr(uplo), chr(transa), chr(diag), iv(m), iv(n), sc(alpha), dpl_arg_ptr(a),  \
                         iv(ia), iv(ja), desc_list(desca), dpl_arg_ptr(b), iv(ib), iv(jb), desc_list(descb)});   \
  }                                                                                                              \
  DPL_CAPI void p##P##latsqr_(int* m, int* n, T* a, int* ia, int* ja, int* desca, T* tau, T* work, int* lwork,   \
                              int* info) {                                                                     \
    *info = 0;                                                                                                   \
    if (*m == 0 || *n == 0) return;                                                                              \
    /* optimal workspace NB_A * (Mp0 + Nq0 + NB_A) in WORK(1); LWORK = -1 is a pure query */                     \
    const int lw = latsqr_work(desca);                                                                           \
    if (work) work[0] = (T)lw;                                                                                   \
    if (*lwork == -1) return;                                                                                    \
    if (native_grid(desca) && job_world() > 1) {                                                                 \
      /* a multi-process grid: the native flat-tree QR of the grid (native_dist.cpp), R above and V below    */   \
      /* the diagonal in LAPACK's layout, TAU (replicated, MIN(M, N) entries) = the T factors' diagonal     */   \
      *info = nat_p##P##latsqr(*m, *n, a, *ia, *ja, desca, tau);                                                 \
      return;                                                                                                    \
    }                                                                                                            \
    DplGil g;                                                                                                    \
    int dpy[9];                                                                                                  \
    std::memcpy(dpy, desca, sizeof dpy);                                                                         \
    if (native_grid(desca)) dpy[1] = python_grid();   /* no native QR: the Python layer, 1 x 1 grid */        \
    *info = f77("p" #P "latsqr_", {iv(m), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(dpy),                 \
                                   dpl_arg_ptr(tau)});                                                           \
  }

DPL_F77_PREC(s, float)
DPL_F77_PREC(d, double)
DPL_F77_PREC(c, dplasma_complex32_t)
DPL_F77_PREC(z, dplasma_complex64_t)

}  // extern "C"
