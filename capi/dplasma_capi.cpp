// C ABI of dplasma_amd: embeds CPython and forwards each dplasma_<p><op>() to the framework.
//
// The reference exposes its algorithms as C functions over parsec_context_t and
// parsec_tiled_matrix_t (src/include/dplasma/dplasma_z.h).  Here the handles are Python objects
// (dplasma_amd.context.Context, dplasma_amd.descriptor.TiledMatrix) owned by this library; every
// call takes the GIL, converts the C arguments, calls dplasma_amd.capi.call() and returns int /
// double.  Works inside an existing interpreter too (then Py_Initialize is skipped).
#include "capi_bridge.h"

#include <dlfcn.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

static PyObject* g_capi = nullptr;   // module dplasma_amd.capi
static thread_local std::string g_err;
void dpl_set_error(const char* msg) { g_err = msg ? msg : ""; }

void dpl_keep_error();
static void keep_error() { dpl_keep_error(); }
void dpl_keep_error() {
  if (!PyErr_Occurred()) return;
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyObject* s = v ? PyObject_Str(v) : nullptr;
  g_err = s ? PyUnicode_AsUTF8(s) : "python error";
  Py_XDECREF(s);
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
}

// repository root = <dir of libdplasma.so>/../.. (dplasma_amd/lib/libdplasma.so)
static std::string lib_root() {
  Dl_info info;
  if (dladdr((void*)&lib_root, &info) && info.dli_fname) {
    // resolve symlinks: an installed prefix links lib/libdplasma.so -> lib/dplasma_amd/lib/libdplasma.so
    char* real = realpath(info.dli_fname, nullptr);
    std::string p(real ? real : info.dli_fname);
    free(real);
    for (int up = 0; up < 3; ++up) {
      const size_t s = p.find_last_of('/');
      if (s == std::string::npos) return ".";
      p = p.substr(0, s);
    }
    return p;
  }
  return ".";
}

static bool ensure_python();
bool dpl_ensure_python() { return ensure_python(); }
static bool ensure_python() {
  if (!Py_IsInitialized()) {
    Py_InitializeEx(0);
    PyEval_SaveThread();   // release the GIL; every entry point takes it with PyGILState_Ensure
  }
  if (g_capi) return true;
  PyGILState_STATE st = PyGILState_Ensure();
  const char* env = std::getenv("DPLASMA_ROOT");
  const std::string root = env ? env : lib_root();
  PyObject* sys_path = PySys_GetObject("path");  // borrowed
  PyObject* r = PyUnicode_FromString(root.c_str());
  if (sys_path && r) PyList_Insert(sys_path, 0, r);
  Py_XDECREF(r);
  g_capi = PyImport_ImportModule("dplasma_amd.capi");
  if (!g_capi) keep_error();
  PyGILState_Release(st);
  return g_capi != nullptr;
}

PyObject* dpl_arg_desc(const dplasma_desc_t* d) {
  if (!d) { Py_RETURN_NONE; }
  Py_INCREF(d->obj);
  return d->obj;
}
PyObject* dpl_arg_int(long long v) { return PyLong_FromLongLong(v); }
PyObject* dpl_arg_u64(unsigned long long v) { return PyLong_FromUnsignedLongLong(v); }
PyObject* dpl_arg_real(double v) { return PyFloat_FromDouble(v); }
PyObject* dpl_arg_cplx(dplasma_complex64_t v) { return PyComplex_FromDoubles(__real__ v, __imag__ v); }
PyObject* dpl_arg_cplx(dplasma_complex32_t v) { return PyComplex_FromDoubles(__real__ v, __imag__ v); }

PyObject* dpl_arg_ptr(const void* p) { return PyLong_FromUnsignedLongLong((unsigned long long)(uintptr_t)p); }
PyObject* dpl_arg_str(const char* s, int len) { return PyUnicode_FromStringAndSize(s ? s : "", s ? len : 0); }

static PyObject* call_obj(dplasma_context_t* ctx, const char* fname, const char* opname,
                          std::initializer_list<PyObject*> args) {
  if (!g_capi) {  // dplasma_amd could not be imported (or the interpreter is not up)
    for (PyObject* a : args) Py_XDECREF(a);
    if (g_err.empty()) g_err = "dplasma_amd is not initialised (dplasma_init failed or was not called)";
    return nullptr;
  }
  const size_t n = args.size() + (ctx ? 1 : 0) + (opname ? 1 : 0);
  PyObject* tup = PyTuple_New((Py_ssize_t)n);
  size_t i = 0;
  if (ctx) { Py_INCREF(ctx->obj); PyTuple_SET_ITEM(tup, i++, ctx->obj); }
  if (opname) PyTuple_SET_ITEM(tup, i++, PyUnicode_FromString(opname));
  bool bad = false;
  for (PyObject* a : args) {
    if (!a) { bad = true; a = Py_None; Py_INCREF(a); }
    PyTuple_SET_ITEM(tup, i++, a);
  }
  PyObject* res = nullptr;
  if (!bad) {
    PyObject* f = PyObject_GetAttrString(g_capi, fname);
    if (f) res = PyObject_CallObject(f, tup);
    Py_XDECREF(f);
  }
  Py_DECREF(tup);
  if (!res) keep_error();
  return res;
}

int dpl_call_int(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args) {
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  g_err.clear();
  PyObject* r = call_obj(ctx, "call", name, args);
  int v = -1;
  if (r) { v = (int)PyLong_AsLong(r); if (PyErr_Occurred()) { PyErr_Clear(); v = (int)PyFloat_AsDouble(r); } }
  Py_XDECREF(r);
  PyGILState_Release(st);
  return v;
}

double dpl_call_real(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args) {
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  g_err.clear();
  PyObject* r = call_obj(ctx, "call", name, args);
  double v = r ? PyFloat_AsDouble(r) : NAN;
  Py_XDECREF(r);
  PyGILState_Release(st);
  return v;
}

PyObject* dpl_call_fn(const char* fname, std::initializer_list<PyObject*> args) {
  g_err.clear();
  return call_obj(nullptr, fname, nullptr, args);
}

PyObject* dpl_arg_qrtree(const dplasma_qrtree_t* q) {
  PyObject* o = q && q->args ? (PyObject*)q->args : Py_None;
  Py_INCREF(o);
  return o;
}

PyObject* dpl_arg_obj(const void* h) {
  PyObject* o = h ? (PyObject*)h : Py_None;
  Py_INCREF(o);
  return o;
}

// a framework call that returns bytes: copied into a malloc'd array the caller owns (free / dplasma_but_free)
int dpl_call_bytes_out(dplasma_context_t* ctx, const char* name, void** out, std::initializer_list<PyObject*> args) {
  g_err.clear();
  PyObject* r = call_obj(ctx, "call_obj", name, args);
  if (!r) return -1;
  char* src = nullptr;
  Py_ssize_t len = 0;
  if (PyBytes_AsStringAndSize(r, &src, &len) != 0) {
    PyErr_Clear();
    Py_DECREF(r);
    g_err = std::string(name) + ": the framework did not return a byte vector";
    return -1;
  }
  void* v = std::malloc(len > 0 ? (size_t)len : 1);
  if (!v) {
    Py_DECREF(r);
    g_err = std::string(name) + ": host allocation failed";
    return -1;
  }
  std::memcpy(v, src, (size_t)len);
  Py_DECREF(r);
  if (out) *out = v;
  else std::free(v);
  return 0;
}

void dpl_tp_setter(dplasma_taskpool_t* tp, const char* name, int v) {
  if (!tp || !tp->obj) return;   // native taskpools have no recursive sub-DAGs to size
  DplGil g;
  g_err.clear();
  PyObject* r = call_obj(nullptr, "tp_setter", nullptr, {(Py_INCREF(tp->obj), tp->obj), PyUnicode_FromString(name),
                                                          PyLong_FromLong(v)});
  Py_XDECREF(r);
}

// ---- QR reduction trees (qr_param.h): the tree object lives in the framework; the query functions of
// the C handle ask it (each call takes the GIL)
static int qt_call(const dplasma_qrtree_t* q, const char* meth, std::initializer_list<int> a) {
  if (!q || !q->args) return -1;
  DplGil g;
  PyObject* tup = PyTuple_New((Py_ssize_t)a.size());
  Py_ssize_t i = 0;
  for (int v : a) PyTuple_SET_ITEM(tup, i++, PyLong_FromLong(v));
  PyObject* f = PyObject_GetAttrString((PyObject*)q->args, meth);
  PyObject* r = f ? PyObject_CallObject(f, tup) : nullptr;
  Py_XDECREF(f);
  Py_DECREF(tup);
  int v = -1;
  if (r) v = (int)PyLong_AsLong(r);
  else keep_error();
  Py_XDECREF(r);
  return v;
}
static int qt_getnbgeqrf(const dplasma_qrtree_t* q, int k) { return qt_call(q, "getnbgeqrf", {k}); }
static int qt_getm(const dplasma_qrtree_t* q, int k, int i) { return qt_call(q, "getm", {k, i}); }
static int qt_geti(const dplasma_qrtree_t* q, int k, int m) { return qt_call(q, "geti", {k, m}); }
static int qt_gettype(const dplasma_qrtree_t* q, int k, int m) { return qt_call(q, "gettype", {k, m}); }
static int qt_currpiv(const dplasma_qrtree_t* q, int k, int m) { return qt_call(q, "currpiv", {k, m}); }
static int qt_nextpiv(const dplasma_qrtree_t* q, int k, int p, int m) { return qt_call(q, "nextpiv", {k, p, m}); }
static int qt_prevpiv(const dplasma_qrtree_t* q, int k, int p, int m) { return qt_call(q, "prevpiv", {k, p, m}); }

// kind: "hqr" / "systolic" / "svd"; ints: that init's integer parameters (capi.qrtree_init)
static int qt_init(dplasma_qrtree_t* q, const char* kind, int trans, dplasma_desc_t* A, std::initializer_list<int> ints) {
  if (!q || !A) return -1;
  if (!A->obj) return nat_qrtree_init(q, kind, trans, A, ints);   // a native descriptor: the C++ tree (native_qrtree.cpp)
  DplGil g;
  g_err.clear();
  PyObject* il = PyTuple_New((Py_ssize_t)ints.size());
  Py_ssize_t i = 0;
  for (int v : ints) PyTuple_SET_ITEM(il, i++, PyLong_FromLong(v));
  PyObject* r = call_obj(nullptr, "qrtree_init", nullptr,
                         {PyUnicode_FromString(kind), PyLong_FromLong(trans), (Py_INCREF(A->obj), A->obj), il});
  if (!r) return -1;
  q->args = r;   // new reference, released by *_finalize
  q->getnbgeqrf = qt_getnbgeqrf;
  q->getm = qt_getm;
  q->geti = qt_geti;
  q->gettype = qt_gettype;
  q->currpiv = qt_currpiv;
  q->nextpiv = qt_nextpiv;
  q->prevpiv = qt_prevpiv;
  auto attr = [&](const char* n) {
    PyObject* v = PyObject_GetAttrString(r, n);
    const int x = v ? (int)PyLong_AsLong(v) : 0;
    Py_XDECREF(v);
    return x;
  };
  q->mt = attr("mt");
  q->nt = attr("nt");
  q->a = attr("a");
  q->p = attr("p");
  return 0;
}

static void qt_fini(dplasma_qrtree_t* q) {
  if (nat_qrtree_is(q)) return nat_qrtree_fini(q);
  if (!q || !q->args) return;
  DplGil g;
  Py_DECREF((PyObject*)q->args);
  q->args = nullptr;
}

static void qt_print(dplasma_desc_t* A, dplasma_qrtree_t* q, const char* what, int k, int* perm, const char* file) {
  (void)A;
  if (nat_qrtree_is(q)) return nat_qrtree_print(q, what, k, perm, file);
  if (!q || !q->args) return;
  DplGil g;
  PyObject* r = call_obj(nullptr, "qrtree_print", nullptr,
                         {(Py_INCREF((PyObject*)q->args), (PyObject*)q->args), PyUnicode_FromString(what),
                          PyLong_FromLong(k), PyLong_FromUnsignedLongLong((unsigned long long)(uintptr_t)perm),
                          PyUnicode_FromString(file ? file : "")});
  Py_XDECREF(r);
}

extern "C" {
DPL_CAPI int dplasma_hqr_init(dplasma_qrtree_t* q, int trans, dplasma_desc_t* A, int type_llvl, int type_hlvl, int a,
                              int p, int domino, int tsrr) {
  return qt_init(q, "hqr", trans, A, {type_llvl, type_hlvl, a, p, domino, tsrr});
}
DPL_CAPI void dplasma_hqr_finalize(dplasma_qrtree_t* q) { qt_fini(q); }
DPL_CAPI int dplasma_systolic_init(dplasma_qrtree_t* q, int trans, dplasma_desc_t* A, int p, int qq) {
  return qt_init(q, "systolic", trans, A, {p, qq});
}
DPL_CAPI void dplasma_systolic_finalize(dplasma_qrtree_t* q) { qt_fini(q); }
DPL_CAPI int dplasma_svd_init(dplasma_qrtree_t* q, int trans, dplasma_desc_t* A, int type_hlvl, int p,
                              int nbcores_per_node, int ratio) {
  return qt_init(q, "svd", trans, A, {type_hlvl, p, nbcores_per_node, ratio});
}
DPL_CAPI void dplasma_svd_finalize(dplasma_qrtree_t* q) { qt_fini(q); }
DPL_CAPI int dplasma_qrtree_check(dplasma_desc_t* A, dplasma_qrtree_t* q) {
  (void)A;
  if (nat_qrtree_is(q)) return nat_qrtree_check(q);
  if (!q || !q->args) return -1;
  DplGil g;
  g_err.clear();
  PyObject* r = call_obj(nullptr, "qrtree_check", nullptr, {(Py_INCREF((PyObject*)q->args), (PyObject*)q->args)});
  const int v = r ? (int)PyLong_AsLong(r) : 1;
  Py_XDECREF(r);
  return v;
}
DPL_CAPI void dplasma_qrtree_print_dag(dplasma_desc_t* A, dplasma_qrtree_t* q, char* f) { qt_print(A, q, "dag", -1, nullptr, f); }
DPL_CAPI void dplasma_qrtree_print_type(dplasma_desc_t* A, dplasma_qrtree_t* q) { qt_print(A, q, "type", -1, nullptr, nullptr); }
DPL_CAPI void dplasma_qrtree_print_pivot(dplasma_desc_t* A, dplasma_qrtree_t* q) { qt_print(A, q, "pivot", -1, nullptr, nullptr); }
DPL_CAPI void dplasma_qrtree_print_nbgeqrt(dplasma_desc_t* A, dplasma_qrtree_t* q) { qt_print(A, q, "nbgeqrt", -1, nullptr, nullptr); }
DPL_CAPI void dplasma_qrtree_print_perm(dplasma_desc_t* A, dplasma_qrtree_t* q, int* perm) { qt_print(A, q, "perm", -1, perm, nullptr); }
DPL_CAPI void dplasma_qrtree_print_next_k(dplasma_desc_t* A, dplasma_qrtree_t* q, int k) { qt_print(A, q, "next_k", k, nullptr, nullptr); }
DPL_CAPI void dplasma_qrtree_print_prev_k(dplasma_desc_t* A, dplasma_qrtree_t* q, int k) { qt_print(A, q, "prev_k", k, nullptr, nullptr); }
DPL_CAPI void dplasma_qrtree_print_geqrt_k(dplasma_desc_t* A, dplasma_qrtree_t* q, int k) { qt_print(A, q, "geqrt_k", k, nullptr, nullptr); }
// hebut's vector is a plain malloc'd array on native and framework contexts alike
DPL_CAPI void dplasma_but_free(void* h) { std::free(h); }
}  // extern "C"

dplasma_taskpool_t* dpl_call_new(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args) {
  g_err.clear();
  PyObject* o = call_obj(ctx, "new", name, args);
  if (!o) return nullptr;
  dplasma_taskpool_t* tp = new dplasma_taskpool_s;
  tp->obj = o;
  return tp;
}

extern "C" {

DPL_CAPI const char* dplasma_last_error(void) { return g_err.c_str(); }

// 1 once the embedded interpreter is up (never on a program that only uses native contexts)
DPL_CAPI int dplasma_python_active(void) { return Py_IsInitialized() ? 1 : 0; }

// ---- taskpool lifecycle (dplasma_<p><op>_New / _Destruct, parsec_context_add_taskpool / start / wait)
DPL_CAPI void dplasma_taskpool_free(dplasma_taskpool_t* tp) {
  if (!tp) return;
  if (tp->nat) {
    nat_free(tp);
    delete tp;
    return;
  }
  DplGil g;
  PyObject* r = call_obj(nullptr, "destruct", nullptr, {(Py_INCREF(tp->obj), tp->obj)});
  Py_XDECREF(r);
  Py_DECREF(tp->obj);
  delete tp;
}

DPL_CAPI int dplasma_context_add_taskpool(dplasma_context_t* ctx, dplasma_taskpool_t* tp) {
  if (!ctx || !tp) return -1;
  if (ctx->nat) return nat_add(ctx, tp);
  DplGil g;
  g_err.clear();
  PyObject* r = call_obj(ctx, "add_taskpool", nullptr, {(Py_INCREF(tp->obj), tp->obj)});
  const int v = r ? 0 : -1;
  Py_XDECREF(r);
  return v;
}

static int ctx_call(dplasma_context_t* ctx, const char* fn) {
  if (!ctx) return -1;
  if (ctx->nat) return fn[0] == 's' ? nat_start(ctx) : nat_wait(ctx);
  DplGil g;
  g_err.clear();
  PyObject* r = call_obj(ctx, fn, nullptr, {});
  const int v = r ? (int)PyLong_AsLong(r) : -1;
  Py_XDECREF(r);
  return v;
}
DPL_CAPI int dplasma_context_start(dplasma_context_t* ctx) { return ctx_call(ctx, "start"); }
DPL_CAPI int dplasma_context_wait(dplasma_context_t* ctx) { return ctx_call(ctx, "wait"); }

// info / result of a completed taskpool (what the blocking call would have returned)
DPL_CAPI int dplasma_taskpool_result(const dplasma_taskpool_t* tp) {
  if (!tp) return -1;
  if (tp->nat) return nat_result(tp);
  DplGil g;
  g_err.clear();
  PyObject* r = call_obj(nullptr, "tp_result", nullptr, {(Py_INCREF(tp->obj), tp->obj)});
  const int v = r ? (int)PyLong_AsLong(r) : -1;
  Py_XDECREF(r);
  return v;
}

// descriptor over caller-owned memory in ScaLAPACK / LAPACK local layout (column-major, lld):
// on_device != 0 -> a device pointer of the context's GPU (zero copy), else host memory.
DPL_CAPI dplasma_desc_t* dplasma_desc_block_cyclic_lapack(dplasma_context_t* ctx, int prec, int mb, int nb, int m,
                                                          int n, int P, int Q, int ip, int jq, void* data, int lld,
                                                          int on_device) {
  if (dpl_native(ctx)) {
    if (ip != 0 || jq != 0) { g_err = "native descriptor: ip = jq = 0 (one process)"; return nullptr; }
    return nat_desc(ctx, prec, mb, nb, m, n, P, Q, data, lld, on_device);
  }
  DplGil g;
  g_err.clear();
  PyObject* o = call_obj(ctx, "desc_lapack", nullptr,
                         {PyLong_FromLong(prec), PyLong_FromLong(mb), PyLong_FromLong(nb), PyLong_FromLong(m),
                          PyLong_FromLong(n), PyLong_FromLong(P), PyLong_FromLong(Q), PyLong_FromLong(ip),
                          PyLong_FromLong(jq), dpl_arg_ptr(data), PyLong_FromLong(lld), PyLong_FromLong(on_device)});
  if (!o) return nullptr;
  dplasma_desc_t* d = new dplasma_desc_s;
  d->obj = o;
  return d;
}

DPL_CAPI dplasma_context_t* dplasma_init(int nb_cores, int gpus) {
  if (!ensure_python()) return nullptr;
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* o = call_obj(nullptr, "init", nullptr, {PyLong_FromLong(nb_cores), PyLong_FromLong(gpus)});
  dplasma_context_t* c = nullptr;
  if (o) { c = new dplasma_context_s; c->obj = o; }
  PyGILState_Release(st);
  return c;
}

DPL_CAPI void dplasma_fini(dplasma_context_t* ctx) {
  if (!ctx) return;
  if (ctx->nat) {
    nat_fini(ctx);
    delete ctx;
    return;
  }
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* r = call_obj(ctx, "fini", nullptr, {});
  Py_XDECREF(r);
  Py_DECREF(ctx->obj);
  PyGILState_Release(st);
  delete ctx;
}

static int ctx_attr(const dplasma_context_t* ctx, const char* a) {
  if (!ctx) return -1;
  if (ctx->nat) return nat_ctx_attr(ctx, a[0] == 'r');
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* v = PyObject_GetAttrString(ctx->obj, a);
  const int r = v ? (int)PyLong_AsLong(v) : -1;
  Py_XDECREF(v);
  PyGILState_Release(st);
  return r;
}
DPL_CAPI int dplasma_context_rank(const dplasma_context_t* ctx) { return ctx_attr(ctx, "rank"); }
DPL_CAPI int dplasma_context_world(const dplasma_context_t* ctx) { return ctx_attr(ctx, "world"); }

DPL_CAPI dplasma_desc_t* dplasma_desc_block_cyclic(dplasma_context_t* ctx, int prec, int mb, int nb, int m, int n,
                                                   int P, int Q, dplasma_enum_t uplo) {
  if (dpl_native(ctx)) return nat_desc(ctx, prec, mb, nb, m, n, P, Q, nullptr, 0, 1);
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* o = call_obj(ctx, "desc_block_cyclic", nullptr,
                         {PyLong_FromLong(prec), PyLong_FromLong(mb), PyLong_FromLong(nb), PyLong_FromLong(m),
                          PyLong_FromLong(n), PyLong_FromLong(P), PyLong_FromLong(Q), PyLong_FromLong(uplo)});
  dplasma_desc_t* d = nullptr;
  if (o) { d = new dplasma_desc_s; d->obj = o; }
  PyGILState_Release(st);
  return d;
}

DPL_CAPI dplasma_desc_t* dplasma_desc_ipiv(dplasma_context_t* ctx, int mb, int nb, int m, int n, int P, int Q) {
  if (dpl_native(ctx)) {
    if (P > 1 || Q > 1) { nat_unsupported("desc_ipiv: P = Q = 1 on a native context"); return nullptr; }
    return nat_desc_int(ctx, mb, nb, m, n);
  }
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* o = call_obj(ctx, "desc_int", nullptr,
                         {PyLong_FromLong(mb), PyLong_FromLong(nb), PyLong_FromLong(m), PyLong_FromLong(n),
                          PyLong_FromLong(P), PyLong_FromLong(Q)});
  dplasma_desc_t* d = nullptr;
  if (o) { d = new dplasma_desc_s; d->obj = o; }
  PyGILState_Release(st);
  return d;
}

DPL_CAPI void dplasma_desc_destroy(dplasma_desc_t* A) {
  if (!A) return;
  if (A->nat) {
    nat_desc_free(A);
    delete A;
    return;
  }
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  Py_DECREF(A->obj);
  PyGILState_Release(st);
  delete A;
}

static int desc_io(const dplasma_desc_t* A, const void* host, int lda, const char* fn) {
  if (A && A->nat) return nat_desc_io(A, const_cast<void*>(host), lda, fn[5] == 's');
  dpl_ensure_python();
  PyGILState_STATE st = PyGILState_Ensure();
  PyObject* r = call_obj(nullptr, fn, nullptr,
                         {dpl_arg_desc(A), PyLong_FromUnsignedLongLong((unsigned long long)(uintptr_t)host),
                          PyLong_FromLong(lda)});
  const int v = r ? (int)PyLong_AsLong(r) : -1;
  Py_XDECREF(r);
  PyGILState_Release(st);
  return v;
}
DPL_CAPI int dplasma_desc_set_lapack(dplasma_desc_t* A, const void* host, int lda) {
  return desc_io(A, host, lda, "desc_set_lapack");
}
DPL_CAPI int dplasma_desc_get_lapack(const dplasma_desc_t* A, void* host, int lda) {
  return desc_io(A, host, lda, "desc_get_lapack");
}

}  // extern "C"
