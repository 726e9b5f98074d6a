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

#include <complex>

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

}  // namespace

extern "C" {

// ---- runtime (parsec_init_wrapper_ / parsec_fini_wrapper_)
DPL_CAPI void parsec_init_wrapper_(void) { DplGil g; f77("init", {}); }
DPL_CAPI void parsec_fini_wrapper_(void) { DplGil g; f77("fini", {}); }

// ---- BLACS / TOOLS subset (weak: a real BLACS library takes precedence)
DPL_CAPI __attribute__((weak)) void blacs_pinfo_(int* mypnum, int* nprocs) {
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
  DplGil g;  // the argument objects are built before f77() runs: hold the GIL here
  *icontxt = f77("gridinit", {iv(nprow), iv(npcol)});
}
DPL_CAPI __attribute__((weak)) void blacs_gridinfo_(int* icontxt, int* nprow, int* npcol, int* myrow, int* mycol) {
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
#define DPL_F77_PREC(P, T)                                                                                      \
  DPL_CAPI void p##P##gemm_(const char* transa, const char* transb, int* m, int* n, int* k, T* alpha, T* a,      \
                            int* ia, int* ja, int* desca, T* b, int* ib, int* jb, int* descb, T* beta, T* c,     \
                            int* ic, int* jc, int* descc) { DplGil g;                                                      \
    f77("p" #P "gemm_", {chr(transa), chr(transb), iv(m), iv(n), iv(k), sc(alpha), dpl_arg_ptr(a), iv(ia),       \
                         iv(ja), desc_list(desca), dpl_arg_ptr(b), iv(ib), iv(jb), desc_list(descb), sc(beta),   \
                         dpl_arg_ptr(c), iv(ic), iv(jc), desc_list(descc)});                                     \
  }                                                                                                              \
  DPL_CAPI void p##P##potrf_(const char* uplo, int* n, T* a, int* ia, int* ja, int* desca, int* info) { DplGil g; \
    *info = f77("p" #P "potrf_", {chr(uplo), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(desca)});          \
  }                                                                                                              \
  DPL_CAPI void p##P##getrf_(int* m, int* n, T* a, int* ia, int* ja, int* desca, int* ipiv, int* info) { DplGil g; \
    *info = f77("p" #P "getrf_",                                                                                 \
                {iv(m), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(desca), dpl_arg_ptr(ipiv)});            \
  }                                                                                                              \
  DPL_CAPI void p##P##trsm_(const char* side, const char* uplo, const char* transa, const char* diag, int* m,    \
                            int* n, T* alpha, T* a, int* ia, int* ja, int* desca, T* b, int* ib, int* jb,        \
                            int* descb) { DplGil g;                                                              \
    f77("p" #P "trsm_", {chr(side), chr(uplo), chr(transa), chr(diag), iv(m), iv(n), sc(alpha), dpl_arg_ptr(a),  \
                         iv(ia), iv(ja), desc_list(desca), dpl_arg_ptr(b), iv(ib), iv(jb), desc_list(descb)});   \
  }                                                                                                              \
  DPL_CAPI void p##P##trmm_(const char* side, const char* uplo, const char* transa, const char* diag, int* m,    \
                            int* n, T* alpha, T* a, int* ia, int* ja, int* desca, T* b, int* ib, int* jb,        \
                            int* descb) { DplGil g;                                                              \
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
    DplGil g;                                                                                                    \
    *info = f77("p" #P "latsqr_", {iv(m), iv(n), dpl_arg_ptr(a), iv(ia), iv(ja), desc_list(desca),               \
                                   dpl_arg_ptr(tau)});                                                           \
  }

DPL_F77_PREC(s, float)
DPL_F77_PREC(d, double)
DPL_F77_PREC(c, dplasma_complex32_t)
DPL_F77_PREC(z, dplasma_complex64_t)

}  // extern "C"
