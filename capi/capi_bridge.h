// Internal header of the C ABI: Python embedding bridge used by the generated wrappers.
#pragma once
#include <Python.h>
#include <initializer_list>

#define DPL_CAPI __attribute__((visibility("default")))

typedef int dplasma_enum_t;
typedef __complex__ float dplasma_complex32_t;    // ABI of C's float _Complex
typedef __complex__ double dplasma_complex64_t;   // ABI of C's double _Complex
// Python-backed handles carry obj; handles of a native context (dplasma_init_native, native.cpp)
// carry nat instead and never touch the interpreter
struct NatCtx;
struct NatDesc;
struct NatProgram;
struct dplasma_context_s { PyObject* obj = nullptr; NatCtx* nat = nullptr; };
struct dplasma_desc_s { PyObject* obj = nullptr; NatDesc* nat = nullptr; };
struct dplasma_taskpool_s { PyObject* obj = nullptr; NatProgram* nat = nullptr; };
typedef struct dplasma_context_s dplasma_context_t;
typedef struct dplasma_desc_s dplasma_desc_t;
typedef struct dplasma_taskpool_s dplasma_taskpool_t;

// starts the interpreter and imports dplasma_amd.capi on first use (false + error kept on failure)
bool dpl_ensure_python();

// GIL held for the whole forwarded call, including the construction of its arguments; the
// interpreter is brought up first, so any entry point may be the first call of the program
struct DplGil {
  PyGILState_STATE st;
  DplGil() : st((dpl_ensure_python(), PyGILState_Ensure())) {}
  ~DplGil() { PyGILState_Release(st); }
};

// one argument of a forwarded call (a new reference, or nullptr on error)
PyObject* dpl_arg_desc(const dplasma_desc_t* d);
PyObject* dpl_arg_int(long long v);
PyObject* dpl_arg_u64(unsigned long long v);
PyObject* dpl_arg_real(double v);
PyObject* dpl_arg_cplx(dplasma_complex64_t v);
PyObject* dpl_arg_cplx(dplasma_complex32_t v);

// QR reduction tree handle (same layout as dplasma.h / the reference's qr_param.h struct)
typedef struct dplasma_qrtree_s dplasma_qrtree_t;
#ifndef DPLASMA_QRTREE_DEFINED
#define DPLASMA_QRTREE_DEFINED
struct dplasma_qrtree_s {
  int (*getnbgeqrf)(const dplasma_qrtree_t*, int);
  int (*getm)(const dplasma_qrtree_t*, int, int);
  int (*geti)(const dplasma_qrtree_t*, int, int);
  int (*gettype)(const dplasma_qrtree_t*, int, int);
  int (*currpiv)(const dplasma_qrtree_t*, int, int);
  int (*nextpiv)(const dplasma_qrtree_t*, int, int, int);
  int (*prevpiv)(const dplasma_qrtree_t*, int, int, int);
  int mt, nt, a, p;
  void* args;   // PyObject* of the framework's tree (a strong reference)
};
#endif
PyObject* dpl_arg_qrtree(const dplasma_qrtree_t* q);
// trees of native descriptors (native_qrtree.cpp): q->args is the C++ tree, the queries answer from it
namespace nq { class Tree; }
bool nat_qrtree_is(const dplasma_qrtree_t* q);
nq::Tree* nat_qrtree(const dplasma_qrtree_t* q);
int nat_qrtree_init(dplasma_qrtree_t* q, const char* kind, int trans, dplasma_desc_t* A, std::initializer_list<int> ints);
void nat_qrtree_fini(dplasma_qrtree_t* q);
int nat_qrtree_check(const dplasma_qrtree_t* q);
void nat_qrtree_print(const dplasma_qrtree_t* q, const char* what, int k, int* perm, const char* file);
// an opaque framework object handed to C earlier (butterfly vectors): a new reference to it
PyObject* dpl_arg_obj(const void* h);
// "call" returning an object: stored as a new reference in *out (0), or -1
int dpl_call_bytes_out(dplasma_context_t* ctx, const char* name, void** out, std::initializer_list<PyObject*> args);
// tp_setter(tp, name, v): a taskpool parameter (dplasma_<p>potrf_setrecursive, ...)
void dpl_tp_setter(dplasma_taskpool_t* tp, const char* name, int v);

PyObject* dpl_arg_ptr(const void* p);
PyObject* dpl_arg_str(const char* s, int len);
void dpl_keep_error();

// dplasma_amd.capi.<fname>(*args) with the GIL held -> new reference or nullptr (error kept)
PyObject* dpl_call_fn(const char* fname, std::initializer_list<PyObject*> args);
// dplasma_amd.capi.new(ctx, name, *args) -> taskpool handle (nullptr on error)
dplasma_taskpool_t* dpl_call_new(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args);

// dplasma_amd.capi.call(ctx, name, *args) -> int / double (errors: -1 / NaN, message kept)
int dpl_call_int(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args);
double dpl_call_real(dplasma_context_t* ctx, const char* name, std::initializer_list<PyObject*> args);

// error message of the calling thread (dplasma_last_error)
void dpl_set_error(const char* msg);

// ---- native single-GPU engine (native.cpp)
bool dpl_native(const dplasma_context_t* ctx);
int nat_ctx_attr(const dplasma_context_t* ctx, bool rank);   // rank / world of a native context
int nat_unsupported(const char* op);
NatProgram* nat_potrf(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A);
NatProgram* nat_potrs(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_posv(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_gemm(dplasma_context_t* ctx, int prec, int tA, int tB, const void* alpha, dplasma_desc_t* A,
                     dplasma_desc_t* B, const void* beta, dplasma_desc_t* C);
NatProgram* nat_trsm(dplasma_context_t* ctx, int prec, int side, int uplo, int trans, int diag, const void* alpha,
                     dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_plghe(dplasma_context_t* ctx, int prec, double bump, int uplo, dplasma_desc_t* A,
                      unsigned long long seed);
NatProgram* nat_plrnt(dplasma_context_t* ctx, int prec, int diagdom, dplasma_desc_t* A, unsigned long long seed);
NatProgram* nat_plgsy(dplasma_context_t* ctx, int prec, const void* bump, int uplo, dplasma_desc_t* A,
                      unsigned long long seed);
NatProgram* nat_herk(dplasma_context_t* ctx, int prec, int uplo, int trans, double alpha, dplasma_desc_t* A,
                     double beta, dplasma_desc_t* C);
NatProgram* nat_syrk(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                     const void* beta, dplasma_desc_t* C);
NatProgram* nat_her2k(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      dplasma_desc_t* B, double beta, dplasma_desc_t* C);
NatProgram* nat_syr2k(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      dplasma_desc_t* B, const void* beta, dplasma_desc_t* C);
NatProgram* nat_trtri(dplasma_context_t* ctx, int prec, int uplo, int diag, dplasma_desc_t* A);
NatProgram* nat_lauum(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A);
NatProgram* nat_potri(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A);
NatProgram* nat_poinv(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A);
NatProgram* nat_geadd(dplasma_context_t* ctx, int prec, int trans, const void* alpha, dplasma_desc_t* A,
                      const void* beta, dplasma_desc_t* B);
NatProgram* nat_tradd(dplasma_context_t* ctx, int prec, int uplo, int trans, const void* alpha, dplasma_desc_t* A,
                      const void* beta, dplasma_desc_t* B);
NatProgram* nat_lacpy(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_laset(dplasma_context_t* ctx, int prec, int uplo, const void* alpha, const void* beta,
                      dplasma_desc_t* A);
NatProgram* nat_lascal(dplasma_context_t* ctx, int prec, int uplo, const void* alpha, dplasma_desc_t* A);
double nat_lange(dplasma_context_t* ctx, int prec, int ntype, dplasma_desc_t* A);   // NAN + error on failure
double nat_lantr(dplasma_context_t* ctx, int prec, int ntype, int uplo, int diag, dplasma_desc_t* A);
NatProgram* nat_trmm(dplasma_context_t* ctx, int prec, int side, int uplo, int trans, int diag, const void* alpha,
                     dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_symm(dplasma_context_t* ctx, int prec, int side, int uplo, const void* alpha, dplasma_desc_t* A,
                     dplasma_desc_t* B, const void* beta, dplasma_desc_t* C);
NatProgram* nat_hemm(dplasma_context_t* ctx, int prec, int side, int uplo, const void* alpha, dplasma_desc_t* A,
                     dplasma_desc_t* B, const void* beta, dplasma_desc_t* C);
double nat_lansy(dplasma_context_t* ctx, int prec, int ntype, int uplo, dplasma_desc_t* A);
double nat_lanhe(dplasma_context_t* ctx, int prec, int ntype, int uplo, dplasma_desc_t* A);
NatProgram* nat_getrf_1d(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* IPIV);
NatProgram* nat_getrs(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* A, dplasma_desc_t* IPIV,
                      dplasma_desc_t* B);
NatProgram* nat_gesv_1d(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* IPIV,
                        dplasma_desc_t* B);
dplasma_desc_t* nat_desc_int(dplasma_context_t* ctx, int mb, int nb, int m, int n);
NatProgram* nat_geqrf(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T);
NatProgram* nat_unmqr(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_desc_t* A, dplasma_desc_t* T,
                      dplasma_desc_t* C);
NatProgram* nat_ungqr(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T, dplasma_desc_t* Q);
NatProgram* nat_geqrs(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T, dplasma_desc_t* B);
NatProgram* nat_gels(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* A, dplasma_desc_t* T,
                     dplasma_desc_t* B);
// F77 layer: ScaLAPACK submatrix (ia, ja, m x n of a matrix in mb x nb blocks from process (rsrc, csrc)) <->
// the aligned block-cyclic copy (from process (0, 0)); host local arrays of this rank; 0 on success
int nat_redistribute(dplasma_context_t* ctx, int es, char* src, int slld, int mb, int nb, int rsrc, int csrc, int ia,
                     int ja, int m, int n, char* dst, int dlld, bool to_aligned);
int nat_qr_tau(dplasma_desc_t* T, void* tau, int k);
NatProgram* nat_getrf_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* L, dplasma_desc_t* IPIV);
NatProgram* nat_trsmpl_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* L,
                              dplasma_desc_t* IPIV, dplasma_desc_t* B);
NatProgram* nat_getrs_incpiv(dplasma_context_t* ctx, int prec, int trans, dplasma_desc_t* A, dplasma_desc_t* L,
                             dplasma_desc_t* IPIV, dplasma_desc_t* B);
NatProgram* nat_gesv_incpiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* L,
                            dplasma_desc_t* IPIV, dplasma_desc_t* B);
NatProgram* nat_getrf_nopiv(dplasma_context_t* ctx, int prec, dplasma_desc_t* A);
NatProgram* nat_gelqf(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T);
NatProgram* nat_unmlq(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_desc_t* A, dplasma_desc_t* T,
                      dplasma_desc_t* C);
NatProgram* nat_unglq(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T, dplasma_desc_t* Q);
NatProgram* nat_gelqs(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* T, dplasma_desc_t* B);
NatProgram* nat_ger(dplasma_context_t* ctx, int prec, int conj, const void* alpha, dplasma_desc_t* X, dplasma_desc_t* Y,
                    dplasma_desc_t* A);
NatProgram* nat_laswp(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* IPIV, int inc);
double nat_lanm2(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, int* info);
NatProgram* nat_trsmpl_ptgpanel(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* IPIV,
                                dplasma_desc_t* B);
NatProgram* nat_hetrf(dplasma_context_t* ctx, int prec, dplasma_desc_t* A);
int nat_hetrs(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A, dplasma_desc_t* B, const void* U_but_vec,
              int level);
int nat_gebmm(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, const void* U, int level, int trans);
int nat_gebut(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, const void* U, int level);
int nat_hebut(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, void** U_out, int level);
NatProgram* nat_geqrf_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT);
NatProgram* nat_gelqf_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT);
NatProgram* nat_unmqr_param(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_qrtree_t* q, dplasma_desc_t* A,
                            dplasma_desc_t* TS, dplasma_desc_t* TT, dplasma_desc_t* C);
NatProgram* nat_unmlq_param(dplasma_context_t* ctx, int prec, int side, int trans, dplasma_qrtree_t* q, dplasma_desc_t* A,
                            dplasma_desc_t* TS, dplasma_desc_t* TT, dplasma_desc_t* C);
NatProgram* nat_ungqr_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT, dplasma_desc_t* Q);
NatProgram* nat_unglq_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT, dplasma_desc_t* Q);
NatProgram* nat_geqrs_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT, dplasma_desc_t* B);
NatProgram* nat_gelqs_param(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* TS,
                            dplasma_desc_t* TT, dplasma_desc_t* B);
NatProgram* nat_getrf_qrf(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* IPIV,
                          dplasma_desc_t* TS, dplasma_desc_t* TT, int criteria, double alpha, int* lu_tab, int* INFO);
NatProgram* nat_trsmpl_qrf(dplasma_context_t* ctx, int prec, dplasma_qrtree_t* q, dplasma_desc_t* A, dplasma_desc_t* IPIV,
                           dplasma_desc_t* B, dplasma_desc_t* TS, dplasma_desc_t* TT, int* lu_tab);
NatProgram* nat_herbt(dplasma_context_t* ctx, int prec, int uplo, int ib, dplasma_desc_t* A, dplasma_desc_t* T);
NatProgram* nat_hbrdt(dplasma_context_t* ctx, int prec, dplasma_desc_t* A);
NatProgram* nat_heev(dplasma_context_t* ctx, int prec, int jobz, int uplo, dplasma_desc_t* A, dplasma_desc_t* W,
                     dplasma_desc_t* Z);
NatProgram* nat_gebrd_ge2gb(dplasma_context_t* ctx, int prec, int ib, dplasma_desc_t* A, dplasma_desc_t* Band);
NatProgram* nat_gebrd_ge2gbx(dplasma_context_t* ctx, int prec, int ib, dplasma_qrtree_t* qt0, dplasma_qrtree_t* qt,
                             dplasma_qrtree_t* lqt, dplasma_desc_t* A, dplasma_desc_t* TS0, dplasma_desc_t* TT0,
                             dplasma_desc_t* TS, dplasma_desc_t* TT, dplasma_desc_t* Band);
NatProgram* nat_trdsm(dplasma_context_t* ctx, int prec, dplasma_desc_t* A, dplasma_desc_t* B);
NatProgram* nat_trmdm(dplasma_context_t* ctx, int prec, dplasma_desc_t* A);
int nat_latms(dplasma_context_t* ctx, int prec, int mtxtype, double cond, dplasma_desc_t* A, unsigned long long seed);
int nat_pltmg(dplasma_context_t* ctx, int prec, int mtxtype, dplasma_desc_t* A, unsigned long long seed);
int nat_print(dplasma_context_t* ctx, int prec, int uplo, dplasma_desc_t* A);
int nat_execute(dplasma_context_t* ctx, NatProgram* P);     // run + wait + info, frees P
dplasma_taskpool_t* nat_wrap(NatProgram* P);
void nat_fini(dplasma_context_t* ctx);
dplasma_desc_t* nat_desc(dplasma_context_t* ctx, int prec, int mb, int nb, int m, int n, int P, int Q, void* data,
                         int lld, int on_device);
void nat_desc_free(dplasma_desc_t* A);
int nat_desc_io(const dplasma_desc_t* A, void* host, int lda, bool to_device);
int nat_add(dplasma_context_t* ctx, dplasma_taskpool_t* tp);
int nat_start(dplasma_context_t* ctx);
int nat_wait(dplasma_context_t* ctx);
int nat_result(const dplasma_taskpool_t* tp);
void nat_free(dplasma_taskpool_t* tp);
