// Internal header of the C ABI: Python embedding bridge used by the generated wrappers.
#pragma once
#include <Python.h>
#include <initializer_list>

#define DPL_CAPI __attribute__((visibility("default")))

typedef int dplasma_enum_t;
typedef __complex__ float dplasma_complex32_t;    // ABI of C's float _Complex
typedef __complex__ double dplasma_complex64_t;   // ABI of C's double _Complex
struct dplasma_context_s { PyObject* obj; };
struct dplasma_desc_s { PyObject* obj; };
struct dplasma_taskpool_s { PyObject* obj; };
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
