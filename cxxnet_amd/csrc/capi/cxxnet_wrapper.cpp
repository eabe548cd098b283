// libcxxnetwrapper.so: the CXN* C ABI over cxxnet_amd.
//
// The trainer, executor and kernels live behind the Python-level orchestration
// (cxxnet_amd.wrapper).  This library embeds CPython, or joins the running
// interpreter when it is loaded from Python.  Each CXN* call holds the GIL and
// forwards to the wrapper objects.  Result arrays are copied into buffers owned
// by the handle, matching the reference's "valid until the next call" contract
// (wrapper/cxxnet_wrapper.cpp: res_pred / temp2 / temp4 members).
#include "cxxnet_wrapper.h"

#include <Python.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::once_flag g_init;
PyObject *g_mod = nullptr;  // cxxnet_amd.wrapper

std::string PackageRoot() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void *>(&PackageRoot), &info) == 0 || info.dli_fname == nullptr) return "";
  std::string p = info.dli_fname;  // <root>/cxxnet_amd/_native/libcxxnetwrapper.so
  for (int i = 0; i < 3; ++i) {
    size_t s = p.find_last_of('/');
    if (s == std::string::npos) return "";
    p = p.substr(0, s);
  }
  return p;
}

void Init() {
  std::call_once(g_init, [] {
    bool own = !Py_IsInitialized();
    if (own) Py_InitializeEx(0);
    PyGILState_STATE st = PyGILState_Ensure();
    std::string root = PackageRoot();
    if (!root.empty()) {
      PyObject *sys_path = PySys_GetObject("path");  // borrowed
      PyObject *r = PyUnicode_FromString(root.c_str());
      if (sys_path != nullptr && r != nullptr && PySequence_Contains(sys_path, r) == 0) PyList_Insert(sys_path, 0, r);
      Py_XDECREF(r);
    }
    g_mod = PyImport_ImportModule("cxxnet_amd.wrapper");
    if (g_mod == nullptr) {
      PyErr_Print();
      std::fprintf(stderr, "cxxnet: cannot import cxxnet_amd.wrapper\n");
    }
    PyGILState_Release(st);
    // An interpreter we created keeps running; release the GIL so that any
    // thread (including this one, through PyGILState_Ensure) can take it.
    if (own) PyEval_SaveThread();
  });
}

struct Gil {
  PyGILState_STATE st;
  Gil() {
    Init();
    st = PyGILState_Ensure();
  }
  ~Gil() { PyGILState_Release(st); }
};

// Reports a pending Python exception the way the reference reports errors.
bool Failed(PyObject *r, const char *what) {
  if (r != nullptr) return false;
  std::fprintf(stderr, "cxxnet: %s failed\n", what);
  PyErr_Print();
  return true;
}

PyObject *Attr(const char *name) { return g_mod ? PyObject_GetAttrString(g_mod, name) : nullptr; }

struct Handle {
  PyObject *obj = nullptr;
  std::vector<float> buf;  // last returned array
  std::string str;         // last returned string
};

PyObject *Shape(const cxx_uint *s, int n) {
  PyObject *t = PyTuple_New(n);
  for (int i = 0; i < n; ++i) PyTuple_SET_ITEM(t, i, PyLong_FromUnsignedLong(s[i]));
  return t;
}

PyObject *View(const float *p, size_t n) {
  return PyMemoryView_FromMemory(reinterpret_cast<char *>(const_cast<float *>(p)),
                                 static_cast<Py_ssize_t>(n * sizeof(float)), PyBUF_READ);
}

size_t Count(const cxx_uint *s, int n) {
  size_t c = 1;
  for (int i = 0; i < n; ++i) c *= s[i];
  return c;
}

// (bytes, shape) -> handle buffer; writes up to `maxdim` dims into oshape.
const float *Take(Handle *h, PyObject *res, cxx_uint *oshape, int maxdim, cxx_uint *ndim) {
  if (res == nullptr) return nullptr;
  PyObject *b = PyTuple_GetItem(res, 0);
  PyObject *shape = PyTuple_GetItem(res, 1);
  char *data = nullptr;
  Py_ssize_t len = 0;
  if (b == nullptr || shape == nullptr || PyBytes_AsStringAndSize(b, &data, &len) != 0) {
    PyErr_Print();
    Py_DECREF(res);
    return nullptr;
  }
  Py_ssize_t nd = PyTuple_Size(shape);
  if (ndim != nullptr) *ndim = static_cast<cxx_uint>(nd);
  for (int i = 0; i < maxdim; ++i) {
    oshape[i] = 1;
  }
  // Dims beyond the array's rank stay 1.
  for (Py_ssize_t i = 0; i < nd && i < maxdim; ++i) {
    oshape[i] = static_cast<cxx_uint>(PyLong_AsUnsignedLong(PyTuple_GetItem(shape, i)));
  }
  h->buf.assign(reinterpret_cast<float *>(data), reinterpret_cast<float *>(data) + len / sizeof(float));
  Py_DECREF(res);
  return h->buf.empty() ? nullptr : h->buf.data();
}

}  // namespace

extern "C" {

// ----------------------------------------------------------------------------- iterator
void *CXNIOCreateFromConfig(const char *cfg) {
  Gil g;
  PyObject *cls = Attr("DataIter");
  PyObject *obj = cls ? PyObject_CallFunction(cls, "s", cfg) : nullptr;
  Py_XDECREF(cls);
  if (Failed(obj, "CXNIOCreateFromConfig")) return nullptr;
  Handle *h = new Handle();
  h->obj = obj;
  return h;
}

int CXNIONext(void *handle) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *r = PyObject_CallMethod(h->obj, "next", nullptr);
  if (Failed(r, "CXNIONext")) return 0;
  int ok = PyObject_IsTrue(r);
  Py_DECREF(r);
  return ok;
}

void CXNIOBeforeFirst(void *handle) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *r = PyObject_CallMethod(h->obj, "before_first", nullptr);
  if (!Failed(r, "CXNIOBeforeFirst")) Py_DECREF(r);
}

const cxx_real_t *CXNIOGetData(void *handle, cxx_uint oshape[4], cxx_uint *ostride) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_io_data");
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, nullptr) : nullptr;
  Py_XDECREF(fn);
  if (Failed(r, "CXNIOGetData")) return nullptr;
  const float *p = Take(h, r, oshape, 4, nullptr);
  *ostride = oshape[3];
  return p;
}

const cxx_real_t *CXNIOGetLabel(void *handle, cxx_uint oshape[2], cxx_uint *ostride) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_io_label");
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, nullptr) : nullptr;
  Py_XDECREF(fn);
  if (Failed(r, "CXNIOGetLabel")) return nullptr;
  const float *p = Take(h, r, oshape, 2, nullptr);
  *ostride = oshape[1];
  return p;
}

void CXNIOFree(void *handle) {
  if (handle == nullptr) return;
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  Py_XDECREF(h->obj);
  delete h;
}

// ----------------------------------------------------------------------------- net
void *CXNNetCreate(const char *device, const char *cfg) {
  Gil g;
  PyObject *cls = Attr("Net");
  PyObject *obj = cls ? PyObject_CallFunction(cls, "ss", device ? device : "", cfg ? cfg : "") : nullptr;
  Py_XDECREF(cls);
  if (Failed(obj, "CXNNetCreate")) return nullptr;
  Handle *h = new Handle();
  h->obj = obj;
  return h;
}

void CXNNetFree(void *handle) { CXNIOFree(handle); }

#define CXN_VOID_CALL(what, ...)                                         \
  do {                                                                   \
    Gil g;                                                               \
    Handle *h = static_cast<Handle *>(handle);                          \
    PyObject *r = PyObject_CallMethod(h->obj, __VA_ARGS__);              \
    if (!Failed(r, what)) Py_DECREF(r);                                  \
  } while (0)

void CXNNetSetParam(void *handle, const char *name, const char *val) {
  CXN_VOID_CALL("CXNNetSetParam", "set_param", "ss", name, val);
}
void CXNNetInitModel(void *handle) { CXN_VOID_CALL("CXNNetInitModel", "init_model", nullptr); }
void CXNNetSaveModel(void *handle, const char *fname) { CXN_VOID_CALL("CXNNetSaveModel", "save_model", "s", fname); }
void CXNNetLoadModel(void *handle, const char *fname) { CXN_VOID_CALL("CXNNetLoadModel", "load_model", "s", fname); }
void CXNNetStartRound(void *handle, int round) { CXN_VOID_CALL("CXNNetStartRound", "start_round", "i", round); }

void CXNNetUpdateIter(void *handle, void *data_handle) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  Handle *d = static_cast<Handle *>(data_handle);
  PyObject *r = PyObject_CallMethod(h->obj, "update", "O", d->obj);
  if (!Failed(r, "CXNNetUpdateIter")) Py_DECREF(r);
}

void CXNNetSetWeight(void *handle, cxx_real_t *p_weight, cxx_uint size_weight, const char *layer_name,
                     const char *wtag) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_set_weight");
  PyObject *mv = View(p_weight, size_weight);
  PyObject *r = fn ? PyObject_CallFunction(fn, "OOIss", h->obj, mv, size_weight, layer_name, wtag) : nullptr;
  Py_XDECREF(fn);
  Py_XDECREF(mv);
  if (!Failed(r, "CXNNetSetWeight")) Py_DECREF(r);
}

const cxx_real_t *CXNNetGetWeight(void *handle, const char *layer_name, const char *wtag, cxx_uint wshape[4],
                                  cxx_uint *out_dim) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_get_weight");
  PyObject *r = fn ? PyObject_CallFunction(fn, "Oss", h->obj, layer_name, wtag) : nullptr;
  Py_XDECREF(fn);
  *out_dim = 0;
  if (Failed(r, "CXNNetGetWeight")) return nullptr;
  return Take(h, r, wshape, 4, out_dim);
}

void CXNNetUpdateBatch(void *handle, cxx_real_t *p_data, const cxx_uint dshape[4], cxx_real_t *p_label,
                       const cxx_uint lshape[2]) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_update_batch");
  PyObject *md = View(p_data, Count(dshape, 4));
  PyObject *ml = View(p_label, Count(lshape, 2));
  PyObject *sd = Shape(dshape, 4), *sl = Shape(lshape, 2);
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, md, sd, ml, sl, nullptr) : nullptr;
  Py_XDECREF(fn);
  Py_XDECREF(md);
  Py_XDECREF(ml);
  Py_XDECREF(sd);
  Py_XDECREF(sl);
  if (!Failed(r, "CXNNetUpdateBatch")) Py_DECREF(r);
}

const cxx_real_t *CXNNetPredictBatch(void *handle, cxx_real_t *p_data, const cxx_uint dshape[4],
                                     cxx_uint *out_size) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_predict_batch");
  PyObject *md = View(p_data, Count(dshape, 4));
  PyObject *sd = Shape(dshape, 4);
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, md, sd, nullptr) : nullptr;
  Py_XDECREF(fn);
  Py_XDECREF(md);
  Py_XDECREF(sd);
  *out_size = 0;
  if (Failed(r, "CXNNetPredictBatch")) return nullptr;
  cxx_uint shp[1];
  const float *p = Take(h, r, shp, 1, nullptr);
  *out_size = static_cast<cxx_uint>(h->buf.size());
  return p;
}

const cxx_real_t *CXNNetPredictIter(void *handle, void *data_handle, cxx_uint *out_size) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  Handle *d = static_cast<Handle *>(data_handle);
  PyObject *fn = Attr("_capi_predict_iter");
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, d->obj, nullptr) : nullptr;
  Py_XDECREF(fn);
  *out_size = 0;
  if (Failed(r, "CXNNetPredictIter")) return nullptr;
  cxx_uint shp[1];
  const float *p = Take(h, r, shp, 1, nullptr);
  *out_size = static_cast<cxx_uint>(h->buf.size());
  return p;
}

const cxx_real_t *CXNNetExtractBatch(void *handle, cxx_real_t *p_data, const cxx_uint dshape[4],
                                     const char *node_name, cxx_uint oshape[4]) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  PyObject *fn = Attr("_capi_extract_batch");
  PyObject *md = View(p_data, Count(dshape, 4));
  PyObject *sd = Shape(dshape, 4);
  PyObject *nm = PyUnicode_FromString(node_name);
  PyObject *r = fn ? PyObject_CallFunctionObjArgs(fn, h->obj, md, sd, nm, nullptr) : nullptr;
  Py_XDECREF(fn);
  Py_XDECREF(md);
  Py_XDECREF(sd);
  Py_XDECREF(nm);
  if (Failed(r, "CXNNetExtractBatch")) return nullptr;
  return Take(h, r, oshape, 4, nullptr);
}

const cxx_real_t *CXNNetExtractIter(void *handle, void *data_handle, const char *node_name, cxx_uint oshape[4]) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  Handle *d = static_cast<Handle *>(data_handle);
  PyObject *fn = Attr("_capi_extract_iter");
  PyObject *r = fn ? PyObject_CallFunction(fn, "OOs", h->obj, d->obj, node_name) : nullptr;
  Py_XDECREF(fn);
  if (Failed(r, "CXNNetExtractIter")) return nullptr;
  return Take(h, r, oshape, 4, nullptr);
}

const char *CXNNetEvaluate(void *handle, void *data_handle, const char *data_name) {
  Gil g;
  Handle *h = static_cast<Handle *>(handle);
  Handle *d = static_cast<Handle *>(data_handle);
  PyObject *r = PyObject_CallMethod(h->obj, "evaluate", "Os", d->obj, data_name);
  if (Failed(r, "CXNNetEvaluate")) return "";
  const char *s = PyUnicode_AsUTF8(r);
  h->str = s ? s : "";
  Py_DECREF(r);
  return h->str.c_str();
}

}  // extern "C"
