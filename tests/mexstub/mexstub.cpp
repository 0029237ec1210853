// tests/mexstub/mexstub.cpp -- TEST-ONLY model of MATLAB's mxArray and MEX runtime (see mex.h here),
// linked into each adaptor of mex/ to make libmex_<name>.so, plus a small C API (stub_*) through
// which tests/mexsim.py builds the prhs vector MATLAB would pass and reads plhs back.
//
// Semantics kept from MATLAB where the adaptors depend on them: column-major numeric arrays with
// their class and dimensions; char arrays (mxGetString fails on a non-char or too-short buffer);
// logical scalars; 1 x N object arrays with named properties per element (mxGetProperty /
// mxGetPropertyShared -- the shared form returns the stored value without a copy, the other a deep
// copy the caller may destroy); cell arrays; mexErrMsgTxt unwinds out of mexFunction (here as a C++
// exception caught by stub_call, which reports the message).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mex.h"

struct mxArray_tag {
  mxClassID cls = mxUNKNOWN_CLASS;
  std::vector<mwSize> dims;
  std::vector<unsigned char> data;  // numeric / char (uint16 code units) / logical payload
  std::string class_name;           // objects
  std::vector<std::map<std::string, mxArray *>> props;
  std::vector<mxArray *> cells;
};

namespace {

std::string g_error, g_warnings, g_printed;
int g_locks = 0;

size_t elem_size(mxClassID c) {
  switch (c) {
    case mxLOGICAL_CLASS: case mxINT8_CLASS: case mxUINT8_CLASS: return 1;
    case mxCHAR_CLASS: case mxINT16_CLASS: case mxUINT16_CLASS: return 2;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    default: return 0;
  }
}

size_t numel(const mxArray *a) {
  size_t n = 1;
  for (mwSize d : a->dims) n *= d;
  return a->dims.empty() ? 0 : n;
}

mxArray *deep_copy(const mxArray *a) {
  if (!a) return nullptr;
  mxArray *b = new mxArray_tag(*a);
  for (auto &m : b->props)
    for (auto &kv : m) kv.second = deep_copy(kv.second);
  for (auto &c : b->cells) c = deep_copy(c);
  return b;
}

template <class T>
double as_double(const mxArray *a) {
  T v;
  std::memcpy(&v, a->data.data(), sizeof(T));
  return (double)v;
}

}  // namespace

extern "C" {

// ---- mex.h -------------------------------------------------------------------------------------
void mexErrMsgTxt(const char *msg) { throw std::runtime_error(msg ? msg : ""); }
void mexWarnMsgTxt(const char *msg) { g_warnings += std::string(msg ? msg : "") + "\n"; }
int mexPrintf(const char *fmt, ...) {
  char buf[1 << 16];
  va_list ap;
  va_start(ap, fmt);
  const int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_printed += buf;
  return n;
}
void mexLock(void) { ++g_locks; }
void mexUnlock(void) { --g_locks; }

// ---- matrix.h ----------------------------------------------------------------------------------
int mxGetString(const mxArray *a, char *buf, mwSize buflen) {
  if (!a || a->cls != mxCHAR_CLASS || !buf || buflen == 0) return 1;
  const size_t n = numel(a);
  const uint16_t *u = reinterpret_cast<const uint16_t *>(a->data.data());
  size_t k = 0;
  for (; k < n && k + 1 < buflen; ++k) buf[k] = (char)u[k];
  buf[k] = 0;
  return k < n ? 1 : 0;  // truncated
}

double mxGetScalar(const mxArray *a) {
  if (!a || a->data.empty()) return 0.0;
  switch (a->cls) {
    case mxDOUBLE_CLASS: return as_double<double>(a);
    case mxSINGLE_CLASS: return as_double<float>(a);
    case mxLOGICAL_CLASS: case mxUINT8_CLASS: return as_double<uint8_t>(a);
    case mxINT8_CLASS: return as_double<int8_t>(a);
    case mxINT16_CLASS: return as_double<int16_t>(a);
    case mxUINT16_CLASS: case mxCHAR_CLASS: return as_double<uint16_t>(a);
    case mxINT32_CLASS: return as_double<int32_t>(a);
    case mxUINT32_CLASS: return as_double<uint32_t>(a);
    case mxINT64_CLASS: return as_double<int64_t>(a);
    case mxUINT64_CLASS: return as_double<uint64_t>(a);
    default: return 0.0;
  }
}

void *mxGetData(const mxArray *a) {
  return a && !a->data.empty() ? const_cast<unsigned char *>(a->data.data()) : nullptr;
}
double *mxGetPr(const mxArray *a) { return static_cast<double *>(mxGetData(a)); }
size_t mxGetNumberOfElements(const mxArray *a) { return a ? numel(a) : 0; }
mwSize mxGetNumberOfDimensions(const mxArray *a) { return a ? a->dims.size() : 0; }
const mwSize *mxGetDimensions(const mxArray *a) { return a ? a->dims.data() : nullptr; }
size_t mxGetM(const mxArray *a) { return a && !a->dims.empty() ? a->dims[0] : 0; }
size_t mxGetN(const mxArray *a) {
  if (!a || a->dims.size() < 2) return 0;
  size_t n = 1;
  for (size_t i = 1; i < a->dims.size(); ++i) n *= a->dims[i];
  return n;
}
mxClassID mxGetClassID(const mxArray *a) { return a ? a->cls : mxUNKNOWN_CLASS; }
int mxIsComplex(const mxArray *) { return 0; }
int mxIsSingle(const mxArray *a) { return a && a->cls == mxSINGLE_CLASS; }
int mxIsCell(const mxArray *a) { return a && a->cls == mxCELL_CLASS; }
int mxIsClass(const mxArray *a, const char *name) {
  if (!a || !name) return 0;
  static const std::map<std::string, mxClassID> builtin = {
      {"logical", mxLOGICAL_CLASS}, {"char", mxCHAR_CLASS},     {"double", mxDOUBLE_CLASS},
      {"single", mxSINGLE_CLASS},   {"uint64", mxUINT64_CLASS}, {"cell", mxCELL_CLASS}};
  auto it = builtin.find(name);
  if (it != builtin.end()) return a->cls == it->second;
  return a->cls == mxOBJECT_CLASS && a->class_name == name;
}
mxArray *mxGetCell(const mxArray *a, mwIndex i) {
  return a && a->cls == mxCELL_CLASS && i < a->cells.size() ? a->cells[i] : nullptr;
}
const mxArray *mxGetPropertyShared(const mxArray *obj, mwIndex i, const char *name) {
  if (!obj || obj->cls != mxOBJECT_CLASS || i >= obj->props.size()) return nullptr;
  auto it = obj->props[i].find(name);
  return it == obj->props[i].end() ? nullptr : it->second;
}
mxArray *mxGetProperty(const mxArray *obj, mwIndex i, const char *name) {
  return deep_copy(mxGetPropertyShared(obj, i, name));
}
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity) {
  mxArray *a = new mxArray_tag();
  a->cls = cls;
  a->dims.assign(dims, dims + ndim);
  while (a->dims.size() < 2) a->dims.push_back(1);
  a->data.assign(numel(a) * elem_size(cls), 0);
  return a;
}
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c) {
  const mwSize d[2] = {m, n};
  return mxCreateNumericArray(2, d, cls, c);
}
void mxDestroyArray(mxArray *a) {
  if (!a) return;
  for (auto &m : a->props)
    for (auto &kv : m) mxDestroyArray(kv.second);
  for (mxArray *c : a->cells) mxDestroyArray(c);
  delete a;
}

// ---- the test side -----------------------------------------------------------------------------
mxArray *stub_numeric(int cls, int ndim, const size_t *dims, const void *data) {
  mxArray *a = mxCreateNumericArray((mwSize)ndim, dims, (mxClassID)cls, mxREAL);
  if (data && !a->data.empty()) std::memcpy(a->data.data(), data, a->data.size());
  return a;
}
mxArray *stub_string(const char *s) {
  const size_t n = std::strlen(s), d[2] = {1, n};
  mxArray *a = mxCreateNumericArray(2, d, mxCHAR_CLASS, mxREAL);
  uint16_t *u = reinterpret_cast<uint16_t *>(a->data.data());
  for (size_t k = 0; k < n; ++k) u[k] = (uint16_t)(unsigned char)s[k];
  return a;
}
mxArray *stub_object(const char *class_name, size_t n) {
  mxArray *a = new mxArray_tag();
  a->cls = mxOBJECT_CLASS;
  a->class_name = class_name;
  a->dims = {1, n};
  a->props.resize(n);
  return a;
}
void stub_set_prop(mxArray *obj, size_t i, const char *name, mxArray *v) { obj->props.at(i)[name] = v; }
mxArray *stub_cell(size_t n) {
  mxArray *a = new mxArray_tag();
  a->cls = mxCELL_CLASS;
  a->dims = {1, n};
  a->cells.assign(n, nullptr);
  return a;
}
void stub_set_cell(mxArray *c, size_t i, mxArray *v) { c->cells.at(i) = v; }
int stub_class(const mxArray *a) { return a ? (int)a->cls : -1; }
size_t stub_ndim(const mxArray *a) { return a ? a->dims.size() : 0; }
const size_t *stub_dims(const mxArray *a) { return a ? a->dims.data() : nullptr; }
void *stub_data(const mxArray *a) { return mxGetData(a); }
size_t stub_bytes(const mxArray *a) { return a ? a->data.size() : 0; }
void stub_free(mxArray *a) { mxDestroyArray(a); }
const char *stub_last_error(void) { return g_error.c_str(); }
const char *stub_warnings(void) { return g_warnings.c_str(); }
const char *stub_printed(void) { return g_printed.c_str(); }
int stub_lock_count(void) { return g_locks; }
void stub_clear_log(void) {
  g_error.clear();
  g_warnings.clear();
  g_printed.clear();
}

// mexFunction under MATLAB's calling convention: returns 0, or 1 with stub_last_error() set when
// mexErrMsgTxt was raised (plhs entries the call did not set stay NULL).
int stub_call(int nlhs, mxArray **plhs, int nrhs, const mxArray **prhs) {
  g_error.clear();
  for (int i = 0; i < nlhs; ++i) plhs[i] = nullptr;
  try {
    mexFunction(nlhs, plhs, nrhs, prhs);
  } catch (const std::exception &e) {
    g_error = e.what();
    return 1;
  }
  return 0;
}

}  // extern "C"
