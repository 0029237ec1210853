/*
 * tests/mexstub/mex.h -- TEST-ONLY stand-in for the parts of MATLAB's MEX / matrix API that the
 * adaptors in mex/ use, so that they can be compiled and their mexFunction driven from pytest
 * (tests/test_mex_adaptor.py) in an image without MATLAB.  The mxArray model lives in mexstub.cpp.
 * Not part of the product: a maintainer builds the mex/ adaptors against MATLAB's own mex.h
 * (INTEGRATION.md).
 */
#ifndef VR_TEST_MEXSTUB_MEX_H_
#define VR_TEST_MEXSTUB_MEX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;

typedef enum {
  mxUNKNOWN_CLASS = 0,
  mxCELL_CLASS,
  mxSTRUCT_CLASS,
  mxLOGICAL_CLASS,
  mxCHAR_CLASS,
  mxVOID_CLASS,
  mxDOUBLE_CLASS,
  mxSINGLE_CLASS,
  mxINT8_CLASS,
  mxUINT8_CLASS,
  mxINT16_CLASS,
  mxUINT16_CLASS,
  mxINT32_CLASS,
  mxUINT32_CLASS,
  mxINT64_CLASS,
  mxUINT64_CLASS,
  mxFUNCTION_CLASS,
  mxOBJECT_CLASS
} mxClassID;

typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;

/* mex.h */
void mexErrMsgTxt(const char *msg); /* raises (does not return), as in MATLAB */
void mexWarnMsgTxt(const char *msg);
int mexPrintf(const char *fmt, ...);
void mexLock(void);
void mexUnlock(void);

/* matrix.h */
int mxGetString(const mxArray *a, char *buf, mwSize buflen);
double mxGetScalar(const mxArray *a);
void *mxGetData(const mxArray *a);
double *mxGetPr(const mxArray *a);
size_t mxGetNumberOfElements(const mxArray *a);
mwSize mxGetNumberOfDimensions(const mxArray *a);
const mwSize *mxGetDimensions(const mxArray *a);
size_t mxGetM(const mxArray *a);
size_t mxGetN(const mxArray *a);
mxClassID mxGetClassID(const mxArray *a);
int mxIsComplex(const mxArray *a);
int mxIsSingle(const mxArray *a);
int mxIsCell(const mxArray *a);
int mxIsClass(const mxArray *a, const char *name);
mxArray *mxGetCell(const mxArray *a, mwIndex i);
mxArray *mxGetProperty(const mxArray *obj, mwIndex i, const char *name);
const mxArray *mxGetPropertyShared(const mxArray *obj, mwIndex i, const char *name);
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity c);
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c);
void mxDestroyArray(mxArray *a);

#ifdef __cplusplus
}
#endif

/* the adaptor's entry point */
#ifdef __cplusplus
extern "C"
#endif
void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);

#endif /* VR_TEST_MEXSTUB_MEX_H_ */
