// HenyeyGreenstein_mex.cpp -- `HenyeyGreenstein(N[, g])` MEX over vr_henyey_greenstein (the
// reference's src/C/mex/HenyeyGreenstein.cc:29-96 interface; g defaults to 0.8).  Build like
// volumeRender_mex.cpp with `-output HenyeyGreenstein`.  Returns single(N, N, N).
#include "mex.h"
#include "vrhip.h"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if (nrhs == 0) mexErrMsgTxt("no parameter!");
  if (nlhs > 1) mexErrMsgTxt("Too many output arguments.");
  const uint32_t n = (uint32_t)mxGetScalar(prhs[0]);
  const float g = nrhs == 2 ? (float)mxGetScalar(prhs[1]) : 0.8f;
  if (g > 1 || g < -1) mexErrMsgTxt("g must be in interval [-1,1]");
  const mwSize dim[3] = {n, n, n};
  plhs[0] = mxCreateNumericArray(3, dim, mxSINGLE_CLASS, mxREAL);
  if (vr_henyey_greenstein(n, g, static_cast<float *>(mxGetData(plhs[0]))) != VR_OK) mexErrMsgTxt(vr_last_error());
}
