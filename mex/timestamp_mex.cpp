// timestamp_mex.cpp -- `timestamp()` MEX over vr_timestamp (reference src/C/mex/timestamp.cpp:17-33:
// milliseconds since the epoch, low 32 bits, as uint64).  Build with `-output timestamp`.
#include "mex.h"
#include "vrhip.h"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if (nrhs > 0) mexErrMsgTxt("No one input argument accepted\n\n");
  plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
  *static_cast<uint64_t *>(mxGetData(plhs[0])) = vr_timestamp();
  (void)nlhs, (void)nrhs, (void)prhs;
}
