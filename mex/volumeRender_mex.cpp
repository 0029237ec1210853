// volumeRender_mex.cpp -- the MATLAB-side binding of libvrhip.so: a mexFunction named
// `volumeRender` that keeps the reference's command protocol (src/C/mex/render.cpp:50-278) so that
// VolumeRender.m / Volume.m / LightSource.m run unchanged on MI355X.
//
// Not built in this repository (it needs MATLAB's mex.h / libmx); a maintainer builds it with
//   mex -R2018a -I<repo>/include -L<repo>/volume_renderer_amd -lvrhip volumeRender_mex.cpp \
//       -output volumeRender
// and puts the result where src/make.m put the CUDA mex (src/matlab/VolumeRender/).  See
// INTEGRATION.md.  All marshalling permutations (reversed ElementSizeUm and light positions,
// flip(R) un-flipping, [H W] order) happen inside libvrhip exactly as the reference's mex did them;
// this file only unpacks mxArrays into the C-ABI structs of include/vrhip.h.
#include <string.h>
#include <string>
#include <vector>

#include "mex.h"
#include "vrhip.h"

namespace {

[[noreturn]] void fail(int rc) {
  const char *msg = vr_last_error();
  mexErrMsgTxt((msg && *msg) ? msg : (rc == VR_ERR_HANDLE ? "Handle not valid." : "volumeRender failed"));
  throw 0;  // not reached: mexErrMsgTxt does not return
}

void check(int rc) {
  if (rc != VR_OK) fail(rc);
}

// A MATLAB `Volume` object (Data single, TimeLastUpdate uint64), borrowed for this call.
vr_volume make_volume(const mxArray *obj) {
  const mxArray *data = mxGetPropertyShared(obj, 0, "Data");
  const mxArray *stamp = mxGetPropertyShared(obj, 0, "TimeLastUpdate");
  if (!data || !mxIsSingle(data)) mexErrMsgTxt("Volume.Data must be single.");
  vr_volume v{};
  v.data = static_cast<const float *>(mxGetData(data));
  const mwSize nd = mxGetNumberOfDimensions(data);
  const mwSize *d = mxGetDimensions(data);
  v.dims[0] = d[0];
  v.dims[1] = nd > 1 ? d[1] : 1;
  v.dims[2] = nd > 2 ? d[2] : 1;
  v.last_update = stamp ? (uint64_t)mxGetScalar(stamp) : 0;
  v.location = VR_HOST;
  return v;
}

vr_context *handle(const mxArray *a) {
  if (mxGetNumberOfElements(a) != 1 || mxGetClassID(a) != mxUINT64_CLASS || mxIsComplex(a))
    mexErrMsgTxt("Input must be a real uint64 scalar.");
  return reinterpret_cast<vr_context *>(*static_cast<uint64_t *>(mxGetData(a)));
}

template <typename T>
const T *data_of(const mxArray *a, size_t n, const char *what) {
  if (mxGetNumberOfElements(a) < n) mexErrMsgTxt(what);
  return static_cast<const T *>(mxGetData(a));
}

}  // namespace

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if (nrhs == 0) mexErrMsgTxt("no parameter!");
  char cmd[64];
  if (mxGetString(prhs[0], cmd, sizeof(cmd)))
    mexErrMsgTxt("First input should be a command string less than 64 characters long.");

  if (!strcmp(cmd, "new")) {
    if (nlhs != 1) mexErrMsgTxt("New: One output expected.");
    vr_context *h = nullptr;
    check(vr_new(&h));
    mexLock();  // the module-global device state must outlive `clear functions`
    plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
    *static_cast<uint64_t *>(mxGetData(plhs[0])) = reinterpret_cast<uint64_t>(h);
    return;
  }
  if (nrhs < 2) mexErrMsgTxt("Second input should be a class instance handle.");
  vr_context *h = handle(prhs[1]);

  if (!strcmp(cmd, "delete")) {
    check(vr_delete(h));
    mexUnlock();
    if (nlhs != 0 || nrhs != 2) mexWarnMsgTxt("Delete: Unexpected arguments ignored.");
    return;
  }
  if (!strcmp(cmd, "mem_info")) {
    std::vector<char> buf(1 << 16);
    check(vr_mem_info(h, buf.data(), buf.size()));
    mexPrintf("%s", buf.data());
    return;
  }
  if (!strcmp(cmd, "sync_volumes")) {
    if (nrhs < 6) mexErrMsgTxt("insufficient parameter!");
    const uint64_t t_sync = (uint64_t)mxGetScalar(prhs[2]);
    const vr_volume em = make_volume(prhs[3]), re = make_volume(prhs[4]), ab = make_volume(prhs[5]);
    if (nrhs >= 9) {
      const vr_volume dx = make_volume(prhs[6]), dy = make_volume(prhs[7]), dz = make_volume(prhs[8]);
      check(vr_sync_volumes(h, t_sync, &em, &re, &ab, &dx, &dy, &dz));
    } else {
      check(vr_sync_volumes(h, t_sync, &em, &re, &ab, nullptr, nullptr, nullptr));
    }
    if (nlhs != 0 || nrhs > 9) mexWarnMsgTxt("SyncVolumes: Unexpected arguments ignored.");
    return;
  }
  if (!strcmp(cmd, "render")) {
    if (nlhs > 1) mexErrMsgTxt("Too many output arguments.");
    if (nrhs < 11) mexErrMsgTxt("insufficient parameter!");
    vr_render_args a{};
    std::vector<vr_light> lights;
    vr_volume illum{};
    const bool lit = !(mxIsClass(prhs[2], "logical") || mxIsClass(prhs[3], "logical"));
    if (lit) {
      const size_t n = mxGetN(prhs[2]);
      lights.resize(n);
      for (size_t l = 0; l < n; ++l) {
        const float *pos = static_cast<const float *>(mxGetData(mxGetProperty(prhs[2], l, "Position")));
        const float *col = static_cast<const float *>(mxGetData(mxGetProperty(prhs[2], l, "Color")));
        memcpy(lights[l].position, pos, sizeof(lights[l].position));
        memcpy(lights[l].color, col, sizeof(lights[l].color));
      }
      illum = make_volume(prhs[3]);
      a.lights = lights.data();
      a.num_lights = (int64_t)n;
      a.illumination = &illum;
    } else {
      a.num_lights = -1;  // the logical `false`
      a.illumination = nullptr;
    }
    memcpy(a.factors, data_of<float>(prhs[4], 3, "factors: 3 singles expected"), sizeof(a.factors));
    memcpy(a.element_size_um, data_of<float>(prhs[5], 3, "ElementSizeUm: 3 singles expected"),
           sizeof(a.element_size_um));
    memcpy(a.resolution, data_of<uint64_t>(prhs[6], 2, "resolution: uint64 [H W] expected"), sizeof(a.resolution));
    memcpy(a.rotation_flipped, data_of<float>(prhs[7], 9, "rotation: 3x3 single expected"),
           sizeof(a.rotation_flipped));
    memcpy(a.props, data_of<float>(prhs[8], 3, "properties: 3 singles expected"), sizeof(a.props));
    a.opacity_threshold = (float)mxGetScalar(prhs[9]);
    memcpy(a.color, data_of<float>(prhs[10], 3, "Color: 3 singles expected"), sizeof(a.color));
    const mwSize dim[3] = {(mwSize)a.resolution[0], (mwSize)a.resolution[1], 3};
    mxArray *img = mxCreateNumericArray(3, dim, mxSINGLE_CLASS, mxREAL);
    check(vr_render(h, &a, static_cast<float *>(mxGetData(img))));
    plhs[0] = img;
    return;
  }
  mexErrMsgTxt(("Unknown command: " + std::string(cmd)).c_str());
}
