// volumeRender_mex.cpp -- the MATLAB-side binding of libvrhip.so: a mexFunction named
// `volumeRender` that keeps the reference's command protocol (src/C/mex/render.cpp:50-278) so that
// VolumeRender.m / Volume.m / LightSource.m run unchanged on MI355X.
//
// Built here only against the test stand-in of MATLAB's API (tests/mexstub/: a test-only mex.h and
// mxArray model, driven by tests/test_mex_adaptor.py); a maintainer builds the real MEX with
//   mex -R2018a -I<repo>/include -L<repo>/volume_renderer_amd -lvrhip volumeRender_mex.cpp -output volumeRender
// and puts the result where src/make.m put the CUDA mex (src/matlab/VolumeRender/).  See
// INTEGRATION.md.  All marshalling permutations (reversed ElementSizeUm and light positions,
// flip(R) un-flipping, [H W] order) happen inside libvrhip exactly as the reference's mex did them;
// this file only unpacks mxArrays into the C-ABI structs of include/vrhip.h.
#include <stdlib.h>
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

// The 'render' arguments Lights, Illum, factors, ElementSizeUm, [H W], flip(R), props, thr, Color
// (render.cpp:134-221), p[0] = Lights.  `lights` / `illum` own what a.lights / a.illumination point to.
void unpack_render(const mxArray *const *p, vr_render_args &a, std::vector<vr_light> &lights, vr_volume &illum) {
  a = vr_render_args{};
  const bool lit = !(mxIsClass(p[0], "logical") || mxIsClass(p[1], "logical"));
  if (lit) {
    const size_t n = mxGetN(p[0]);
    lights.resize(n);
    for (size_t l = 0; l < n; ++l) {
      const float *pos = static_cast<const float *>(mxGetData(mxGetProperty(p[0], l, "Position")));
      const float *col = static_cast<const float *>(mxGetData(mxGetProperty(p[0], l, "Color")));
      memcpy(lights[l].position, pos, sizeof(lights[l].position));
      memcpy(lights[l].color, col, sizeof(lights[l].color));
    }
    illum = make_volume(p[1]);
    a.lights = lights.data();
    a.num_lights = (int64_t)n;
    a.illumination = &illum;
  } else {
    a.num_lights = -1;  // the logical `false`
    a.illumination = nullptr;
  }
  memcpy(a.factors, data_of<float>(p[2], 3, "factors: 3 singles expected"), sizeof(a.factors));
  memcpy(a.element_size_um, data_of<float>(p[3], 3, "ElementSizeUm: 3 singles expected"),
         sizeof(a.element_size_um));
  memcpy(a.resolution, data_of<uint64_t>(p[4], 2, "resolution: uint64 [H W] expected"), sizeof(a.resolution));
  memcpy(a.rotation_flipped, data_of<float>(p[5], 9, "rotation: 3x3 single expected"), sizeof(a.rotation_flipped));
  memcpy(a.props, data_of<float>(p[6], 3, "properties: 3 singles expected"), sizeof(a.props));
  a.opacity_threshold = (float)mxGetScalar(p[7]);
  memcpy(a.color, data_of<float>(p[8], 3, "Color: 3 singles expected"), sizeof(a.color));
}

mxArray *new_image(const vr_render_args &a, mwSize views) {
  const mwSize dim[4] = {(mwSize)a.resolution[0], (mwSize)a.resolution[1], 3, views};
  return mxCreateNumericArray(views > 1 ? 4 : 3, dim, mxSINGLE_CLASS, mxREAL);
}

// volumeRender('render_channels', {ch1, ch2, ...}, stereo, base) -> single [H W 3 n*eyes]
// (vr_render_channels; examples/example3.m:61-239 as one call).  A channel is a cell
// {h, TimeLastMemSync, Em, Re, Ab, Lights, Illum, factors, ElementSizeUm, [H W], flip(R), props,
// thr, Color} -- the arguments of its 'sync_volumes' and 'render' -- optionally followed by
// Gx, Gy, Gz (gradient lookup).  Page (i * eyes + e) is channel i's view e; MATLAB adds them.
void render_channels(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if (nlhs > 1) mexErrMsgTxt("Too many output arguments.");
  if (nrhs < 4 || !mxIsCell(prhs[1])) mexErrMsgTxt("render_channels: {channels}, stereo, base expected");
  const mwSize n = mxGetNumberOfElements(prhs[1]);
  if (n == 0) mexErrMsgTxt("render_channels: no channels");
  const int32_t stereo = mxGetScalar(prhs[2]) != 0.0;
  const float base = (float)mxGetScalar(prhs[3]);
  std::vector<vr_volume> vols(6 * n);
  std::vector<vr_render_args> args(n);
  std::vector<std::vector<vr_light>> lights(n);
  std::vector<vr_volume> illum(n);
  std::vector<vr_channel> ch(n);
  for (mwSize i = 0; i < n; ++i) {
    const mxArray *c = mxGetCell(prhs[1], i);
    const mwSize m = c && mxIsCell(c) ? mxGetNumberOfElements(c) : 0;
    if (m != 14 && m != 17) mexErrMsgTxt("render_channels: a channel is a cell of 14 or 17 elements");
    const mxArray *e[17];
    for (mwSize k = 0; k < m; ++k) e[k] = mxGetCell(c, k);
    ch[i].handle = handle(e[0]);
    ch[i].time_last_mem_sync = (uint64_t)mxGetScalar(e[1]);
    for (int k = 0; k < 3; ++k) vols[6 * i + k] = make_volume(e[2 + k]);
    ch[i].emission = &vols[6 * i];
    ch[i].reflection = &vols[6 * i + 1];
    ch[i].absorption = &vols[6 * i + 2];
    if (m == 17) {
      for (int k = 0; k < 3; ++k) vols[6 * i + 3 + k] = make_volume(e[14 + k]);
      ch[i].dx = &vols[6 * i + 3];
      ch[i].dy = &vols[6 * i + 4];
      ch[i].dz = &vols[6 * i + 5];
    }
    unpack_render(e + 5, args[i], lights[i], illum[i]);
    ch[i].args = &args[i];
  }
  mxArray *img = new_image(args[0], n * (stereo ? 2 : 1));
  check(vr_render_channels(ch.data(), (int32_t)n, stereo, base, static_cast<float *>(mxGetData(img))));
  plhs[0] = img;
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
    // VR_DEVICES="0,1,...,7": every render of this handle spans those GPUs (vr_new_multi)
    std::vector<int32_t> devs;
    if (const char *ev = getenv("VR_DEVICES")) {
      for (const char *q = ev; *q;) {
        char *end = nullptr;
        const long d = strtol(q, &end, 10);
        if (end == q) break;
        devs.push_back((int32_t)d);
        q = (*end == ',') ? end + 1 : end;
      }
    }
    check(devs.empty() ? vr_new(&h) : vr_new_multi(devs.data(), (int32_t)devs.size(), &h));
    mexLock();  // the module-global device state must outlive `clear functions`
    plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
    *static_cast<uint64_t *>(mxGetData(plhs[0])) = reinterpret_cast<uint64_t>(h);
    return;
  }
  if (!strcmp(cmd, "render_channels")) {
    render_channels(nlhs, plhs, nrhs, prhs);
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
    if (nrhs == 9) {  // gradient volumes given (render.cpp:105-110)
      const vr_volume dx = make_volume(prhs[6]), dy = make_volume(prhs[7]), dz = make_volume(prhs[8]);
      check(vr_sync_volumes(h, t_sync, &em, &re, &ab, &dx, &dy, &dz));
    } else if (nrhs == 6) {  // gradient volumes reset (render.cpp:111-112)
      check(vr_sync_volumes(h, t_sync, &em, &re, &ab, nullptr, nullptr, nullptr));
    } else {  // 7, 8, > 9: the previous gradient volumes are kept; the extra arguments are not read
      const vr_volume unread{};
      check(vr_sync_volumes(h, t_sync, &em, &re, &ab, &unread, nrhs == 7 ? nullptr : &unread, nullptr));
    }
    if (nlhs != 0 || nrhs > 9) mexWarnMsgTxt("SyncVolumes: Unexpected arguments ignored.");
    return;
  }
  if (!strcmp(cmd, "render") || !strcmp(cmd, "render_stereo")) {
    const bool stereo = cmd[6] != '\0';
    if (nlhs > (stereo ? 2 : 1)) mexErrMsgTxt("Too many output arguments.");
    if (nrhs < (stereo ? 12 : 11)) mexErrMsgTxt("insufficient parameter!");
    vr_render_args a;
    std::vector<vr_light> lights;
    vr_volume illum{};
    unpack_render(prhs + 2, a, lights, illum);
    if (!stereo) {
      mxArray *img = new_image(a, 1);
      check(vr_render(h, &a, static_cast<float *>(mxGetData(img))));
      plhs[0] = img;
      return;
    }
    // volumeRender('render_stereo', h, <render args>, base) -> [left, right] (vr_render_stereo;
    // VolumeRender.m:278-307's two renders at camera offsets -base / +base in one launch)
    mxArray *left = new_image(a, 1), *right = new_image(a, 1);
    check(vr_render_stereo(h, &a, (float)mxGetScalar(prhs[11]), static_cast<float *>(mxGetData(left)),
                           static_cast<float *>(mxGetData(right))));
    plhs[0] = left;
    if (nlhs > 1) plhs[1] = right; else mxDestroyArray(right);
    return;
  }
  mexErrMsgTxt(("Unknown command: " + std::string(cmd)).c_str());
}
