#!/usr/bin/env python3
"""tools/stereo_pair_bench.py [OUT.json] -- what the two eyes of a stereo pair can share (SURVEY.md 8f
row 2, DESIGN.md s9 "shared reads"), measured on BASELINE config C4's camera.

The main channel of examples/example3.m (V_shell(1024), one light example3.m:76, LUT 64, thr 0.95,
rotate(90,0,0) then rotate(-15,15,15), f 4.5, dist 6) as an off-axis stereo pair with CameraXOffset
0.06 (VolumeRender.m:278-287: eyes at -+base = 0.03, each 1920 + delta = 1936 x 1080), marched three
ways on one GPU, the images compared bit for bit:
  two     -- the reference's two renders (vr_render_device, camera offset -base, then +base);
  fused   -- both eyes in one launch, each workgroup one eye (vr_render_stereo_device);
  paired  -- both eyes in one launch with paired tiles (VR_STEREO_PAIR=1): each wave marches the
             right eye's columns c.. and the left eye's c + shift.., the shift making the bundles
             meet at the volume's centre, so that one staged box serves both (the converging
             pairing the round-4 verdict asked for).
Per mode: kernel ms (HIP events, median of 9), and -- with a counter build (VR_LIB_PATH to a
`tools/ab_full.sh cnt -DVR_COUNT_K=1` library, VR_COUNT_PROD=1 set here) -- the production-K chunk
counters: staged / leaped / global chunks, staged box volume (staging bytes), the probe's runs.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import volume_renderer_amd as vr  # noqa: E402
from volume_renderer_amd import mex  # noqa: E402
from volume_renderer_amd.volume_render import stereo_geometry  # noqa: E402
import oracle as O  # noqa: E402


def main():
    mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    n, W, H = 1024, 1920, 1080
    f, dist, xoff = 4.5, 6.0, 0.06
    base, delta, res = stereo_geometry(xoff, f, [W, H])
    Wd = W + delta
    R = O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0))
    t = torch.empty(n ** 3, dtype=torch.float32, device="cuda")
    mex.synth_shell_device(t.data_ptr(), n)
    torch.cuda.synchronize()
    em = mex.DeviceVolume(t.data_ptr(), (n, n, n), last_update=20, owner=t)
    refl = vr.Volume(1)
    refl.TimeLastUpdate = np.uint64(5)
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    lut.TimeLastUpdate = np.uint64(7)
    light = [vr.LightSource([-15, 15, 0], [0.5, 0.5, 0.5])]
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    del t

    def args(props):
        return mex.render_args(light, lut, np.float32([1, 1, 1]), np.float32([1, 1, 1]), np.uint64([H, Wd]),
                               np.flip(R, 0).astype(np.float32), np.float32(props), np.float32(0.95),
                               np.float32([1, 1, 1]))

    ra_l, k1 = args([-base, f, dist])
    ra_r, k2 = args([base, f, dist])
    left = torch.zeros(3 * Wd * H, dtype=torch.float32, device="cuda")
    right = torch.zeros_like(left)
    steps = torch.zeros(48, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def run(mode, d_steps=0):
        if mode == "two":
            mex.render_device(h, ra_l, left.data_ptr(), None, d_steps, s)
            mex.render_device(h, ra_r, right.data_ptr(), None, d_steps, s)
        else:
            if mode == "paired":
                os.environ["VR_STEREO_PAIR"] = "1"
            try:
                mex.render_stereo_device(h, ra_l, float(base), left.data_ptr(), right.data_ptr(), d_steps, s)
            finally:
                os.environ.pop("VR_STEREO_PAIR", None)

    res_all = {"config": "C4 main channel: V_shell(1024), %dx%d per eye (delta %d), base %g, f %g, dist %g, "
                         "1 light, LUT 64, thr 0.95" % (Wd, H, delta, base, f, dist)}
    imgs = {}
    counted = os.environ.get("VR_LIB_PATH", "").find("cnt") >= 0
    for mode in ("two", "fused", "paired"):
        for _ in range(3):
            run(mode)
        torch.cuda.synchronize()
        ms = []
        for _ in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(mode)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        kn = mex.last_march_kernel()
        imgs[mode] = (left.cpu().numpy().copy(), right.cpu().numpy().copy())
        r = {"ms_median": round(float(np.median(ms)), 3), "ms": [round(x, 3) for x in ms], "kernel": kn}
        if counted:  # the production-K chunk counters of one launch (both eyes)
            os.environ["VR_COUNT_PROD"] = "1"
            try:
                steps.zero_()
                run(mode, steps.data_ptr())
                torch.cuda.synchronize()
            finally:
                os.environ.pop("VR_COUNT_PROD", None)
            c = [int(v) for v in steps.tolist()]
            r["counters"] = {"kernel": mex.last_march_kernel(), "chunks_staged_leaped_global": c[2:5],
                             "wave_iterations_total_lit": c[5:7], "probe_runs_leaped_failed": [c[7], c[44]],
                             "staged_box_floats": c[45], "staging_bytes": 4 * c[45],
                             "staged_chunks_by_S": c[40:44]}
        res_all[mode] = r
        print(mode, json.dumps(r)[:400], flush=True)
    ref = imgs["two"]
    res_all["bit_identical"] = {m: bool(all(np.array_equal(a.view(np.uint32), b.view(np.uint32))
                                            for a, b in zip(imgs[m], ref))) for m in ("fused", "paired")}
    res_all["paired_over_two"] = round(res_all["paired"]["ms_median"] / res_all["two"]["ms_median"], 4)
    res_all["fused_over_two"] = round(res_all["fused"]["ms_median"] / res_all["two"]["ms_median"], 4)
    print(json.dumps(res_all))
    if out_path:
        with open(out_path, "w") as fh:
            json.dump(res_all, fh, indent=1)
    vr.volumeRender("delete", h)


if __name__ == "__main__":
    main()
