#!/usr/bin/env python3
"""End-to-end timing of the MATLAB-facing host path (SURVEY.md 8d "end-to-end mex-call time",
8f row 3 "upload path"), run on the GPU box:

  * sync_volumes of a host V_shell(n) volume (H2D + apron padding + statistics): upload GB/s;
  * one VolumeRender.render (VolumeRender.m:497-583): 'sync_volumes' with the previous sync time
    (nothing changed) then 'render' through vr_render (the MEX path: LUT/light upload, launch,
    D2H of the [H, W, 3] image), compute gradient;
  * the same with the three lookup-gradient volumes as host Volumes (example1_grad.m), whose
    'sync_volumes' runs setGradientTextures (volumeRender_kernel.cu:703-722);
  * a movie whose Data changes every frame (example3.m:151), serial vs upload overlapped with the
    previous frame's render (movie()).

Each render figure is the median of --reps calls after one warm-up.  Set VR_ALWAYS_REUPLOAD=1 for
the reference's behaviour (LUT and gradients re-uploaded by every render).
usage: python tools/e2e_bench.py [--n 1024 --width 1920 --height 1080 --reps 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-lookup", action="store_true")
    ap.add_argument("--upload-only", action="store_true", help="median 'sync_volumes' time of a changed host volume")
    ap.add_argument("--movie-only", action="store_true", help="only the data-changing movie (movie())")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import volume_renderer_amd as vr
    from volume_renderer_amd import mex
    mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
    from bench import rotation

    n, W, H = args.n, args.width, args.height
    t = torch.empty(n * n * n, dtype=torch.float32, device="cuda")
    mex.synth_shell_device(t.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    host = t.cpu().numpy().reshape((n, n, n), order="F")
    del t
    torch.cuda.synchronize()

    em = vr.Volume(host)
    if args.upload_only:
        h = vr.volumeRender("new")
        refl = vr.Volume(1)
        ts = []
        for _ in range(args.reps + 1):
            em.touch()
            t0 = time.perf_counter()
            vr.volumeRender("sync_volumes", h, np.uint64(1), em, refl, em)
            ts.append(time.perf_counter() - t0)
        vr.volumeRender("delete", h)
        t = float(np.median(ts[1:]))
        print(json.dumps({"volume": n, "chunk_mb": os.environ.get("VR_UPLOAD_CHUNK_MB", "default"),
                          "sync_ms": round(t * 1e3, 2), "GBps": round(host.nbytes / t / 1e9, 2)}), flush=True)
        return
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    refl = vr.Volume(1)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    h = vr.volumeRender("new")
    if args.movie_only:
        R = rotation(125, 25, 0)
        call = ("render", h, lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64([H, W]),
                np.flip(R, 0).astype(np.float32), np.float32([0, 3.0, 6.0]), np.float32(0.9), np.float32([1, 1, 0]))
        vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
        print(json.dumps(movie(args, vr, mex, h, host, refl, lut, lights, call)), flush=True)
        vr.volumeRender("delete", h)
        return
    t0 = time.perf_counter()
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    t_sync = time.perf_counter() - t0
    R = rotation(125, 25, 0)
    call = ("render", h, lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64([H, W]),
            np.flip(R, 0).astype(np.float32), np.float32([0, 3.0, 6.0]), np.float32(0.9), np.float32([1, 1, 0]))

    def med(fn):
        fn()
        ts = []
        for _ in range(args.reps):
            t1 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t1)
        return float(np.median(ts)) * 1e3

    t_last = np.uint64(mex.timestamp())

    def p_render(*grads):
        vr.volumeRender("sync_volumes", h, t_last, em, refl, em, *grads)
        return vr.volumeRender(*call)

    out = {"volume": n, "image": [W, H], "always_reupload": os.environ.get("VR_ALWAYS_REUPLOAD", "0"),
           "sync_s": round(t_sync, 3), "sync_GBps": round(host.nbytes / t_sync / 1e9, 2),
           "p_render_ms": round(med(p_render), 2)}
    # stereo pair (example3.m CameraXOffset 0.06, f = 3 here): the reference's two renders vs the
    # fused launch (vr_render_stereo); each at the widened resolution [H, W + delta]
    from volume_renderer_amd.volume_render import stereo_geometry
    base, delta, _ = stereo_geometry(0.06, 3.0, [W, H])  # delta from ImageResolution(2) = H
    scall = list(call)
    scall[6] = np.uint64([H, W + delta])

    def two_renders():
        for off in (base, -base):
            c = list(scall)
            c[8] = np.float32([off, 3.0, 6.0])
            vr.volumeRender(*c)

    out["stereo_two_renders_ms"] = round(med(two_renders), 2)
    out["stereo_fused_ms"] = round(med(lambda: vr.volumeRender("render_stereo", *scall[1:], np.float32(base))), 2)
    # two channels x stereo (BASELINE C4 shape, examples/example3.m): a structure channel with its
    # own object (colour [0 1 0], Fe 0.5) beside the main one; per channel a fused stereo render
    # vs all four views in one vr_render_channels launch
    em2 = vr.Volume(host)
    h2 = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h2, np.uint64(0), em2, refl, em2)
    t_last2 = np.uint64(mex.timestamp())
    c2 = list(scall)
    c2[1] = h2
    c2[4] = np.float32([0.5, 0.4, 1.0])
    c2[10] = np.float32([0, 1, 0])

    def per_channel():
        vr.volumeRender("sync_volumes", h, t_last, em, refl, em)
        vr.volumeRender("render_stereo", *scall[1:], np.float32(base))
        vr.volumeRender("sync_volumes", h2, t_last2, em2, refl, em2)
        vr.volumeRender("render_stereo", *c2[1:], np.float32(base))

    chans = [(h, t_last, [em, refl, em], scall[2:]), (h2, t_last2, [em2, refl, em2], c2[2:])]
    out["channels2_stereo_per_channel_ms"] = round(med(per_channel), 2)
    out["channels2_stereo_fused_ms"] = round(med(lambda: mex.render_channels(chans, True, np.float32(base))), 2)
    vr.volumeRender("delete", h2)  # resets every handle (cudaDeviceReset): re-sync the main one
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    out.update(movie(args, vr, mex, h, host, refl, lut, lights, call))
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    if not args.no_lookup:
        grads = em.grad() if n <= 256 else _device_grad(host, mex, vr)
        t0 = time.perf_counter()
        vr.volumeRender("sync_volumes", h, t_last, em, refl, em, *grads)
        out["sync_lookup_s"] = round(time.perf_counter() - t0, 3)
        out["p_render_lookup_ms"] = round(med(lambda: p_render(*grads)), 2)
    vr.volumeRender("delete", h)
    print(json.dumps(out), flush=True)


def movie(args, vr, mex, h, host, refl, lut, lights, call, frames=8):
    """A movie whose emission Data changes every frame (examples/example3.m:151 edits
    VolumeEmission.Data inside the frame loop), so every frame re-uploads the whole volume:
      * serial: what VolumeRender.render does per frame -- 'sync_volumes' (the H2D upload) then
        'render' (vr_render: launch, wait, D2H of the image);
      * overlapped: the device API -- frame k's render is issued on a stream (vr_render_device) and
        not waited for; frame k+1's 'sync_volumes' uploads while it runs (the in-flight frame keeps
        its buffer, vr_resources.h), then frame k+1 is issued.  One wait at the end.
    Two host volumes alternate (V_shell and 0.9 V_shell) and each frame re-stamps TimeLastUpdate."""
    vols = [vr.Volume(host), vr.Volume(host * np.float32(0.9))]
    H, W = int(call[6][0]), int(call[6][1])
    ra, keep = mex.render_args(*call[2:])
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(2)]
    stream = torch.cuda.Stream()
    res = {}

    def serial(k):
        v = vols[k % 2]
        v.touch()
        vr.volumeRender("sync_volumes", h, np.uint64(1), v, refl, v)
        return vr.volumeRender(*call)

    sync_ms, issue_ms = [], []

    def overlapped(k):
        v = vols[k % 2]
        v.touch()
        t1 = time.perf_counter()
        vr.volumeRender("sync_volumes", h, np.uint64(1), v, refl, v)
        t2 = time.perf_counter()
        mex.render_device(h, ra, outs[k % 2].data_ptr(), None, 0, stream.cuda_stream)
        sync_ms.append(round((t2 - t1) * 1e3, 1))
        issue_ms.append(round((time.perf_counter() - t2) * 1e3, 2))

    for name, fn in (("serial", serial), ("overlapped", overlapped)):
        fn(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(1, frames + 1):
            fn(k)
        torch.cuda.synchronize()
        res[f"movie_{name}_ms_per_frame"] = round((time.perf_counter() - t0) / frames * 1e3, 2)
    # the same two frames rendered one at a time: the overlapped images must be bit-identical
    got = outs[frames % 2].cpu().numpy()
    ref_prev = serial(frames)
    res["movie_overlapped_bit_identical"] = bool(np.array_equal(
        got.view(np.uint32), np.asarray(ref_prev, np.float32).reshape(-1, order="F").view(np.uint32)))
    res["movie_frames"] = frames
    res["movie_overlapped_sync_ms"] = sync_ms[1:]
    res["movie_overlapped_issue_ms"] = issue_ms[1:]
    res["movie_upload_GB_per_frame"] = round(host.nbytes / 1e9, 3)
    return res


def _device_grad(host, mex, vr):
    """Volume.grad of a large volume via vr_gradient_device, returned as host Volumes."""
    d = torch.from_numpy(host.reshape(-1, order="F")).cuda()
    g = [torch.empty_like(d) for _ in range(3)]
    mex.gradient_device(d.data_ptr(), host.shape, *[x.data_ptr() for x in g], torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [vr.Volume(x.cpu().numpy().reshape(host.shape, order="F")) for x in g]


if __name__ == "__main__":
    main()
