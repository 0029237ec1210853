#!/usr/bin/env python3
"""Predicted vs measured block schedules of full frames (round 6, DESIGN.md s5 "history-free schedule").

Needs a DIAG=1 library (VR_LIB_PATH): per camera of the metric workload (V_shell(n), W x H, the two
example1.m lights, on-the-fly gradient) it times
  rowmajor  -- the unscheduled launch (VR_SCHED=0),
  measured  -- the round-5 schedule: heavy-first by the block durations of an earlier frame of the
               same camera (VR_SCHED_MEASURED=1, after a timed row-major frame),
  predicted -- heavy-first by the occupancy-map prediction (VR_SCHED_PREDICT_ONLY=1),
  default   -- the library's sequence: predicted first render, a timed one, then measured order,
and dumps the measured durations and the predicted costs (tools/sched_dump.py records) for offline
comparison.  Images of the three must be identical (checked, SHA-256).
Usage: VR_LIB_PATH=build_ab/libvrhip_diag.so python tools/sched_predict.py --out gpurun_out/sp
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--volume", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cameras", default="125,25,0;30,10,0;125,37,0;125,61,0;125,85,0;125,145,0;90,0,0")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/sched_predict")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    from bench import rotation
    import volume_renderer_amd as vr
    from volume_renderer_amd import mex
    mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    n, W, H = args.volume, args.width, args.height
    vol = torch.empty(n * n * n, dtype=torch.float32, device=dev)
    mex.synth_shell_device(vol.data_ptr(), n, sptr)
    torch.cuda.synchronize(dev)
    em = mex.DeviceVolume(vol.data_ptr(), (n, n, n), last_update=10, owner=vol)
    refl = vr.Volume(1)
    refl.TimeLastUpdate = np.uint64(5)
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    lut.TimeLastUpdate = np.uint64(7)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    hs = {}

    def handle(mode):  # one handle per mode: each keeps its own schedules (vr_context::sched)
        if mode not in hs:
            hs[mode] = vr.volumeRender("new")
            vr.volumeRender("sync_volumes", hs[mode], np.uint64(0), em, refl, em)
        return hs[mode]

    out = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)

    def timed(ra, reps, mode):
        h = handle(mode)
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            mex.render_device(h, ra, out.data_ptr(), None, 0, sptr)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ts.append(round(e0.elapsed_time(e1), 3))
        return ts, hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()

    def setenv(**kv):
        for k in ("VR_SCHED", "VR_SCHED_MEASURED", "VR_SCHED_DUMP", "VR_SCHED_PRED_DUMP", "VR_SCHED_PREDICT_ONLY"):
            os.environ.pop(k, None)
        os.environ.update({k: str(v) for k, v in kv.items()})

    res = []
    for ci, spec in enumerate(args.cameras.split(";")):
        cam = [float(v) for v in spec.split(",")]
        R = rotation(*cam)
        ra, keep = mex.render_args(lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32([1, 1, 1]),
                                   np.uint64([H, W]), np.flip(R, 0).astype(np.float32), np.float32([0, 3.0, 6.0]),
                                   np.float32(0.9), np.float32([1, 1, 0]))
        rec = {"camera": cam}
        setenv(VR_SCHED=0)
        rec["rowmajor_ms"], s0 = timed(ra, args.reps, "rowmajor")
        # predicted: the first render of this camera (nothing cached) and its repeats
        setenv(VR_SCHED_PRED_DUMP=os.path.join(args.out, f"pred_{ci}.bin"), VR_SCHED_PREDICT_ONLY=1)
        rec["predicted_ms"], s1 = timed(ra, args.reps, "predicted")
        # the default sequence: predicted (first render), timed in that order, then measured order
        setenv()
        rec["default_ms"], s3 = timed(ra, args.reps + 2, "default")
        # measured: a timed row-major frame (durations dumped), then frames in its heavy-first order
        setenv(VR_SCHED_MEASURED=1, VR_SCHED_DUMP=os.path.join(args.out, f"meas_{ci}.bin"))
        rec["measured_first_ms"], _ = timed(ra, 1, "measured")
        rec["measured_ms"], s2 = timed(ra, args.reps + 1, "measured")
        rec["identical"] = s0 == s1 == s2 == s3
        rec["sha256"] = s1
        setenv()
        res.append(rec)
        print(json.dumps(rec), flush=True)
    for h in hs.values():
        vr.volumeRender("delete", h)
        break  # ('delete' resets the module's device state, every handle's: one is enough)
    with open(os.path.join(args.out, "summary.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
