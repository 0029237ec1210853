#!/usr/bin/env python3
"""tools/shade_ablation.py OUT.json NAME=LIB[:ENV=V,...] ... -- parity of shading variants at full size.

Per scene (the BASELINE configs whose parity margin is thinnest: C4's two example3.m channels, C2,
the metric frame) the default library renders the frame, tests/test_full_size.py's stratified
pixel sample is drawn from it and the oracle (fp32 + fp64 envelope) marches those pixels once.
Every variant -- another build of libvrhip (VR_LIB_PATH) and/or environment switches such as
VR_EXACT_SHADE=1 -- renders the same frame in a child process (one library per process), and its
sampled pixels are scored like conftest.assert_parity_full_size: rms_ratio = RMS over lit channels
of (variant - fp32 oracle) / RMS of (fp64 - fp32 oracle), the unfloored SURVEY 8c fraction, the
fraction bit-identical to the fp32 oracle.  Run on the GPU box."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

EX1_LIGHTS = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
EX3_LIGHT = np.array([[-15, 15, 0, 0.5, 0.5, 0.5]], np.float32)


def scene_def(name):
    import oracle as O
    if name.startswith("c4"):
        W0, H = 1920, 1080
        f, dist, xoff = 4.5, 6.0, 0.06
        from volume_renderer_amd.volume_render import stereo_geometry
        base, delta, _ = stereo_geometry(xoff, f, [W0, H])  # delta from ImageResolution(2) = H: 16
        struct = name == "c4_struct"
        return dict(gen="structure" if struct else "shell", n=1024, W=W0 + delta, H=H,
                    R=O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0)), props=[-base, f, dist], thr=0.95,
                    color=[0, 1, 0] if struct else [1, 1, 1], factors=[0.5, 1, 1] if struct else [1, 1, 1],
                    lights=EX3_LIGHT)
    W, H = {"c2": (1024, 768), "metric": (1920, 1080)}[name]
    return dict(gen="shell", n=1024, W=W, H=H, R=O.rotation(125, 25, 0), props=[0, 3, 6], thr=0.9,
                color=[1, 1, 0], factors=[1, 0.4, 0.6], lights=EX1_LIGHTS)


def render(sc):
    """Product render of the scene through the 'render' mex command; returns (img, device tensor)."""
    import volume_renderer_amd as vr
    from volume_renderer_amd import mex
    mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
    import test_full_size as T
    t = T.device_structure(sc["n"]) if sc["gen"] == "structure" else T.device_shell(sc["n"])
    dims = (sc["n"],) * 3
    em = mex.DeviceVolume(t.data_ptr(), dims, last_update=10, owner=t)
    refl = T.stamped(vr.Volume(1), 5)
    lut = T.stamped(vr.Volume(vr.HenyeyGreenstein(64)), 7)
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    rargs = T.argv(sc["R"], [sc["H"], sc["W"]], sc["props"], sc["thr"], sc["color"], sc["factors"])
    img = vr.volumeRender("render", h, T.lights_arg(sc["lights"]), lut, *rargs)
    vr.volumeRender("delete", h)
    return img, t, lut, rargs


def child(scene, pix_file, out_file):
    sc = scene_def(scene)
    img, _, _, _ = render(sc)
    p = np.load(pix_file)
    np.save(out_file, np.ascontiguousarray(np.asarray(img, np.float32)[p["ys"], p["xs"], :]))


def score(got, ref32, ref64):
    g = np.where(np.isnan(got), 0, got).astype(np.float64)
    r = np.where(np.isnan(ref32), 0, ref32).astype(np.float64)
    r64 = np.where(np.isnan(ref64), 0, ref64).astype(np.float64)
    scale = max(float(np.abs(r).max()), 1e-30)
    d, env = np.abs(g - r), np.abs(r - r64)
    lit = np.abs(r) > 1e-3 * scale
    rms_e = float(np.sqrt((env[lit] ** 2).mean()))
    rms_d = float(np.sqrt((d[lit] ** 2).mean()))
    return dict(rms_ratio=rms_d / rms_e if rms_e else 0.0, frac_within_survey=float((d <= 4 * env + 1e-5 * scale).mean()),
                bit_exact=float((np.asarray(got, np.float32).view(np.uint32) == np.asarray(ref32, np.float32).view(np.uint32)).mean()),
                rel_max=float(d.max() / scale), nan_equal=bool(np.array_equal(np.isnan(got), np.isnan(ref32))))


def main():
    if sys.argv[1] == "--child":
        return child(*sys.argv[2:5])
    out_json = sys.argv[1]
    variants = []
    for spec in sys.argv[2:]:
        name, rest = spec.split("=", 1)
        lib, _, envs = rest.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        variants.append((name, lib, env))
    scenes = os.environ.get("ABL_SCENES", "c4_struct,c4_main,c2,metric").split(",")
    import oracle as O
    import test_full_size as T
    res = {}
    tmp = os.path.join(ROOT, "gpurun_out", "abl_tmp")
    os.makedirs(tmp, exist_ok=True)
    for scene in scenes:
        sc = scene_def(scene)
        img, t, lut, rargs = render(sc)
        hem = T.host(t, (sc["n"],) * 3)
        del t
        bmax = (1.0, 1.0, 1.0)
        xs, ys, _ = T.sample_pixels(img, sc["R"], sc["props"], bmax, seed=7)
        pix = os.path.join(tmp, scene + "_pix.npz")
        np.savez(pix, xs=xs, ys=ys)
        S = O.OracleSession(copy=False)
        oh = S.new()
        oem = O.OVolume(hem, 10)
        S.sync_volumes(oh, 0, oem, O.OVolume(np.ones((1, 1), np.float32), 5), oem)
        olut = O.OVolume(lut.Data, 7)
        ref32, _ = S.render(oh, sc["lights"], olut, *rargs, pixels=(xs, ys), threads=16)
        ref64, _ = S.render(oh, sc["lights"], olut, *rargs, pixels=(xs, ys), double=True, threads=16)
        del hem, S, oem
        np.savez(os.path.join(tmp, scene + "_ref.npz"), xs=xs, ys=ys, ref32=ref32, ref64=ref64,
                 prod=np.ascontiguousarray(np.asarray(img, np.float32)[ys, xs, :]))
        res[scene] = {"pixels": int(len(xs))}
        for name, lib, env in variants:
            o = os.path.join(tmp, f"{scene}_{name}.npy")
            e = dict(os.environ)
            e.pop("VR_EXACT_SHADE", None)
            if lib and lib != "default":
                e["VR_LIB_PATH"] = os.path.join(ROOT, lib)
            e.update(env)
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", scene, pix, o], env=e, check=True,
                           timeout=300)
            res[scene][name] = score(np.load(o), ref32, ref64)
            print(scene, name, json.dumps(res[scene][name]), flush=True)
    with open(out_json, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
