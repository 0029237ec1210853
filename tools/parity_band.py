#!/usr/bin/env python3
"""tools/parity_band.py [--full] OUT.json -- the uncertainty band of "parity" (DESIGN.md s6).

The reference cannot run here, so the oracle restates it under assumptions nothing in this image
can observe: 8-bit filter weights by round-to-nearest-even, which a*b+c sites nvcc
contracts, the texture unit's filter formula, rsqrtf / __expf modelled by correctly rounded
functions, NaN coordinates sampling at 0.  oracle/Makefile builds the fp32 restatement once per
alternative assumption (oracle/variants/, switches in vr_oracle.c).  For each scene this tool
renders every variant and reports how far it lands from the baseline oracle, next to the fp32-vs-
fp64 envelope and -- on a GPU box -- next to the HIP product:

  rel_max   max |variant - oracle| / max(oracle)
  rms_ratio RMS over lit pixel-channels of (variant - oracle), divided by that of (fp64 - fp32)
  differ    fraction of pixel-channels not bit-identical

Scenes: the four golden scenes of tests/golden_cases.py (whole images; CPU), and with --full (GPU
box) the metric frame of BASELINE.json (V_shell(1024), 1920x1080, 2 lights) on tests/
test_full_size.py's stratified pixel sample.  The product row uses the default (fast) kernel."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402

VARIANTS = ["trunc", "axis_fma", "lerp_2mul", "nofma", "rsqrt_cr", "exp2", "nan_prop"]
VARDIR = os.path.join(ROOT, "oracle", "variants")


def stats(img, base, env):
    b = np.asarray(base, np.float64)
    d = np.abs(np.asarray(img, np.float64) - b)
    scale = max(float(np.abs(b).max()), 1e-30)
    lit = np.abs(b) > 1e-3 * scale
    rms_e = float(np.sqrt((env[lit] ** 2).mean())) if lit.any() else 0.0
    rms_d = float(np.sqrt((d[lit] ** 2).mean())) if lit.any() else 0.0
    return dict(rel_max=float(d.max() / scale), rms_ratio=(rms_d / rms_e) if rms_e else 0.0,
                differ=float((np.asarray(img, np.float32).view(np.uint32) != np.asarray(base, np.float32).view(np.uint32)).mean()))


def golden_rows(gpu):
    import golden_cases as G
    rows = {}
    for name in sorted(G.SCENES):
        sc = G.SCENES[name]
        em = sc["em"]()
        S = O.OracleSession()
        h = S.new()
        v = O.OVolume(em, G.STAMP_EM)
        r = O.OVolume(sc["re"]() if sc["re"] else np.ones((1, 1), np.float32), G.STAMP_RE)
        if sc["grads"]:
            S.sync_volumes(h, 0, v, r, v, *(O.OVolume(g, G.STAMP_GRAD) for g in O.matlab_gradient(em)))
        else:
            S.sync_volumes(h, 0, v, r, v)
        lut = O.OVolume(O.hg_lut(sc["lut"]), G.STAMP_LUT) if sc["lut"] else None
        args = G.render_argv(sc, None, None)[2:]
        base, _ = S.render(h, sc["lights"], lut, *args, threads=8)
        f64, _ = S.render(h, sc["lights"], lut, *args, double=True, threads=8)
        env = np.abs(base.astype(np.float64) - f64.astype(np.float64))
        row = {}
        for var in VARIANTS:
            img, _ = S.render(h, sc["lights"], lut, *args, threads=8,
                              lib_path=os.path.join(VARDIR, f"liboracle_{var}.so"))
            row[var] = stats(img, base, env)
        row["fp64"] = stats(f64, base, env)
        if gpu:
            import test_gpu_golden as TG
            row["product"] = stats(TG.product_render(name), base, env)
        rows[name] = row
    return rows


def full_rows():
    import test_full_size as F
    sc = F.ex1_scene(1024, 1920, 1080)
    xs, ys, _ = F.sample_pixels(sc["img"], sc["R"], [0, 3, 6], (1, 1, 1), seed=1)
    S, oh = sc["S"], sc["oh"]
    base, _ = S.render(oh, F.EX1_LIGHTS, sc["olut"], *sc["rargs"], pixels=(xs, ys), threads=F.THREADS)
    f64, _ = S.render(oh, F.EX1_LIGHTS, sc["olut"], *sc["rargs"], pixels=(xs, ys), double=True, threads=F.THREADS)
    env = np.abs(base.astype(np.float64) - f64.astype(np.float64))
    row = {}
    for var in VARIANTS:
        img, _ = S.render(oh, F.EX1_LIGHTS, sc["olut"], *sc["rargs"], pixels=(xs, ys), threads=F.THREADS,
                          lib_path=os.path.join(VARDIR, f"liboracle_{var}.so"))
        row[var] = stats(img, base, env)
        print("metric", var, row[var], flush=True)
    row["fp64"] = stats(f64, base, env)
    row["product"] = stats(np.ascontiguousarray(np.asarray(sc["img"], np.float32)[ys, xs, :]), base, env)
    return {"metric V_shell(1024) 1920x1080 (stratified pixel sample)": row}


def main():
    full = "--full" in sys.argv
    out = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    gpu = False
    try:
        import torch
        gpu = torch.cuda.is_available()
    except Exception:
        pass
    rows = golden_rows(gpu)
    if full:
        rows.update(full_rows())
    with open(out, "w") as f:
        json.dump(rows, f, indent=1)
    for scene, row in rows.items():
        print(scene)
        for k, v in row.items():
            print(f"  {k:10s} rel_max {v['rel_max']:.2e}  rms_ratio {v['rms_ratio']:.3f}  differ {v['differ']:.3f}")


if __name__ == "__main__":
    main()
