"""Render the kernel-variant scenes of tests/test_gpu_parity.py::test_kernel_variants_are_bit_identical
and save every image to gpurun_out/variants.npz for offline comparison (diagnostic tool)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.append(os.path.join(os.path.dirname(__file__), ".."))
import oracle as O  # noqa: E402  (checker only: builds the synthetic shell volume)
import volume_renderer_amd as vr  # noqa: E402
vr.mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
from test_gpu_parity import ex1_renderer  # noqa: E402

VARIANTS = [("default", {}), ("plain", {"VR_NO_LDS": "1"}), ("noskip", {"VR_NO_EMPTY_SKIP": "1"}),
            ("plain_noskip", {"VR_NO_LDS": "1", "VR_NO_EMPTY_SKIP": "1"}), ("tiles1", {"VR_TILE_MODE": "1"}),
                      ("big", {"VR_FORCE_BIG": "1"}), ("plain_big", {"VR_NO_LDS": "1", "VR_FORCE_BIG": "1"}),
                      ("lut_general", {"VR_NO_SMALL_LUT": "1"}), ("wide", {"VR_WIDE_SLOT": "1"}), ("nogvec", {"VR_NO_GVEC": "1"})]
out = {}
for scene in ("hg2", "lookup", "ea"):
    v = vr.Volume(O.shell_volume(56))
    r = ex1_renderer(v, res=(120, 88), lights=(scene != "ea"))
    if scene == "lookup":
        r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = v.grad()
    for name, env in VARIANTS:
        for k in ("VR_NO_LDS", "VR_NO_EMPTY_SKIP", "VR_TILE_MODE", "VR_FORCE_BIG", "VR_NO_SMALL_LUT", "VR_WIDE_SLOT", "VR_NO_GVEC"):
            os.environ.pop(k, None)
        os.environ.update(env)
        out[f"{scene}_{name}"] = r.render()
    for k in ("VR_NO_LDS", "VR_NO_EMPTY_SKIP", "VR_TILE_MODE", "VR_FORCE_BIG", "VR_NO_SMALL_LUT", "VR_WIDE_SLOT", "VR_NO_GVEC"):
        os.environ.pop(k, None)
    r.delete()
    base = out[f"{scene}_default"]
    for name, _ in VARIANTS:
        img = out[f"{scene}_{name}"]
        bad = img.view(np.uint32) != base.view(np.uint32)
        print(scene, name, "differ:", int(bad.sum()), "max|d|:", float(np.abs(img - base).max()) if bad.any() else 0.0)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/variants.npz", **out)
