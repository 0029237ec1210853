#!/usr/bin/env python3
"""Regenerate the oracle golden fixtures in tests/golden/ (run from the repo root after
`make -C oracle`).  The reference itself cannot be run here, so these pin the
oracle against accidental change and give the GPU test (tests/test_gpu_golden.py) committed
expected images with their fp64 envelope; the HG LUT hash is additionally anchored by the reference
generator's known answers (tests/test_oracle.py)."""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
import golden_cases as G  # noqa: E402

for name, fn in G.CASES.items():
    img, steps = fn()
    img64, _ = G.oracle_render(name, double=True)  # the fp64 envelope render (SURVEY.md 8c tolerance)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), image=img, image64=img64, steps=np.int64(steps))
    print(name, img.shape, steps)
lut = O.hg_lut(64, 0.8).reshape(-1, order="F")
with open(os.path.join(HERE, "hg64_g0.8.sha256"), "w") as f:
    f.write(hashlib.sha256(np.ascontiguousarray(lut).tobytes()).hexdigest() + "  HenyeyGreenstein(64, 0.8) fp32\n")
np.save(os.path.join(HERE, "hg16_g0.8.npy"), O.hg_lut(16, 0.8).reshape(-1, order="F"))
