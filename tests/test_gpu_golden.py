"""The HIP product against the committed golden images (tests/golden/*.npz, written by
tests/golden/make_golden.py from the oracle in fp32 and fp64).  No oracle code runs here: each scene
of tests/golden_cases.py is replayed through the product's 'new' / 'sync_volumes' / 'render' mex
commands with the product's own HenyeyGreenstein LUT and Volume.grad, and the image must meet the
SURVEY.md 8c tolerance against the fixture's fp32 image and fp64 envelope."""
import os

import numpy as np
import pytest

import golden_cases as G
from conftest import assert_parity

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("volume_renderer_amd")

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _volume(data, stamp):
    v = vr.Volume(data)
    v.TimeLastUpdate = np.uint64(stamp)
    return v


def product_render(name):
    sc = G.SCENES[name]
    em = _volume(sc["em"](), G.STAMP_EM)
    re = _volume(sc["re"]() if sc["re"] else np.ones((1, 1), np.float32), G.STAMP_RE)
    h = vr.volumeRender("new")
    try:
        if sc["grads"]:
            grads = [_volume(g.Data, G.STAMP_GRAD) for g in em.grad()]  # Volume.grad (product mirror)
            vr.volumeRender("sync_volumes", h, np.uint64(0), em, re, em, *grads)
        else:
            vr.volumeRender("sync_volumes", h, np.uint64(0), em, re, em)
        if sc["lights"] is None:
            lights_arg, lut_arg = False, False
        else:
            lights_arg = [vr.LightSource(l[:3], l[3:]) for l in sc["lights"]]
            lut_arg = _volume(vr.HenyeyGreenstein(sc["lut"]), G.STAMP_LUT)
        return vr.volumeRender("render", h, *G.render_argv(sc, lights_arg, lut_arg))
    finally:
        vr.volumeRender("delete", h)


@pytest.mark.parametrize("name", sorted(G.SCENES))
def test_product_matches_golden_fixture(name):
    data = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    img = product_render(name)
    assert img.shape == data["image"].shape
    assert data["image"].max() > 0
    stats = assert_parity(np.asarray(img, np.float32), data["image"], data["image64"], what=name)
    print(name, stats)
