"""Golden scenes for the oracle (SURVEY.md 8c item ii): small synthetic volumes and images that
exercise EA-only, HG with 2 lights + on-the-fly gradient, HG with a lookup gradient, and a stereo
(off-axis) camera.  tests/golden/make_golden.py writes their images; test_oracle checks them."""
import numpy as np

import oracle as O

EX1_LIGHTS = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)


def _session(em, re=None, grads=None):
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(em, 5)
    r = O.OVolume(re if re is not None else np.ones((1, 1), np.float32), 3)
    if grads is None:
        S.sync_volumes(h, 0, v, r, v)
    else:
        S.sync_volumes(h, 0, v, r, v, *(O.OVolume(g, 9) for g in grads))
    return S, h


def c1_ea_64():
    S, h = _session(O.shell_volume(64))
    R = np.flip(O.rotation(125, 25, 0), 0)
    return S.render(h, None, None, [1, 0.4, 0.6], [1, 1, 1], [256, 256], R, [0, 3, 6], 0.9, [1, 1, 0], threads=4)


def hg2_compute_32():
    S, h = _session(O.shell_volume(32))
    R = np.flip(O.rotation(125, 25, 0), 0)
    return S.render(h, EX1_LIGHTS, O.OVolume(O.hg_lut(64), 7), [1, 0.4, 0.6], [1, 1, 1], [48, 64], R, [0, 3, 6],
                    0.9, [1, 1, 0], threads=4)


def hg1_lookup_24():
    vol = O.shell_volume(24)
    S, h = _session(vol, grads=O.matlab_gradient(vol))
    R = np.flip(O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0)), 0)
    L = np.array([[-15, 15, 0, 0.5, 0.5, 0.5]], np.float32)
    return S.render(h, L, O.OVolume(O.hg_lut(32), 7), [1, 1, 1], [1, 1, 1], [40, 36], R, [0, 4.5, 6], 0.95,
                    [1, 1, 1], threads=4)


def stereo_right_24():
    S, h = _session(O.shell_volume(24), re=O.rand_volume(8))
    R = np.flip(O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0)), 0)
    L = np.array([[-15, 15, 0, 0.5, 0.5, 0.5]], np.float32)
    return S.render(h, L, O.OVolume(O.hg_lut(32), 7), [0.5, 1, 1], [2, 1, 1], [32, 41], R, [0.03, 4.5, 6],
                    0.95, [0, 1, 0], threads=4)


CASES = {"c1_ea_64": c1_ea_64, "hg2_compute_32": hg2_compute_32, "hg1_lookup_24": hg1_lookup_24,
         "stereo_right_24": stereo_right_24}
