"""Golden scenes for the oracle (SURVEY.md 8c item ii): small synthetic volumes and images that
exercise EA-only, HG with 2 lights + on-the-fly gradient, HG with a lookup gradient, and a stereo
(off-axis) camera.  tests/golden/make_golden.py writes their images (fp32 oracle and the fp64
envelope render); test_oracle checks the oracle against them on the CPU, test_gpu_golden checks the
HIP product against them on the GPU.

Each scene is declared once (SCENES) as the arguments MATLAB would hand the mex: the volumes with
their TimeLastUpdate stamps, then the positional 'render' arguments."""
import numpy as np

import oracle as O

EX1_LIGHTS = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
EX3_LIGHT = np.array([[-15, 15, 0, 0.5, 0.5, 0.5]], np.float32)
EX1_R = O.rotation(125, 25, 0)
EX3_R = O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0))

# name -> scene; stamps: emission 5, reflection 3, gradients 9, LUT 7 (sync with TimeLastMemSync 0)
SCENES = {
    "c1_ea_64": dict(em=lambda: O.shell_volume(64), re=None, grads=False, lights=None, lut=None,
                     factors=[1, 0.4, 0.6], es=[1, 1, 1], res=[256, 256], R=EX1_R, props=[0, 3, 6], thr=0.9,
                     color=[1, 1, 0]),
    "hg2_compute_32": dict(em=lambda: O.shell_volume(32), re=None, grads=False, lights=EX1_LIGHTS, lut=64,
                           factors=[1, 0.4, 0.6], es=[1, 1, 1], res=[48, 64], R=EX1_R, props=[0, 3, 6], thr=0.9,
                           color=[1, 1, 0]),
    "hg1_lookup_24": dict(em=lambda: O.shell_volume(24), re=None, grads=True, lights=EX3_LIGHT, lut=32,
                          factors=[1, 1, 1], es=[1, 1, 1], res=[40, 36], R=EX3_R, props=[0, 4.5, 6], thr=0.95,
                          color=[1, 1, 1]),
    "stereo_right_24": dict(em=lambda: O.shell_volume(24), re=lambda: O.rand_volume(8), grads=False,
                            lights=EX3_LIGHT, lut=32, factors=[0.5, 1, 1], es=[2, 1, 1], res=[32, 41], R=EX3_R,
                            props=[0.03, 4.5, 6], thr=0.95, color=[0, 1, 0]),
}

STAMP_EM, STAMP_RE, STAMP_GRAD, STAMP_LUT = 5, 3, 9, 7


def render_argv(sc, lights_arg, lut_arg):
    """The positional 'render' arguments after the handle (render.cpp:142-240 order)."""
    return (lights_arg, lut_arg, np.float32(sc["factors"]), np.float32(sc["es"]), np.uint64(sc["res"]),
            np.flip(sc["R"], 0).astype(np.float32), np.float32(sc["props"]), np.float32(sc["thr"]),
            np.float32(sc["color"]))


def oracle_render(name, double=False):
    """The scene through the oracle's model of the reference: (image [H,W,3], total samples)."""
    sc = SCENES[name]
    em = sc["em"]()
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(em, STAMP_EM)
    r = O.OVolume(sc["re"]() if sc["re"] else np.ones((1, 1), np.float32), STAMP_RE)
    if sc["grads"]:
        S.sync_volumes(h, 0, v, r, v, *(O.OVolume(g, STAMP_GRAD) for g in O.matlab_gradient(em)))
    else:
        S.sync_volumes(h, 0, v, r, v)
    lut = O.OVolume(O.hg_lut(sc["lut"]), STAMP_LUT) if sc["lut"] else None
    return S.render(h, sc["lights"], lut, *render_argv(sc, None, None)[2:], double=double, threads=4)


def c1_ea_64():
    return oracle_render("c1_ea_64")


def hg2_compute_32():
    return oracle_render("hg2_compute_32")


def hg1_lookup_24():
    return oracle_render("hg1_lookup_24")


def stereo_right_24():
    return oracle_render("stereo_right_24")


CASES = {"c1_ea_64": c1_ea_64, "hg2_compute_32": hg2_compute_32, "hg1_lookup_24": hg1_lookup_24,
         "stereo_right_24": stereo_right_24}
