"""The MATLAB boundary as MATLAB calls it: the C++ MEX adaptors of mex/ (volumeRender,
HenyeyGreenstein, timestamp) compiled against the test-only stand-in of MATLAB's API
(tests/mexstub/) and driven through mexFunction with the prhs vectors VolumeRender.m builds
(syncVolumes, VolumeRender.m:188-219; p_render, :556-581).  CPU tests cover argument handling and the
helpers; GPU tests render through mexFunction and compare with the Python path (the same C-ABI
through volume_renderer_amd.mex) bit for bit, and the argument-count forms of 'sync_volumes'
(render.cpp:105-113) against the oracle."""
import numpy as np
import pytest

import mexsim as M
import oracle as O

vr = pytest.importorskip("volume_renderer_amd")


def _stamped(data, t):
    v = vr.Volume(data)
    v.TimeLastUpdate = np.uint64(t)
    return v


# ---- CPU: loading, argument handling, the helper MEX files ------------------------------------

def test_adaptors_load_and_export_mexfunction():
    for name in ("volumeRender", "HenyeyGreenstein", "timestamp"):
        assert hasattr(M.lib(name), "mexFunction")


@pytest.mark.parametrize("args,msg", [
    ((), "no parameter!"),
    ((np.float64(3),), "First input should be a command string less than 64 characters long."),
    (("x" * 70,), "First input should be a command string less than 64 characters long."),
    (("render",), "Second input should be a class instance handle."),
    (("delete", np.uint64(12345)), "Handle not valid."),
    (("render", np.float64(1.0)), "Input must be a real uint64 scalar."),
])
def test_volume_render_argument_errors(args, msg):
    with pytest.raises(M.MexError, match=msg.replace("(", r"\(").replace(")", r"\)").replace(".", r"\.")):
        M.call("volumeRender", 0, *args)


def test_render_with_invalid_handle_and_too_few_arguments():
    with pytest.raises(M.MexError, match="insufficient parameter!"):
        M.call("volumeRender", 1, "render", np.uint64(1), False, False)
    v = vr.Volume(np.ones((2, 2, 2), np.float32))
    with pytest.raises(M.MexError, match="Handle not valid."):
        M.call("volumeRender", 1, "render", np.uint64(1), False, False, np.float32([1, 1, 1]), np.float32([1, 1, 1]),
               np.uint64([4, 4]), np.eye(3, dtype=np.float32), np.float32([0, 3, 6]), np.float32(0.9),
               np.float32([1, 1, 1]))
    with pytest.raises(M.MexError, match="Handle not valid."):
        M.call("volumeRender", 0, "sync_volumes", np.uint64(1), np.uint64(0), v, v, v)


def test_henyey_greenstein_mex_matches_library_and_oracle():
    (lut,) = M.call("HenyeyGreenstein", 1, np.float64(16))
    assert lut.dtype == np.float32 and lut.shape == (16, 16, 16)
    assert np.array_equal(lut.view(np.uint32), vr.HenyeyGreenstein(16).view(np.uint32))
    assert np.array_equal(lut.view(np.uint32), O.hg_lut(16, 0.8).view(np.uint32))
    (lut5,) = M.call("HenyeyGreenstein", 1, np.float64(8), np.float64(-0.5))
    assert np.array_equal(lut5.view(np.uint32), O.hg_lut(8, -0.5).view(np.uint32))
    with pytest.raises(M.MexError, match=r"g must be in interval \[-1,1\]"):
        M.call("HenyeyGreenstein", 1, np.float64(8), np.float64(1.5))


def test_timestamp_mex():
    (t,) = M.call("timestamp", 1)
    assert t.dtype == np.uint64 and t.shape == (1, 1)
    assert abs(int(t[0, 0]) - int(vr.lib().vr_timestamp())) < 10_000
    with pytest.raises(M.MexError, match="No one input argument accepted"):
        M.call("timestamp", 1, np.float64(1))


# ---- GPU: renders through mexFunction ---------------------------------------------------------

EX1 = dict(lights=[vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])],
           factors=np.float32([1, 0.4, 0.6]), es=np.float32([1, 1, 1]), R=np.flip(O.rotation(125, 25, 0), 0),
           props=np.float32([0, 3, 6]), thr=np.float32(0.9), color=np.float32([1, 1, 0]))


def _render_argv(lut, res=(56, 64), lit=True, props=None):
    """p_render's 'render' arguments after the handle (VolumeRender.m:574-578)."""
    return [EX1["lights"] if lit else False, lut if lit else False, EX1["factors"], EX1["es"], np.uint64(res),
            EX1["R"].astype(np.float32), EX1["props"] if props is None else np.float32(props), EX1["thr"],
            EX1["color"]]


@pytest.mark.gpu
@pytest.mark.parametrize("lit", [True, False])
def test_render_through_mexfunction_equals_python_path(counter_clock, lit):
    """new -> sync_volumes (6 arguments) -> render (11 arguments) -> delete through mexFunction, and
    the same calls through the Python binding: bit-identical images; mexLock / mexUnlock balance."""
    em = _stamped(O.shell_volume(40), 11)
    re = _stamped(np.float32(1.0), 12)
    lut = _stamped(vr.HenyeyGreenstein(32), 13)
    locks = M.lock_count("volumeRender")
    (h,) = M.call("volumeRender", 1, "new")
    assert h.dtype == np.uint64 and h.shape == (1, 1)
    assert M.lock_count("volumeRender") == locks + 1
    M.call("volumeRender", 0, "sync_volumes", h, np.uint64(0), em, re, em)
    (img,) = M.call("volumeRender", 1, "render", h, *_render_argv(lut, lit=lit))
    assert img.dtype == np.float32 and img.shape == (56, 64, 3)
    M.call("volumeRender", 0, "mem_info", h)
    assert "Memory Information" in M.printed("volumeRender")
    M.call("volumeRender", 0, "delete", h)
    assert M.lock_count("volumeRender") == locks
    hp = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", hp, np.uint64(0), em, re, em)
    ref = vr.volumeRender("render", hp, *_render_argv(lut, lit=lit))
    vr.volumeRender("delete", hp)
    assert ref.max() > 0
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_sync_volumes_argument_count_forms(counter_clock):
    """render.cpp:105-113 through mexFunction: 9 arguments select the gradient lookup, 7, 8 and 10
    keep the previous gradient volumes (10 also warns), 6 resets them; each render matches the oracle
    driven with the same argument counts, and 14-argument renders (VolumeRender.m:565-572, the
    gradient volumes appended) equal 11-argument ones."""
    from conftest import assert_parity
    data = O.shell_volume(36)
    em = _stamped(data, 21)
    re = _stamped(np.float32(1.0), 22)
    lut = _stamped(vr.HenyeyGreenstein(32), 23)
    gx, gy, gz = (_stamped(g.Data * np.float32(1.5), 24 + i) for i, g in enumerate(em.grad()))
    S = O.OracleSession()
    oh = S.new()
    ov = lambda v: O.OVolume(v.Data, int(v.TimeLastUpdate))  # noqa: E731
    lights = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
    argv = _render_argv(lut)
    (h,) = M.call("volumeRender", 1, "new")
    imgs = {}
    t = 0
    for nrhs in (9, 7, 8, 10, 6, 9, 8):
        extra = [gx, gy, gz, np.float64(1)][:nrhs - 6]
        M.call("volumeRender", 0, "sync_volumes", h, np.uint64(t), em, re, em, *extra)
        assert ("Unexpected arguments ignored" in M.warnings("volumeRender")) == (nrhs > 9)
        S.sync_volumes(oh, t, ov(em), ov(re), ov(em), *([ov(g) for g in (gx, gy, gz)] if nrhs == 9 else []),
                       nrhs=nrhs)
        (img,) = M.call("volumeRender", 1, "render", h, *argv)
        (img14,) = M.call("volumeRender", 1, "render", h, *argv, gx, gy, gz)
        assert np.array_equal(img.view(np.uint32), img14.view(np.uint32))
        rargs = (np.float32(argv[2]), argv[3], argv[4], argv[5], argv[6], argv[7], argv[8])
        ref32, _ = S.render(oh, lights, ov(lut), *rargs)
        ref64, _ = S.render(oh, lights, ov(lut), *rargs, double=True)
        assert_parity(img, ref32, ref64, f"nrhs {nrhs}")
        imgs.setdefault(nrhs, img)
        t = 1000 + len(imgs)  # later syncs: nothing changed since
    bits = lambda x: x.view(np.uint32)  # noqa: E731
    lookup, compute = imgs[9], imgs[6]
    assert not np.array_equal(bits(lookup), bits(compute))  # the 1.5x gradients change the shading
    for n in (7, 8, 10):  # kept gradient volumes: still the lookup image
        assert np.array_equal(bits(imgs[n]), bits(lookup)), n
    M.call("volumeRender", 0, "delete", h)


@pytest.mark.gpu
def test_stereo_and_channels_through_mexfunction(counter_clock):
    """'render_stereo' and 'render_channels' (the adaptor's extensions for VolumeRender.render's
    stereo pair and example3.m's channels) equal the Python path."""
    em = _stamped(O.shell_volume(32), 31)
    em2 = _stamped(O.rand_volume(24) * np.float32(0.3), 32)
    re = _stamped(np.float32(1.0), 33)
    lut = _stamped(vr.HenyeyGreenstein(16), 34)
    (h,) = M.call("volumeRender", 1, "new")
    M.call("volumeRender", 0, "sync_volumes", h, np.uint64(0), em, re, em)
    left, right = M.call("volumeRender", 2, "render_stereo", h, *_render_argv(lut), np.float32(0.25))
    hp = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", hp, np.uint64(0), em, re, em)
    pl, pr = vr.volumeRender("render_stereo", hp, *_render_argv(lut), np.float32(0.25))
    for a, b in ((left, pl), (right, pr)):
        assert a.max() > 0 and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    (h2,) = M.call("volumeRender", 1, "new")
    chans = [[h, np.uint64(0), em, re, em] + _render_argv(lut),
             [h2, np.uint64(0), em2, re, em2] + _render_argv(lut)]
    (pages,) = M.call("volumeRender", 1, "render_channels", chans, np.float64(1), np.float32(0.25))
    assert pages.shape == (56, 64, 3, 4)
    hp2 = vr.volumeRender("new")
    ref = vr.volumeRender("render_channels", [(hp, np.uint64(0), [em, re, em], _render_argv(lut)),
                                              (hp2, np.uint64(0), [em2, re, em2], _render_argv(lut))],
                          True, np.float32(0.25))
    k = 0
    for l, r in ref:
        for img in (l, r):
            assert np.array_equal(np.ascontiguousarray(pages[:, :, :, k]).view(np.uint32),
                                  np.ascontiguousarray(img).view(np.uint32)), k
            k += 1
    for x in (h, h2):
        M.call("volumeRender", 0, "delete", x)
    for x in (hp, hp2):
        vr.volumeRender("delete", x)
