"""Round-6 GPU tests: the empty-space probe on adversarial volumes (bit identity with the probe and
the empty-sample skip turned off, oracle parity), the probe margin of the fused multi-view launch,
the device stereo entry, and the history-free (occupancy-predicted) block schedule under a camera
that turns every frame (examples/example2.m:53-66)."""
import gc

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("volume_renderer_amd")


@pytest.fixture(autouse=True)
def _clean():
    gc.collect()
    yield
    gc.collect()


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def renderer(vol, res, rot=(125, 25, 0), lights=True):
    """examples/example1.m:32-58 on synthetic data (as tests/test_gpu_parity.py ex1_renderer)."""
    r = vr.VolumeRender()
    if lights:
        r.VolumeIllumination = vr.Volume(vr.HenyeyGreenstein(64))
        r.LightSources = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    r.ElementSizeUm = [1, 1, 1]
    r.FocalLength = 3.0
    r.DistanceToObject = 6
    r.rotate(*rot)
    r.OpacityThreshold = 0.9
    r.ImageResolution = list(res)
    r.VolumeEmission = vol
    r.VolumeAbsorption = vol
    r.FactorAbsorption = 0.6
    r.FactorReflection = 0.4
    r.Color = [1, 1, 0]
    return r


def adversarial_volume(n):
    """Mostly +-0 (a -0 plane included) with isolated non-zero voxels on the faces, edges and corners
    of the occupancy map's 8^3 bricks (padded index i + 1: voxel 7 opens brick 1, voxel 6 closes
    brick 0), a negative voxel, a subnormal one, and voxels at the volume's own corners -- so that
    rays graze single occupied bricks over long empty runs (vr_stage.h probe_run)."""
    v = np.zeros((n, n, n), np.float32, order="F")
    v[:, :, n // 3] = -0.0
    pts = {(7, n // 2, n // 2): 0.9,            # brick face (x)
           (n // 2, 15, n // 2 + 1): 0.8,       # brick face (y)
           (n // 2 - 3, n // 2 + 2, 23): 0.7,   # brick face (z)
           (15, 15, n // 2 - 5): 0.95,          # brick edge
           (23, 23, 23): 1.0, (6, 6, 6): 0.6,   # brick corners (opening / closing)
           (31, 39, 47): 0.85, (39, 31, 7): 0.5,
           (n - 1, n - 1, n - 1): 0.75, (0, 0, 0): 0.65, (0, n - 1, 7): 0.7,  # volume corners / edge
           (n // 2 + 9, 12, n // 2 + 1): -0.7,  # negative
           (n // 2 - 11, n // 2 - 9, n // 2 + 7): 1e-39}  # subnormal
    for (x, y, z), val in pts.items():
        v[x, y, z] = np.float32(val)
    return v


@pytest.mark.parametrize("n", [64, 72])
@pytest.mark.parametrize("rot", [(125, 25, 0), (0, 0, 0), (90, 0, 0), (30, 10, 0)])
def test_probe_is_exact_on_adversarial_volumes(monkeypatch, counter_clock, n, rot):
    """The empty-space probe leaps runs of up to 512 samples after one look at the occupancy map; it
    must never leap a sample that could add anything.  On a volume that is empty but for single
    voxels on brick faces / edges / corners, the default render equals, bit for bit, the render with
    the empty-sample skip off (VR_NO_EMPTY_SKIP=1: every sample shaded, nothing leaped) and the render
    of an upload without an occupancy map (VR_NO_PROBE=1, read at upload), and it is within the oracle
    tolerance.  Axis-aligned cameras make rays run along brick faces."""
    from harness import install
    tee = install(monkeypatch)
    data = adversarial_volume(n)
    r = renderer(vr.Volume(data), res=(192, 160), rot=rot)
    base = r.render()
    assert np.isfinite(base).all() and base.max() > 0
    assert len(tee.renders) == 1  # (oracle parity asserted by the harness)
    monkeypatch.setenv("VR_NO_EMPTY_SKIP", "1")
    noskip = r.render()
    monkeypatch.delenv("VR_NO_EMPTY_SKIP")
    assert np.array_equal(bits(noskip), bits(base))
    monkeypatch.setenv("VR_NO_PROBE", "1")
    fresh = vr.Volume(data.copy(order="F"))  # a new upload: built without a map
    r.VolumeEmission = fresh
    r.VolumeAbsorption = fresh
    noprobe = r.render()
    monkeypatch.delenv("VR_NO_PROBE")
    assert np.array_equal(bits(noprobe), bits(base))
    r.delete()


def test_fused_channels_probe_margin(monkeypatch, counter_clock):
    """the fused multi-view launch (vr_render_channels) probes empty space with the
    probe margin set (vr_capi.hip drift_bound) -- channels of volumes with an occupancy map (>= 64^3,
    sparse) equal their own renders and the renders of uploads without a map, bit for bit, both eyes."""
    n = 72

    def pair(noprobe=False):
        if noprobe:
            monkeypatch.setenv("VR_NO_PROBE", "1")
        a = renderer(vr.Volume(adversarial_volume(n)), res=(120, 90))
        s = O.shell_volume(n)
        s[s < 0.35] = 0.0
        b = renderer(vr.Volume(np.asfortranarray(s)), res=(120, 90))
        b.Color = [0, 1, 0]
        b.FactorEmission = 0.5
        for r in (a, b):
            r.CameraXOffset = 0.5
        return a, b

    sep = [r.render() for r in pair()]
    fused = vr.VolumeRender.renderChannels(list(pair()))
    plain = [r.render() for r in pair(noprobe=True)]
    monkeypatch.delenv("VR_NO_PROBE")
    for a, b, c in zip(sep, fused, plain):
        assert a.max() > 0
        assert np.array_equal(bits(a), bits(b))
        assert np.array_equal(bits(a), bits(c))


def test_stereo_device_entry_matches_host_entry(counter_clock):
    """vr_render_stereo_device writes the images vr_render_stereo returns, bit for
    bit, with and without the sample counters."""
    import torch
    from volume_renderer_amd import mex
    n, W, H = 64, 96, 72
    v = vr.Volume(O.shell_volume(n))
    lut = vr.Volume(vr.HenyeyGreenstein(32))
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), v, vr.Volume(1), v)
    R = np.flip(O.rotation(125, 25, 0), 0).astype(np.float32)
    argv = (lights, lut, np.float32([1, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64([H, W]), R,
            np.float32([0, 3, 6]), np.float32(0.9), np.float32([1, 1, 0]))
    left, right = vr.volumeRender("render_stereo", h, *argv, np.float32(0.3))
    ra, keep = mex.render_args(*argv)
    dl = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
    dr = torch.zeros_like(dl)
    steps = torch.zeros(48, dtype=torch.int64, device="cuda")
    for d_steps in (0, steps.data_ptr()):
        dl.zero_()
        dr.zero_()
        mex.render_stereo_device(h, ra, 0.3, dl.data_ptr(), dr.data_ptr(), d_steps)
        torch.cuda.synchronize()
        for host, dev in ((left, dl), (right, dr)):
            want = np.asarray(host, np.float32).reshape(-1, order="F")
            assert want.max() > 0
            assert np.array_equal(dev.cpu().numpy().view(np.uint32), want.view(np.uint32)), bool(d_steps)
    assert int(steps[0].item()) > 0  # the counted launch counted both eyes' samples
    vr.volumeRender("delete", h)


def test_movie_frames_follow_the_predicted_schedule(monkeypatch, counter_clock):
    """examples/example2.m: the camera turns before every frame, so no frame has a measured schedule
    of its own camera; full frames take the heavy-first order predicted from the occupancy map
    (vr_capi.hip attach_schedule).  Every frame equals the unscheduled render bit for bit, and the
    first frame is within the oracle tolerance."""
    from harness import install
    v = vr.Volume(O.shell_volume(64))
    frames = {}
    for mode in ("predicted", "plain"):
        if mode == "plain":
            monkeypatch.setenv("VR_SCHED", "0")
        else:
            monkeypatch.delenv("VR_SCHED", raising=False)
        r = renderer(v, res=(1280, 1280), rot=(30, 10, 0))
        out = []
        for k in range(6):
            if k:
                r.rotate(0, 12, 0)
            out.append(r.render())
        frames[mode] = out
        r.delete()
    monkeypatch.delenv("VR_SCHED", raising=False)
    for k, (a, b) in enumerate(zip(frames["predicted"], frames["plain"])):
        assert a.max() > 0
        assert np.array_equal(bits(a), bits(b)), k
    tee = install(monkeypatch)
    r = renderer(v, res=(320, 256), rot=(30, 10, 0))
    r.render()
    assert len(tee.renders) == 1
    r.delete()


def test_test_switches_are_off_by_default(monkeypatch, counter_clock):
    """The kernel-variant switches of the environment reach the library only after
    vr_set_option("test_switches", 1): without it VR_DEPTH_LANES=1 does not change the launch."""
    from volume_renderer_amd import mex
    v = vr.Volume(O.shell_volume(64))
    r = renderer(v, res=(96, 80))
    r.render()
    prod = mex.last_march_kernel()
    assert not prod.startswith("vr::fast::march_kernel<1,"), prod
    monkeypatch.setenv("VR_DEPTH_LANES", "1")
    try:
        mex.enable_test_switches(False)
        r.render()
        assert mex.last_march_kernel() == prod
        mex.enable_test_switches(True)
        r.render()
        assert mex.last_march_kernel().startswith("vr::fast::march_kernel<1,")
    finally:
        mex.enable_test_switches(True)
    with pytest.raises(Exception):
        mex.set_option("no_such_option", 1)
    r.delete()


@pytest.mark.parametrize("lanes", ["2", "4"])
def test_preleap_launch_keeps_the_image(monkeypatch, counter_clock, lanes):
    """The pre-leap launch (vr_march.hip preleap_kernel): at rotate(30,10,0) the columns next to the
    silhouette run almost parallel to the x = -1 face, so their tiles' rays start hundreds of samples
    apart and are pre-leaped through the occupancy map before the march.  The frames equal, bit for
    bit, those without the pre-leap (VR_NO_PRELEAP=1) and the unscheduled ones (VR_SCHED=0: no
    schedule, no pre-leap launch), at either depth-lane count."""
    monkeypatch.setenv("VR_DEPTH_LANES", lanes)
    v = vr.Volume(O.shell_volume(128))
    out = {}
    for mode, env in (("default", {}), ("nopre", {"VR_NO_PRELEAP": "1"}), ("plain", {"VR_SCHED": "0"})):
        for k in ("VR_NO_PRELEAP", "VR_SCHED"):
            monkeypatch.delenv(k, raising=False)
        for k, val in env.items():
            monkeypatch.setenv(k, val)
        r = renderer(v, res=(1024, 1024), rot=(30, 10, 0))
        out[mode] = [r.render()]
        r.rotate(0, 12, 0)
        out[mode].append(r.render())
        r.delete()
    for mode in ("nopre", "plain"):
        for a, b in zip(out["default"], out[mode]):
            assert a.max() > 0
            assert np.array_equal(bits(a), bits(b)), mode
