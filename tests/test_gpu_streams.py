"""Renders in flight on several streams while the host changes what the next render reads
(vr_resources.h): per-launch light lists, a changed illumination LUT and a re-uploaded volume must
never reach a launch that was issued before the change.  Every image is compared bit for bit with
the same frame rendered alone (the reference serialises everything, so that is its output)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("volume_renderer_amd")
torch = pytest.importorskip("torch")
from volume_renderer_amd import mex  # noqa: E402

R = np.flip(O.rotation(125, 25, 0), 0).astype(np.float32)


def _stamped(data, t):
    v = vr.Volume(data)
    v.TimeLastUpdate = np.uint64(t)
    return v


def _args(lights, lut, res):
    return (lights, lut, np.float32([1, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64(res), R,
            np.float32([0, 3, 6]), np.float32(0.9), np.float32([1, 1, 0]))


LIGHTS_A = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
LIGHTS_B = [vr.LightSource([-300, 200, 800], [1, 0.2, 0.1])]


def test_light_lists_and_luts_alternating_across_streams():
    """Frames alternating two light lists (2 lights / 1 light) and two LUTs, issued round-robin on
    three streams without waiting: each equals its serial render."""
    em = _stamped(O.shell_volume(96), 11)
    re = _stamped(np.float32(1.0), 12)
    luts = [_stamped(vr.HenyeyGreenstein(32, 0.8), 13), _stamped(vr.HenyeyGreenstein(32, 0.3), 14)]
    res = (384, 512)
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, re, em)
    variants = [(LIGHTS_A, luts[0]), (LIGHTS_B, luts[1]), (LIGHTS_B, luts[0]), (LIGHTS_A, luts[1])]
    serial = [vr.volumeRender("render", h, *_args(l, lut, res)) for l, lut in variants]
    for a in serial:
        assert a.max() > 0
    assert not np.array_equal(serial[0], serial[1])
    streams = [torch.cuda.Stream() for _ in range(3)]
    H, W = res
    outs, keep = [], []
    for k in range(12):
        l, lut = variants[k % 4]
        ra, kp = mex.render_args(*_args(l, lut, res))
        keep.append(kp)
        o = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
        mex.render_device(h, ra, o.data_ptr(), None, 0, streams[k % 3].cuda_stream)
        outs.append(o)
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        want = serial[k % 4].reshape(-1, order="F")
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32)), k
    vr.volumeRender("delete", h)


@pytest.mark.parametrize("device_data", [False, True])
def test_volume_upload_while_previous_frame_renders(device_data):
    """A movie frame whose volume changed: 'sync_volumes' uploads the new data (host array or device
    tensor) while the previous frame's render is still running on another stream; both frames
    equal their serial renders (the in-flight frame keeps its buffer until it completes)."""
    n, res = 160, (600, 800)
    data = [O.shell_volume(n), np.asfortranarray(O.shell_volume(n)[::-1, :, ::-1] * np.float32(0.8))]
    lut = _stamped(vr.HenyeyGreenstein(32), 5)
    re = _stamped(np.float32(1.0), 6)
    H, W = res
    h = vr.volumeRender("new")

    def volume(k):
        if device_data:
            t = torch.from_numpy(data[k % 2].reshape(-1, order="F").copy()).cuda()
            return mex.DeviceVolume(t.data_ptr(), (n, n, n), last_update=100 + k, owner=t)
        return _stamped(data[k % 2], 100 + k)

    serial = []
    for k in range(2):
        v = volume(k)
        vr.volumeRender("sync_volumes", h, np.uint64(1), v, re, v)
        serial.append(vr.volumeRender("render", h, *_args(LIGHTS_A, lut, res)))
    assert not np.array_equal(serial[0], serial[1])
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs, vols = [], []
    for k in range(6):
        v = volume(k)
        vols.append(v)
        vr.volumeRender("sync_volumes", h, np.uint64(1), v, re, v)  # while frame k-1 may still run
        ra, kp = mex.render_args(*_args(LIGHTS_A, lut, res))
        o = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
        mex.render_device(h, ra, o.data_ptr(), None, 0, streams[k % 2].cuda_stream)
        outs.append((o, kp))
    torch.cuda.synchronize()
    for k, (o, _) in enumerate(outs):
        want = serial[k % 2].reshape(-1, order="F")
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32)), k
    vr.volumeRender("delete", h)


def test_overlapping_readers_keep_the_volume_until_the_last_one():
    """Two renders of one volume in flight on two streams, the later-issued one much shorter: when
    it has finished, the earlier (longer) one still reads the buffer, so a re-upload of changed data
    of the same size must not rewrite it in place (every in-flight reader is tracked, not only the
    newest launch's event).  The long frame equals its serial render."""
    n = 256
    data = [O.shell_volume(n), np.asfortranarray(O.shell_volume(n)[::-1, :, :] * np.float32(0.7))]
    lut = _stamped(vr.HenyeyGreenstein(32), 5)
    re = _stamped(np.float32(1.0), 6)
    big, small = (2048, 2048), (16, 16)
    h = vr.volumeRender("new")
    v0 = _stamped(data[0], 100)
    vr.volumeRender("sync_volumes", h, np.uint64(1), v0, re, v0)
    want = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, big)).reshape(-1, order="F")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    H, W = big
    o_big = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    o_small = torch.empty(3 * small[0] * small[1], dtype=torch.float32, device="cuda")
    ra, k1 = mex.render_args(*_args(LIGHTS_A, lut, big))
    rs, k2 = mex.render_args(*_args(LIGHTS_A, lut, small))
    mex.render_device(h, ra, o_big.data_ptr(), None, 0, sa.cuda_stream)
    mex.render_device(h, rs, o_small.data_ptr(), None, 0, sb.cuda_stream)
    sb.synchronize()  # the newest reader is done; the first one is most likely still running
    v1 = _stamped(data[1], 200)
    vr.volumeRender("sync_volumes", h, np.uint64(1), v1, re, v1)  # same size: the in-place candidate
    torch.cuda.synchronize()
    assert np.array_equal(o_big.cpu().numpy().view(np.uint32), want.view(np.uint32))
    vr.volumeRender("delete", h)


def test_lookup_gradient_copy_built_on_another_stream():
    """The interleaved copy of the lookup gradients (vr_capi.hip, TexUnit::gvec) is built by the first
    launch that needs it, on that launch's stream.  A launch on another stream that finds it built
    must wait for it (its ready event): here the building launch's stream is held back by a spin
    kernel, and the second launch is issued right after it on another stream.  Both images equal
    the serial render."""
    n, res = 96, (300, 400)
    H, W = res
    data = O.shell_volume(n)
    em = _stamped(data, 31)
    re = _stamped(np.float32(1.0), 32)
    lut = _stamped(vr.HenyeyGreenstein(32), 33)
    g = vr.Volume(data).grad()
    h = vr.volumeRender("new")

    def sync(t0, order):
        grads = [_stamped(g[j].Data, t0 + i) for i, j in enumerate(order)]
        vr.volumeRender("sync_volumes", h, np.uint64(0), em, re, em, *grads)
        return grads

    keep = sync(40, (1, 0, 2))  # x and y swapped: other normals
    first = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, res))  # builds the copy of these
    keep = sync(50, (0, 1, 2))  # the true gradients: the copy is stale (its memory may be pooled and reused)
    ra, kp = mex.render_args(*_args(LIGHTS_A, lut, res))
    a, b = (torch.cuda.Stream() for _ in range(2))
    oa = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    ob = torch.empty_like(oa)
    with torch.cuda.stream(a):
        torch.cuda._sleep(100_000_000)
    mex.render_device(h, ra, oa.data_ptr(), None, 0, a.cuda_stream)  # rebuilds the copy after the spin
    mex.render_device(h, ra, ob.data_ptr(), None, 0, b.cuda_stream)  # finds it built
    torch.cuda.synchronize()
    ref = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, res))
    assert ref.max() > 0 and not np.array_equal(ref, first)
    want = ref.reshape(-1, order="F").view(np.uint32)
    assert np.array_equal(oa.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(ob.cpu().numpy().view(np.uint32), want)
    del keep, kp
    vr.volumeRender("delete", h)


# ---- HIP errors are reported by the call that met them, or logged (vr_resources.h, vr_hip_errors) --


def _scene():
    em = _stamped(O.shell_volume(64), 41)
    re = _stamped(np.float32(1.0), 42)
    lut = _stamped(vr.HenyeyGreenstein(16), 43)
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, re, em)
    return h, lut, (em, re)


def test_failed_launch_is_reported_by_its_call(monkeypatch):
    """A deliberately invalid launch configuration (VR_INJECT_BAD_LAUNCH: 2048 work-items per
    workgroup, which the runtime rejects before dispatch) fails the 'render' call that issued it with
    VR_ERR_DEVICE and the HIP error's text -- it is neither swallowed nor left for a later call: the
    next render is correct and nothing was consumed into the handled-error log."""
    from volume_renderer_amd import _lib
    h, lut, keep = _scene()
    good = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, (96, 128)))
    assert good.max() > 0
    n0, _ = _lib.hip_errors()
    monkeypatch.setenv("VR_INJECT_BAD_LAUNCH", "1")
    with pytest.raises(_lib.VrError) as ei:
        vr.volumeRender("render", h, *_args(LIGHTS_A, lut, (96, 128)))
    monkeypatch.delenv("VR_INJECT_BAD_LAUNCH")
    assert ei.value.code == 4, ei.value  # VR_ERR_DEVICE
    assert "march kernel launch" in str(ei.value), str(ei.value)
    again = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, (96, 128)))
    assert np.array_equal(again.view(np.uint32), good.view(np.uint32))
    n1, lines = _lib.hip_errors()
    assert n1 == n0, lines
    vr.volumeRender("delete", h)
    del keep


def _hip_runtime():
    """The HIP runtime this process (torch, libvrhip) uses, as a ctypes library."""
    import ctypes
    for line in open("/proc/self/maps"):
        path = line.split()[-1] if len(line.split()) >= 6 else ""
        if "libamdhip64.so" in path:
            return ctypes.CDLL(path)
    pytest.skip("libamdhip64 not mapped")


def test_error_pending_at_entry_is_logged():
    """An error another caller left in the thread's HIP error state (here a hipSetDevice of a device
    that does not exist) is logged by the next libvrhip entry -- 'pending at entry', with the entry's
    name -- and consumed there, so the call itself and the ones after it proceed (it is no device
    fault)."""
    import ctypes
    from volume_renderer_amd import _lib
    h, lut, keep = _scene()
    hip = _hip_runtime()
    n0, _ = _lib.hip_errors()
    assert hip.hipSetDevice(ctypes.c_int(4096)) != 0
    img = vr.volumeRender("render", h, *_args(LIGHTS_A, lut, (96, 128)))
    assert img.max() > 0
    n1, lines = _lib.hip_errors()
    assert n1 == n0 + 1, lines
    assert "pending at entry" in lines[-1] and "vr_render" in lines[-1], lines[-1]
    vr.volumeRender("render", h, *_args(LIGHTS_A, lut, (96, 128)))
    assert _lib.hip_errors()[0] == n1
    vr.volumeRender("delete", h)
    del keep
