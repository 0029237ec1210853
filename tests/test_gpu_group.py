"""Multi-device groups inside the library (vr_new_multi; SURVEY.md 8e reached through the unchanged
mex protocol): a group renders column parts on its devices and gathers them to the primary over
xGMI.  The test box has one GPU, so the groups here repeat device 0 -- every step of the group path
runs (replicated bindings, per-device LUT uploads and interleaved gradients, the partitioned
launches on the children's streams, the part gathers and the assembly), with VR_GROUP_REPLICATE=1
the volume replicas are real copies too -- and every image must equal the one-device render bit for
bit, frame after frame, as the camera, the lights and the data change."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("volume_renderer_amd")
torch = pytest.importorskip("torch")
from volume_renderer_amd import mex  # noqa: E402


def _scene(r, v, lit=True):
    if lit:
        r.VolumeIllumination = vr.Volume(vr.HenyeyGreenstein(32))
        r.LightSources = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    r.FocalLength, r.DistanceToObject, r.OpacityThreshold = 3.0, 6, 0.9
    r.rotate(125, 25, 0)
    r.ImageResolution = [150, 97]
    r.VolumeEmission = v
    r.VolumeAbsorption = v
    r.FactorAbsorption, r.FactorReflection = 0.6, 0.4
    r.Color = [1, 1, 0]
    return r


@pytest.mark.parametrize("devices,replicate,peer", [("0,0", "0", "1"), ("0,0,0", "1", "1"),
                                                   ("0,0,0,0,0,0,0,0", "1", "1"), ("0,0,0", "1", "0")])
@pytest.mark.parametrize("grad", ["compute", "lookup"])
def test_group_render_equals_one_device(monkeypatch, counter_clock, devices, replicate, peer, grad):
    """peer "0" (VR_GROUP_PEER=0): the group's children treated as without a peer mapping, so the
    volume replicas and the part gathers go through pinned host memory (the branch a node without
    xGMI peer access takes)."""
    monkeypatch.setenv("VR_GROUP_REPLICATE", replicate)
    monkeypatch.setenv("VR_GROUP_PEER", peer)
    data = [O.shell_volume(48), np.asfortranarray(O.shell_volume(48)[::-1] * np.float32(0.7))]

    def frames(group):
        if group:
            monkeypatch.setenv("VR_DEVICES", devices)
        else:
            monkeypatch.delenv("VR_DEVICES", raising=False)
        r = vr.VolumeRender()
        v = vr.Volume(data[0])
        _scene(r, v)
        if grad == "lookup":
            r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = v.grad()
        out = [r.render()]
        r.rotate(0, 20, 0)                                   # camera change
        out.append(r.render())
        r.LightSources = [vr.LightSource([-200, 100, 900], [0.3, 1, 0.2])]  # lights change
        out.append(r.render())
        r.VolumeEmission.Data = data[1]                      # data change (re-sync, replicas refreshed)
        if grad == "lookup":
            r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = r.VolumeEmission.grad()
        out.append(r.render())
        monkeypatch.delenv("VR_DEVICES", raising=False)
        r.delete()
        return out

    one = frames(False)
    grp = frames(True)
    for k, (a, b) in enumerate(zip(one, grp)):
        assert a.max() > 0
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k


def test_group_render_device_on_a_stream(monkeypatch, counter_clock):
    """vr_render_device on a group handle: the assembled image in device memory on the caller's
    stream, several frames in flight."""
    monkeypatch.setenv("VR_GROUP_REPLICATE", "1")
    n, W, H = 64, 200, 120
    t = torch.empty(n ** 3, dtype=torch.float32, device="cuda")
    mex.synth_shell_device(t.data_ptr(), n)
    torch.cuda.synchronize()
    em = mex.DeviceVolume(t.data_ptr(), (n, n, n), last_update=3, owner=t)
    refl = vr.Volume(1)
    refl.TimeLastUpdate = np.uint64(2)
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    lut.TimeLastUpdate = np.uint64(4)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1])]
    R = np.flip(O.rotation(125, 25, 0), 0).astype(np.float32)
    argv = (lights, lut, np.float32([1, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64([H, W]), R,
            np.float32([0, 3, 6]), np.float32(0.9), np.float32([1, 1, 0]))
    h1 = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h1, np.uint64(0), em, refl, em)
    want = vr.volumeRender("render", h1, *argv).reshape(-1, order="F")
    monkeypatch.setenv("VR_DEVICES", "0,0,0,0")
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)
    ra, keep = mex.render_args(*argv)
    s = torch.cuda.Stream()
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(4)]
    for o in outs:
        mex.render_device(h, ra, o.data_ptr(), None, 0, s.cuda_stream)
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))
    vr.volumeRender("delete", h)
    vr.volumeRender("delete", h1)


def _ex3_channels(monkeypatch, devices, n=48, res=(90, 130)):
    """Two example3.m-style channels (shell, and a second field with its own colour / factors), one
    handle each (a group of `devices` when given)."""
    if devices:
        monkeypatch.setenv("VR_DEVICES", devices)
    else:
        monkeypatch.delenv("VR_DEVICES", raising=False)
    lut = vr.Volume(vr.HenyeyGreenstein(32))
    lut.TimeLastUpdate = np.uint64(7)
    refl = vr.Volume(1)
    refl.TimeLastUpdate = np.uint64(5)
    R = np.flip(O.rotation(-15, 15, 15, R=O.rotation(90, 0, 0)), 0).astype(np.float32)
    light = [vr.LightSource([-15, 15, 0], [0.5, 0.5, 0.5])]
    data = [O.shell_volume(n), np.asfortranarray(O.shell_volume(n)[:, ::-1, :] * np.float32(0.5))]
    chans = []
    for i, (color, fe) in enumerate((([1, 1, 1], 1.0), ([0, 1, 0], 0.5))):
        v = vr.Volume(data[i])
        v.TimeLastUpdate = np.uint64(20 + i)
        h = vr.volumeRender("new")
        argv = (light, lut, np.float32([fe, 1, 1]), np.float32([1, 1, 1]), np.uint64(res), R,
                np.float32([-0.03, 4.5, 6]), np.float32(0.95), np.float32(color))
        chans.append((h, np.uint64(0), [v, refl, v], argv))
    monkeypatch.delenv("VR_DEVICES", raising=False)
    return chans


@pytest.mark.parametrize("devices,peer", [("0,0", "1"), ("0,0,0,0", "1"), ("0,0,0", "0")])
def test_group_fused_stereo_and_channels_equal_one_device(monkeypatch, counter_clock, devices, peer):
    """The fused commands on group handles: a stereo pair (vr_render_stereo) and a C4-style
    two-channel stereo frame (vr_render_channels) rendered on a repeated-device group -- every device
    its column part of every view, parts gathered and assembled per view -- equal one device bit for
    bit, over two frames (the second after a data change of one channel).  peer "0": host-staged
    replicas and part gathers (VR_GROUP_PEER=0)."""
    monkeypatch.setenv("VR_GROUP_REPLICATE", "1")
    monkeypatch.setenv("VR_GROUP_PEER", peer)
    out = {}
    for name, devs in (("one", None), ("group", devices)):
        chans = _ex3_channels(monkeypatch, devs)
        frames = [mex.render_channels(chans, stereo=True, base=np.float32(0.03))]
        v = chans[1][2][0]
        v.Data = np.asfortranarray(v.Data * np.float32(1.5))
        v.TimeLastUpdate = np.uint64(40)
        frames.append(mex.render_channels(chans, stereo=True, base=np.float32(0.03)))
        # the fused stereo pair of channel 0 alone (its handle re-synced)
        h, t, vols, argv = chans[0]
        vr.volumeRender("sync_volumes", h, t, *vols)
        frames.append([vr.volumeRender("render_stereo", h, *argv, np.float32(0.03))])
        out[name] = frames
        for c in chans:
            vr.volumeRender("delete", c[0])
    for f1, f2 in zip(out["one"], out["group"]):
        for pair1, pair2 in zip(f1, f2):
            for a, b in zip(pair1, pair2):
                assert a.max() > 0
                assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_group_mem_info_lists_every_device(monkeypatch, counter_clock):
    """mem_info of a group handle: every device of the group, the replicas of the bound volumes it
    holds and the last launch's kernel time on it (SURVEY.md s5 'Metrics')."""
    import ctypes
    from volume_renderer_amd import _lib
    monkeypatch.setenv("VR_GROUP_REPLICATE", "1")
    monkeypatch.setenv("VR_DEVICES", "0,0,0")
    r = _scene(vr.VolumeRender(), vr.Volume(O.shell_volume(40)))
    monkeypatch.delenv("VR_DEVICES")
    r.render()
    torch.cuda.synchronize()
    buf = ctypes.create_string_buffer(1 << 16)
    _lib.check(_lib.lib().vr_mem_info(mex._handle(r.objectHandle), buf, len(buf)))
    txt = buf.value.decode()
    assert txt.count("(primary)") == 1 and txt.count("(group member)") == 2, txt
    assert txt.count("Emission:") == 3 and "(replica)" in txt, txt
    assert "last launch (ms): n/a" not in txt, txt
    r.delete()


def test_groups_created_and_deleted_in_turn(monkeypatch, counter_clock):
    """Events recorded on a group's streams (replica copies, part renders) outlive the group: the
    buffers that read them stay bound, pooled or retired with the events in their reader lists, and
    later syncs and renders query them (vr_capi.hip idle_streams: group streams are pooled, never
    destroyed).  Groups of 2-4 devices are created, render two frames (data change between) and are
    deleted, in turn with one-device renders that reuse the pool; every image equals the first
    one-device render of its data."""
    monkeypatch.setenv("VR_GROUP_REPLICATE", "1")
    data = [O.shell_volume(40), np.asfortranarray(O.shell_volume(40)[::-1] * np.float32(0.8))]

    def two_frames(devices):
        if devices:
            monkeypatch.setenv("VR_DEVICES", devices)
        else:
            monkeypatch.delenv("VR_DEVICES", raising=False)
        r = _scene(vr.VolumeRender(), vr.Volume(data[0]))
        out = [r.render()]
        r.VolumeEmission.Data = data[1]
        out.append(r.render())
        monkeypatch.delenv("VR_DEVICES", raising=False)
        r.delete()
        return out

    ref = two_frames(None)
    assert ref[0].max() > 0 and ref[1].max() > 0
    for devices in ("0,0", None, "0,0,0,0", "0,0,0", None, "0,0"):
        got = two_frames(devices)
        for k in range(2):
            assert np.array_equal(got[k].view(np.uint32), ref[k].view(np.uint32)), (devices, k)
