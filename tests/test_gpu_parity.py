"""GPU parity: the HIP path (libvrhip via the Python mirror of the MATLAB API) against the CPU
oracle, scenario by scenario, through the harness in tests/harness.py.  Scenarios follow the
reference's examples (examples/example1.m, example1_grad.m, example3.m) and the golden-vector
plan of SURVEY.md 8c (EA-only, HG 1 & 2 lights, lookup gradient, stereo, absorption aliasing,
slot stickiness, several handles, delete semantics, edge cases)."""
import gc

import numpy as np
import pytest

import oracle as O
from conftest import assert_parity

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("volume_renderer_amd")


@pytest.fixture(autouse=True)
def _clean():
    gc.collect()
    yield
    gc.collect()


def ex1_renderer(vol_em, res=(96, 80), lights=True, thr=0.9):
    """examples/example1.m:32-58 set-up on synthetic data."""
    r = vr.VolumeRender()
    if lights:
        r.VolumeIllumination = vr.Volume(vr.HenyeyGreenstein(64))
        r.LightSources = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    r.ElementSizeUm = [1, 1, 1]
    r.FocalLength = 3.0
    r.DistanceToObject = 6
    r.rotate(125, 25, 0)
    r.OpacityThreshold = thr
    r.ImageResolution = list(res)
    r.VolumeEmission = vol_em
    r.VolumeAbsorption = vol_em
    r.FactorAbsorption = 0.6
    r.FactorReflection = 0.4
    r.Color = [1, 1, 0]
    return r


def test_c1_emission_absorption_only(monkeypatch, counter_clock):
    """BASELINE config 1: V_shell(64), 256x256, emission-absorption only."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(64))
    r = ex1_renderer(v, res=(256, 256), lights=False)
    img = r.render()
    assert img.shape == (256, 256, 3)
    assert img.max() > 0
    st = tee.renders[-1][2]
    print("C1 parity", st)
    r.delete()


def test_hg_two_lights_compute_gradient(monkeypatch, counter_clock):
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(48))
    r = ex1_renderer(v, res=(96, 80))
    img = r.render()
    assert np.isfinite(img).all() and img.max() > 0
    print("HG2 parity", tee.renders[-1][2])
    # second image of example1.m: new emission, separate (aliased-away) absorption, new factors
    v2 = vr.Volume(O.shell_volume(48) * np.float32(0.5))
    ab = vr.Volume(O.rand_volume(24))
    r.VolumeEmission = v2
    r.VolumeAbsorption = ab
    r.FactorEmission = 0.1
    r.FactorAbsorption = 0.4
    r.FactorReflection = 0.1
    r.Color = [1, 1, 1]
    r.render()
    r.delete()


@pytest.mark.parametrize("nlights", [1, 3, 4])
@pytest.mark.parametrize("refl", ["voxel", "emission"])
def test_light_counts_and_reflection(monkeypatch, counter_clock, nlights, refl):
    """Odd and even light counts (the march holds the first light pair and the single reflection
    voxel in registers, vr_march.hip VR_LIGHTS_HOIST / VR_REFL_HOIST; the rest come from the light
    list) with the default single-voxel reflection (a value other than 1) or the emission volume as
    the reflection texture: parity with the oracle on every render (harness)."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(40))
    r = ex1_renderer(v, res=(72, 64))
    pos = [[500, 1000, 550], [0, 550, 90], [-300, 200, 700], [90, -400, 20]]
    col = [[0, 1, 1], [1, 0.5, 1], [0.3, 0.9, 0.2], [0.6, 0.6, 0.1]]
    r.LightSources = [vr.LightSource(pos[i], col[i]) for i in range(nlights)]
    r.VolumeReflection = v if refl == "emission" else vr.Volume(np.full((1, 1, 1), 0.7, np.float32))
    img = r.render()
    assert np.isfinite(img).all() and img.max() > 0
    print("lights", nlights, refl, tee.renders[-1][2])
    r.delete()


def test_lookup_gradient_then_compute(monkeypatch, counter_clock):
    """examples/example1_grad.m: precomputed gradient volumes, then resetGradientVolumes."""
    from harness import install
    install(monkeypatch)
    v = vr.Volume(O.shell_volume(40))
    gx, gy, gz = v.grad()
    r = ex1_renderer(v, res=(72, 64))
    r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = gx, gy, gz
    a = r.render()
    r.resetGradientVolumes()
    b = r.render()
    assert not np.array_equal(a, b)
    r.delete()


def test_lookup_gradient_odd_padded_edges(monkeypatch, counter_clock):
    """The bricked lookup-gradient copy (2x2x2 bricks of the padded volume) on a volume
    whose padded edges are all odd (33 x 21 x 15 -> 35 x 23 x 17): the last brick of every axis is
    half padding, and every corner of every cell must still read its voxel -- oracle parity per
    render (harness), as for the cube."""
    from harness import install
    install(monkeypatch)
    v = vr.Volume(np.ascontiguousarray(O.shell_volume(40)[3:36, 9:30, 12:27]))
    assert tuple(v.Data.shape) == (33, 21, 15)
    gx, gy, gz = v.grad()
    r = ex1_renderer(v, res=(72, 64))
    r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = gx, gy, gz
    a = r.render()
    assert np.isfinite(a).all() and a.max() > 0
    r.delete()


def test_large_illumination_lut(monkeypatch, counter_clock):
    """A LUT of more than 2^22 padded voxels (168^3) takes the general 64-bit-offset LUT fetch
    instead of the fp32-offset one; parity against the oracle as for the 64^3 LUT."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(40))
    r = ex1_renderer(v, res=(64, 48))
    r.VolumeIllumination = vr.Volume(vr.HenyeyGreenstein(168))
    img = r.render()
    assert np.isfinite(img).all() and img.max() > 0
    print("large LUT parity", tee.renders[-1][2])
    r.delete()


@pytest.mark.parametrize("shape", [(33, 20, 12), (17, 1, 9), (1, 1, 1), (2, 3, 64)])
def test_gradient_device_matches_matlab_gradient(shape):
    """vr_gradient_device (Volume.grad on the GPU) is bit-identical to MATLAB's single gradient."""
    import torch
    from volume_renderer_amd import mex
    rng = np.random.default_rng(7)
    d = np.asfortranarray(rng.standard_normal(shape).astype(np.float32))
    t = torch.from_numpy(d.reshape(-1, order="F").copy()).cuda()
    g = [torch.full_like(t, np.nan) for _ in range(3)]
    mex.gradient_device(t.data_ptr(), shape, g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr())
    torch.cuda.synchronize()
    for got, ref in zip(g, O.matlab_gradient(d)):
        got = got.cpu().numpy().reshape(shape, order="F")
        assert np.array_equal(got.view(np.uint32), np.asfortranarray(ref).view(np.uint32))


def test_grad_matches_matlab_gradient(counter_clock):
    d = O.rand_volume(12)
    gx, gy, gz = vr.Volume(d).grad()
    ox, oy, oz = O.matlab_gradient(d)
    for g, o in ((gx, ox), (gy, oy), (gz, oz)):
        assert np.array_equal(g.Data, o)


@pytest.mark.parametrize("mode", ["RedCyan", "LeftRightHorizontal"])
def test_stereo(monkeypatch, counter_clock, mode):
    """VolumeRender.render off-axis stereo (VolumeRender.m:277-307), example3.m camera."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(40))
    r = vr.VolumeRender()
    r.VolumeIllumination = vr.Volume(vr.HenyeyGreenstein(32))
    r.LightSources = vr.LightSource([-15, 15, 0], [0.5, 0.5, 0.5])
    r.FocalLength = 4.5
    r.DistanceToObject = 6
    r.OpacityThreshold = 0.95
    r.rotate(90, 0, 0)
    r.rotate(-15, 15, 15)
    r.VolumeAbsorption = v
    r.VolumeEmission = v
    r.ImageResolution = [80, 72]
    r.CameraXOffset = 0.06 * 20  # large offset so that delta > 0 at this small size
    r.StereoOutput = getattr(vr.StereoRenderMode, mode)
    img = r.render()
    assert len(tee.renders) == 2
    delta = int(np.floor(0.6 * 72 / 2 + 0.5))
    right, left = tee.renders[0][0], tee.renders[1][0]
    assert right.shape == (72, 80 + delta, 3)
    if mode == "RedCyan":
        assert img.shape == (72, 80, 3)
        assert np.array_equal(img[:, :, 0], left[:, delta:, 0])
        assert np.array_equal(img[:, :, 1:], right[:, :80, 1:])
    else:
        assert img.shape == (72, 160, 3)
    r.delete()


def test_absorption_volume_is_never_sampled(monkeypatch, counter_clock):
    """d_idxAbsorption stays `emission`; a distinct Absorption volume must not
    change the image."""
    from harness import install
    install(monkeypatch)
    v = vr.Volume(O.shell_volume(32))
    r = ex1_renderer(v, res=(64, 48))
    a = r.render()
    r.VolumeAbsorption = vr.Volume(O.rand_volume(32))
    b = r.render()
    assert np.array_equal(a, b)
    r.delete()


def test_slot_stickiness(monkeypatch, counter_clock):
    """Emission == Reflection makes d_idxReflection `emission`; it stays so after Emission changes
    (kernel.cu:771-774 and no reset), so reflection then samples the NEW emission volume."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(32))
    r = ex1_renderer(v, res=(64, 48))
    r.VolumeReflection = v
    r.VolumeAbsorption = v
    r.VolumeEmission = v
    r.render()
    r.VolumeEmission = vr.Volume(O.shell_volume(32) * np.float32(0.7))
    r.render()
    # a new Reflection volume: every slot index still names the emission texture
    r.VolumeReflection = vr.Volume(O.rand_volume(16))
    r.render()
    assert len(tee.renders) == 3
    r.delete()


@pytest.mark.parametrize("zero_front", [False, True])
def test_emission_through_reflection_slot(monkeypatch, counter_clock, zero_front):
    """Emission == Absorption with only Reflection re-stamped takes the simEmAb branch of the
    volume sync (volumeRender_kernel.cu:853-856): d_idxEmmission becomes the reflection texture
    and the emission texture is unbound.  A second handle then binds its own emission texture
    (module-global), so its render samples emission from ITS reflection volume and absorption
    (d_idxAbsorption = emission) from its emission volume: two distinct bound textures.  Without
    lights the staged march runs; the reflection volume is zero on half of the box where the
    absorption is not, so the march must not leap chunks that are empty in the emission texture
    alone (the opacity accumulated there dims what lies behind)."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(32))
    r1 = ex1_renderer(v, res=(64, 48), lights=False)
    r1.VolumeAbsorption = v
    r1.VolumeReflection = vr.Volume(O.rand_volume(16))
    r1.render()
    r1.VolumeReflection = vr.Volume(O.rand_volume(16))
    r1.render()
    half = O.shell_volume(40).copy(order="F")
    if zero_front:
        half[:, :, :20] = 0
    else:
        half[:, :, 20:] = 0
    r2 = ex1_renderer(vr.Volume(O.shell_volume(40)), res=(64, 48), lights=False)
    r2.VolumeAbsorption = vr.Volume(O.rand_volume(12))
    r2.VolumeReflection = vr.Volume(half)
    img = r2.render()
    assert img.any() and len(tee.renders) == 3
    r2.delete()
    r1.delete()


def test_two_handles_share_module_state(monkeypatch, counter_clock):
    from harness import install
    install(monkeypatch)
    v1 = vr.Volume(O.shell_volume(32))
    v2 = vr.Volume(O.rand_volume(20))
    r1 = ex1_renderer(v1, res=(48, 40))
    r2 = ex1_renderer(v2, res=(40, 48), lights=False)
    r1.render()
    r2.render()
    r1.render()  # nothing changed for r1: textures are still bound to r2's volumes
    r2.delete()  # cudaDeviceReset: everything unbound
    img = r1.render()
    assert not img.any()
    r1.delete()


@pytest.mark.parametrize("case", ["inside", "miss", "tiny", "aniso", "flat2d", "onevoxel", "nan"])
def test_edge_cases(monkeypatch, counter_clock, case):
    from harness import install
    install(monkeypatch)
    data = O.shell_volume(24)
    res = (40, 30)
    r = None
    if case == "inside":      # camera inside the box: tnear < 0 -> 0
        r = ex1_renderer(vr.Volume(data), res=res)
        r.DistanceToObject = 0.2
    elif case == "miss":      # most rays miss the box
        r = ex1_renderer(vr.Volume(data), res=res)
        r.FocalLength = 0.2
        r.DistanceToObject = 40
    elif case == "tiny":      # 1x1 image
        r = ex1_renderer(vr.Volume(data), res=(1, 1))
    elif case == "aniso":     # non-cubic volume, anisotropic voxels
        r = ex1_renderer(vr.Volume(O.rand_volume(20)[:, :14, :9].copy(order="F")), res=res)
        r.ElementSizeUm = [0.5, 1.0, 2.5]
    elif case == "flat2d":    # 2-D emission volume (depth 1)
        r = ex1_renderer(vr.Volume(O.rand_volume(16)[:, :, 0].copy(order="F")), res=res)
    elif case == "onevoxel":
        r = ex1_renderer(vr.Volume(np.float32(0.5)), res=res)
    elif case == "nan":       # NaN voxels propagate identically
        d = data.copy(order="F")
        d[10:12, 10:12, 10:12] = np.nan
        r = ex1_renderer(vr.Volume(d), res=res, lights=False)
    r.render()
    r.delete()


def test_empty_image(counter_clock):
    r = ex1_renderer(vr.Volume(O.shell_volume(16)), res=(0, 8), lights=False)
    img = r.render()
    assert img.shape == (8, 0, 3)
    r.delete()


def test_device_partitions_assemble_to_full_image(counter_clock):
    """Image-space partition: parts rendered separately and assembled on the
    device are bit-identical to the single full render; step counts add up."""
    import torch
    from volume_renderer_amd import mex
    v = vr.Volume(O.shell_volume(40))
    r = ex1_renderer(v, res=(123, 77))
    full = r.render()
    args = ("render", r.objectHandle, r.LightSources, r.VolumeIllumination,
            np.float32([r.FactorEmission, r.FactorReflection, r.FactorAbsorption]), np.float32(r.ElementSizeUm),
            np.uint64([77, 123]), np.flip(r.RotationMatrix, 0).astype(np.float32),
            np.float32([0, r.FocalLength, r.DistanceToObject]), np.float32(r.OpacityThreshold), np.float32(r.Color))
    ra, keep = mex.render_args(*args[2:])
    W, H = 123, 77
    for nparts, bc in ((1, 123), (2, 16), (3, 7), (8, 5)):
        maxc = max(mex.partition_columns(W, mex.partition(bc, p, nparts)) for p in range(nparts))
        parts = torch.zeros((nparts, 3, maxc, H), dtype=torch.float32, device="cuda")
        steps = torch.zeros((nparts, 5), dtype=torch.int64, device="cuda")
        for p in range(nparts):
            mex.render_device(r.objectHandle, ra, parts[p].data_ptr(), mex.partition(bc, p, nparts),
                              steps[p].data_ptr())
        out = torch.zeros((3, W, H), dtype=torch.float32, device="cuda")
        mex.assemble_partitions(parts.data_ptr(), W, H, bc, nparts, maxc, out.data_ptr())
        torch.cuda.synchronize()
        img = out.cpu().numpy().reshape(-1)
        assert np.array_equal(img.view(np.uint32), full.reshape(-1, order="F").view(np.uint32)), (nparts, bc)
    r.delete()


def test_step_count_matches_oracle(counter_clock):
    import torch
    from volume_renderer_amd import mex
    v = vr.Volume(O.shell_volume(64))
    r = ex1_renderer(v, res=(256, 256), lights=False)
    r.render()
    ra, keep = mex.render_args(False, False, np.float32([1, 0.4, 0.6]), np.float32([1, 1, 1]), np.uint64([256, 256]),
                               np.flip(r.RotationMatrix, 0).astype(np.float32), np.float32([0, 3, 6]),
                               np.float32(0.9), np.float32([1, 1, 0]))
    out = torch.zeros(256 * 256 * 3, dtype=torch.float32, device="cuda")
    steps = torch.zeros(48, dtype=torch.int64, device="cuda")
    mex.render_device(r.objectHandle, ra, out.data_ptr(), None, steps.data_ptr())
    torch.cuda.synchronize()
    S = O.OracleSession()
    h = S.new()
    ov = O.OVolume(v.Data, 1)
    S.sync_volumes(h, 0, ov, O.OVolume(np.ones((1, 1), np.float32), 1), ov)
    _, total = S.render(h, None, None, [1, 0.4, 0.6], [1, 1, 1], [256, 256], np.flip(r.RotationMatrix, 0),
                        [0, 3, 6], 0.9, [1, 1, 0])
    assert abs(int(steps[0].item()) - total) <= total * 1e-4, (int(steps[0].item()), total)
    r.delete()


@pytest.mark.parametrize("edge", [56, 64])
@pytest.mark.parametrize("shade", ["fast", "exact"])
@pytest.mark.parametrize("scene", ["hg2", "lookup", "ea"])
def test_kernel_variants_are_bit_identical(monkeypatch, counter_clock, scene, shade, edge):
    """The LDS-staged march, the plain kernel, the empty-sample skip / empty-chunk leap and the
    XCD tile order, the longest-first workgroup schedule (every repeated frame shape after the first
    launch) and the depth lanes (K lanes per ray compositing K consecutive samples) change
    only where data comes from, which exact no-ops are elided and which lane computes a sample:
    the images must agree bit for bit, with either shading arithmetic.  The image
    size is ragged for every tile shape.  Edge 64 (a power-of-two cube) takes the fast variant's
    half-texel gradient taps in every kernel."""
    if shade == "exact":
        monkeypatch.setenv("VR_EXACT_SHADE", "1")
    else:
        monkeypatch.delenv("VR_EXACT_SHADE", raising=False)
    v = vr.Volume(O.shell_volume(edge))
    r = ex1_renderer(v, res=(121, 87), lights=(scene != "ea"))
    if scene == "lookup":
        r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = v.grad()
    imgs = {}
    keys = ("VR_NO_LDS", "VR_NO_EMPTY_SKIP", "VR_TILE_MODE", "VR_FORCE_BIG", "VR_NO_SMALL_LUT", "VR_WIDE_SLOT",
            "VR_NO_GVEC", "VR_DEPTH_LANES", "VR_SCHED", "VR_XCD_RUN", "VR_BLOCK_ROT_ROWS")
    for name, env in [("default", {}), ("plain", {"VR_NO_LDS": "1"}), ("noskip", {"VR_NO_EMPTY_SKIP": "1"}),
                      ("plain_noskip", {"VR_NO_LDS": "1", "VR_NO_EMPTY_SKIP": "1"}), ("tiles1", {"VR_TILE_MODE": "1"}),
                      ("big", {"VR_FORCE_BIG": "1"}), ("plain_big", {"VR_NO_LDS": "1", "VR_FORCE_BIG": "1"}),
                      ("lut_general", {"VR_NO_SMALL_LUT": "1"}), ("wide", {"VR_WIDE_SLOT": "1"}), ("narrow", {"VR_WIDE_SLOT": "0"}),
                      ("nogvec", {"VR_NO_GVEC": "1"}),
                      ("k1", {"VR_DEPTH_LANES": "1"}), ("k2", {"VR_DEPTH_LANES": "2"}), ("k4", {"VR_DEPTH_LANES": "4"}),
                      ("k8", {"VR_DEPTH_LANES": "8"}), ("k2_noskip", {"VR_DEPTH_LANES": "2", "VR_NO_EMPTY_SKIP": "1"}),
                      ("k8_wide", {"VR_DEPTH_LANES": "8", "VR_WIDE_SLOT": "1"}),
                      ("k4_big", {"VR_DEPTH_LANES": "4", "VR_FORCE_BIG": "1"}),
                      ("nosched", {"VR_SCHED": "0"}), ("k2_sched", {"VR_DEPTH_LANES": "2", "VR_SCHED": "1"}),
                      ("k1_sched", {"VR_DEPTH_LANES": "1", "VR_SCHED": "1"}),
                      ("xcd_run2", {"VR_XCD_RUN": "2"}), ("k4_xcd_run4", {"VR_DEPTH_LANES": "4", "VR_XCD_RUN": "4"}),
                      ("rot3", {"VR_BLOCK_ROT_ROWS": "3"}), ("k4_rot2", {"VR_DEPTH_LANES": "4", "VR_BLOCK_ROT_ROWS": "2"}),
                      ("k1_nogvec", {"VR_DEPTH_LANES": "1", "VR_NO_GVEC": "1"})]:
        for k in keys:
            monkeypatch.delenv(k, raising=False)
        for k, val in env.items():
            monkeypatch.setenv(k, val)
        if env.get("VR_DEPTH_LANES") == "8" and vr.mex.depth_lanes(64, 64) != 8:
            continue  # K = 8 is built only in a diagnostic build (make DIAG=1)
        imgs[name] = r.render()
    base = imgs["default"]
    assert base.max() > 0
    for name, img in imgs.items():
        assert np.array_equal(img.view(np.uint32), base.view(np.uint32)), name
    r.delete()


@pytest.mark.parametrize("edge", [64, 128])
def test_half_texel_taps(monkeypatch, counter_clock, edge):
    """Fast variant on a power-of-two cube (vr_capi.hip half_texel_taps): the on-the-fly gradient
    taps derived from the centre's axes equal the reference's pos +- gstep taps except near the
    planes where a coordinate changes binade.  Both renders are within the oracle tolerance, and
    they differ in at most a few pixel-channels, by little."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(edge))
    r = ex1_renderer(v, res=(160, 128))
    monkeypatch.setenv("VR_EXACT_TAPS", "1")
    exact = r.render()
    monkeypatch.delenv("VR_EXACT_TAPS")
    fast = r.render()
    assert len(tee.renders) == 2
    differ = float((fast.view(np.uint32) != exact.view(np.uint32)).mean())
    print("half-texel taps: pixel-channels differing", differ, "max", float(np.abs(fast - exact).max()),
          "of", float(exact.max()))
    assert differ < 2e-3
    assert np.abs(fast - exact).max() <= 1e-3 * exact.max()
    r.delete()


@pytest.mark.parametrize("scene", ["hg2", "lookup"])
def test_exact_shading_matches_oracle(monkeypatch, counter_clock, scene):
    """VR_EXACT_SHADE=1: the oracle's op sequence (correctly rounded roots and quotients, expf);
    only acosf comes from a different library, so most pixel-channels are bit-identical and the
    rest within the tolerance.  The default (fast) shading must also be within the tolerance of
    the same oracle render and close to the exact one."""
    from harness import install
    tee = install(monkeypatch)
    v = vr.Volume(O.shell_volume(48))
    r = ex1_renderer(v, res=(96, 72))
    if scene == "lookup":
        r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = v.grad()
    monkeypatch.setenv("VR_EXACT_SHADE", "1")
    exact = r.render()
    monkeypatch.delenv("VR_EXACT_SHADE")
    fast = r.render()
    assert len(tee.renders) == 2
    assert tee.renders[0][2]["bit_exact"] > 0.5, tee.renders[0][2]
    assert np.abs(fast - exact).max() <= 1e-2 * exact.max()
    r.delete()


def test_unchanged_lut_and_gradients_stay_resident(monkeypatch, counter_clock):
    """Upload path: the LUT and the lookup-gradient volumes are uploaded again
    only when the Volume changed (data pointer, TimeLastUpdate, size -- the reference's own dedup
    identity), not on every render as setIlluminationTexture / setGradientTextures do
    (volumeRender_kernel.cu:682-722).  White-box check: an in-place edit that bypasses
    TimeLastUpdate (impossible in MATLAB, whose arrays are copy-on-write) is not picked up, a
    touch() or VR_ALWAYS_REUPLOAD=1 (the reference's behaviour) is."""
    monkeypatch.delenv("VR_ALWAYS_REUPLOAD", raising=False)
    v = vr.Volume(O.shell_volume(40))
    gx, gy, gz = v.grad()
    r = ex1_renderer(v, res=(72, 64))
    r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ = gx, gy, gz
    a = r.render()
    gx.Data[...] *= -3.0          # in place, TimeLastUpdate unchanged
    r.VolumeIllumination.Data[...] *= 0.5
    b = r.render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))  # still the resident copies
    monkeypatch.setenv("VR_ALWAYS_REUPLOAD", "1")
    c = r.render()
    assert not np.array_equal(a, c)
    monkeypatch.delenv("VR_ALWAYS_REUPLOAD")
    gx.touch()
    r.VolumeIllumination.touch()
    d = r.render()
    assert np.array_equal(c.view(np.uint32), d.view(np.uint32))
    r.delete()


def _slab_chain(data, es, bounds, lights, lut, ra_args, W, H, merged=True):
    """Render `data` as len(bounds)-1 z-slabs, each synced on its own (only its planes resident):
    the ascending sweep over the slabs, then the descending one, chaining the ray state (merged:
    the top slab marches the descending rays in its ascending launch, direction 0, as
    parallel.sort_last_sweeps does; otherwise it runs both sweeps)."""
    import torch
    from volume_renderer_amd import mex
    D = data.shape[2]
    state = torch.zeros(mex.SLAB_PLANES * W * H, dtype=torch.float32, device="cuda")
    ra, keep = mex.render_args(lights, lut, *ra_args)
    nslab = len(bounds) - 1
    if merged:
        order = [(s, +1 if s < nslab - 1 else 0) for s in range(nslab)] + [(s, -1) for s in reversed(range(nslab - 1))]
    else:
        order = [(s, +1) for s in range(nslab)] + [(s, -1) for s in reversed(range(nslab))]
    for i, (s, direction) in enumerate(order):
        z0, z1 = bounds[s], bounds[s + 1]
        first, count = mex.slab_planes(data.shape, es, z0, z1)
        sub = vr.Volume(np.asfortranarray(data[:, :, first:first + count]))
        h = vr.volumeRender("new")
        vr.volumeRender("sync_volumes", h, np.uint64(0), sub, vr.Volume(1), sub)
        mex.render_slab(h, ra, mex.slab(D, first, z0, z1, direction), 0 if i == 0 else state.data_ptr(),
                        state.data_ptr())
        torch.cuda.synchronize()
        vr.volumeRender("delete", h)
    st = state.view(mex.SLAB_PLANES, W, H).cpu().numpy()
    return np.ascontiguousarray(np.transpose(st[:3], (2, 1, 0))), st  # [H, W, 3]


def _slab_case(case):
    if case == "cube3":
        return O.shell_volume(48), [1, 1, 1], [-np.inf, 17, 31, np.inf]
    if case == "one":  # a single slab: one launch marches every ray (direction 0)
        return O.shell_volume(48), [1, 1, 1], [-np.inf, np.inf]
    if case == "pow2":  # a power-of-two cube: the fast variant's half-texel taps; thin slabs
        return O.shell_volume(64), [1, 1, 1], [-np.inf, 20, 21.5, 22, 40, np.inf]
    if case == "gap":  # empty planes up to just before a boundary (and after the next): the staged
        # boxes there are all zero, and an empty-chunk leap must not carry a ray into the next slab
        d = O.shell_volume(48).copy(order="F")
        d[:, :, :24] = 0
        d[:, :, 37:] = 0
        return d, [1, 1, 1], [-np.inf, 26, 35, np.inf]
    # anisotropic element size and depth: the gradient taps reach further than +-0.5 plane; a slab
    # thinner than a step is crossed without an owned sample by some rays
    data = np.asfortranarray(O.shell_volume(48)[:, :40, :])
    data = np.asfortranarray(np.concatenate([data, data[:, :, ::-1]], axis=2)[:, :, :70])
    return data, [2.0, 1.0, 1.0], [-np.inf, 12.5, 30, 30.2, 51, np.inf]


@pytest.mark.parametrize("lanes", ["1", "2", "4"])
@pytest.mark.parametrize("shade", ["fast", "exact"])
@pytest.mark.parametrize("case,merged", [("cube3", True), ("cube3", False), ("aniso5", True), ("one", True),
                                         ("pow2", True), ("gap", True)])
def test_sort_last_slabs_match_the_whole_volume(monkeypatch, counter_clock, case, merged, shade, lanes):
    """Sort-last bricks: a volume split into z-slabs, each rendered with only
    its own planes resident, composited by passing the exact ray state from slab to slab in ray
    order (ascending z for rays with dir.z >= 0, descending for the others), each slab resuming the
    march at the ray's next sample, gives the one-volume image bit for bit -- same sample
    positions, step counts and early exits -- with any depth lanes in the slab launches.  The chain
    is also checked against the oracle's render of the whole volume (SURVEY.md 8c tolerance)."""
    monkeypatch.setenv("VR_DEPTH_LANES", lanes)
    if shade == "exact":
        monkeypatch.setenv("VR_EXACT_SHADE", "1")
    else:
        monkeypatch.delenv("VR_EXACT_SHADE", raising=False)
    data, es, bounds = _slab_case(case)
    W, H = 88, 72
    v = vr.Volume(data)
    r = ex1_renderer(v, res=(W, H))
    r.ElementSizeUm = es
    monkeypatch.delenv("VR_DEPTH_LANES")
    full = r.render()
    monkeypatch.setenv("VR_DEPTH_LANES", lanes)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    ra_args = (np.float32([1.0, 0.4, 0.6]), np.float32(es), np.uint64([H, W]),
               np.flip(r.RotationMatrix, 0).astype(np.float32), np.float32([0, 3.0, 6.0]), np.float32(0.9),
               np.float32([1, 1, 0]))
    img, st = _slab_chain(data, es, bounds, lights, r.VolumeIllumination, ra_args, W, H, merged)
    assert full.max() > 0
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))
    assert not st[4].any()  # every ray finished
    if lanes == "1":  # the chain against the oracle's whole-volume render, default (fast) and exact shading
        S = O.OracleSession()
        oh = S.new()
        ov = O.OVolume(data, 3)
        S.sync_volumes(oh, 0, ov, O.OVolume(np.ones((1, 1), np.float32), 5), ov)
        olut = O.OVolume(r.VolumeIllumination.Data, 7)
        oargs = [np.asarray(a) for a in ra_args]
        olights = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
        ref32, _ = S.render(oh, olights, olut, *oargs, threads=4)
        ref64, _ = S.render(oh, olights, olut, *oargs, double=True, threads=4)
        assert_parity(img, ref32, ref64, f"slab chain {case} {shade}")
    r.delete()


def test_slab_render_checks_the_bound_planes(counter_clock):
    """vr_render_slab reads the BOUND emission volume (the last sync on any handle, as vr_render
    does); a slab whose bound planes would reach past the volume depth is refused, not marched
    (its virtual plane base would address memory outside the resident buffer)."""
    import torch
    from volume_renderer_amd import mex
    W, H = 32, 24
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1])]
    ra, keep = mex.render_args(lights, vr.Volume(vr.HenyeyGreenstein(16)), np.float32([1.0, 0.4, 0.6]),
                               np.float32([1, 1, 1]), np.uint64([H, W]), np.flip(O.rotation(125, 25, 0), 0).astype(np.float32),
                               np.float32([0, 3.0, 6.0]), np.float32(0.9), np.float32([1, 1, 0]))
    state = torch.zeros(mex.SLAB_PLANES * W * H, dtype=torch.float32, device="cuda")
    h = vr.volumeRender("new")
    big = vr.Volume(O.shell_volume(40)[:, :, :30].copy(order="F"))
    vr.volumeRender("sync_volumes", h, np.uint64(0), big, vr.Volume(1), big)
    with pytest.raises(Exception):
        mex.render_slab(h, ra, mex.slab(40, 20, 20.0, np.inf, +1), 0, state.data_ptr())
    mex.render_slab(h, ra, mex.slab(40, 10, 12.0, np.inf, +1), 0, state.data_ptr())  # planes 10..39: fits
    torch.cuda.synchronize()
    vr.volumeRender("delete", h)


@pytest.mark.parametrize("lit", [True, False])
def test_fused_stereo_equals_two_renders(monkeypatch, counter_clock, lit):
    """Fused stereo: vr_render_stereo renders both eyes in one launch; the
    images are those of the reference's two 'render' calls (VolumeRender.m:278-287), bit for bit."""
    v = vr.Volume(O.shell_volume(44))
    r = ex1_renderer(v, res=(90, 70), lights=lit)
    r.CameraXOffset = 0.5
    monkeypatch.setenv("VR_NO_FUSED_STEREO", "1")
    two = r.render()
    monkeypatch.delenv("VR_NO_FUSED_STEREO")
    monkeypatch.setenv("VR_FUSED_STEREO", "1")
    fused = r.render()
    monkeypatch.delenv("VR_FUSED_STEREO")
    assert two.max() > 0 and two.shape == fused.shape
    assert np.array_equal(np.asarray(two, np.float32).view(np.uint32), np.asarray(fused, np.float32).view(np.uint32))
    r.delete()


@pytest.mark.gpu
@pytest.mark.parametrize("k", ["2", "4"])
def test_paired_stereo_tiles_equal_two_renders(monkeypatch, counter_clock, k):
    """Fused stereo with paired tiles (VR_STEREO_PAIR=1, vr_march.hip SCHED 4): each wave
    marches half a tile of each eye -- the right eye's column c with the left eye's c + shift -- and
    stages one box for both.  Every pixel of both eyes is marched once with its own arithmetic, so
    the pair is bit for bit the reference's two renders, for the converging shift and others
    (none, odd, wider than the image)."""
    from volume_renderer_amd import mex
    monkeypatch.setenv("VR_DEPTH_LANES", k)
    monkeypatch.setenv("VR_WIDE_SLOT", "0")  # (paired tiles are built for the default slot only)
    v = vr.Volume(O.shell_volume(64))  # a power-of-two cube: the half-texel tap launch
    r = ex1_renderer(v, res=(90, 70), lights=True)
    r.CameraXOffset = 0.5
    monkeypatch.setenv("VR_NO_FUSED_STEREO", "1")
    two = np.asarray(r.render(), np.float32)
    monkeypatch.delenv("VR_NO_FUSED_STEREO")
    monkeypatch.setenv("VR_FUSED_STEREO", "1")
    monkeypatch.setenv("VR_STEREO_PAIR", "1")
    assert two.max() > 0
    for shift in (None, "1", "4", "13", "200"):
        if shift is None:
            monkeypatch.delenv("VR_STEREO_PAIR_SHIFT", raising=False)
        else:
            monkeypatch.setenv("VR_STEREO_PAIR_SHIFT", shift)
        img = np.asarray(r.render(), np.float32)
        # (the SCHED argument, before the light-count specialisation NL)
        assert mex.last_march_kernel().split(",")[-2].strip() == "4", (shift, mex.last_march_kernel())
        assert np.array_equal(img.view(np.uint32), two.view(np.uint32)), (k, shift)
    r.delete()


def _channel_pair(lit):
    """Two channels of an examples/example3.m-style frame: the main channel (V_shell) and a
    structure channel (a second field) with their own colour and factors, one object each."""
    n = 40
    g = np.linspace(-1.0, 1.0, n, dtype=np.float32)
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    blob = np.asfortranarray(np.exp(-4.0 * ((X - 0.2) ** 2 + (Y + 0.1) ** 2 + Z ** 2)).astype(np.float32))
    main = ex1_renderer(vr.Volume(O.shell_volume(n)), res=(90, 70), lights=lit)
    struct = ex1_renderer(vr.Volume(blob), res=(90, 70), lights=lit)
    struct.Color = [0, 1, 0]
    struct.FactorEmission = 0.5
    struct.FactorAbsorption = 1.0
    return main, struct


@pytest.mark.gpu
@pytest.mark.parametrize("lit", [True, False])
@pytest.mark.parametrize("stereo", [False, True])
def test_fused_channels_equal_separate_renders(monkeypatch, counter_clock, lit, stereo):
    """Multi-channel frame: VolumeRender.renderChannels marches the channels
    (x both stereo eyes) in one launch; each channel's image is bit for bit what its own render()
    gives (the reference renders the channels one after the other, examples/example3.m)."""
    def pair():  # fresh objects and volumes: every channel's sync uploads (see below)
        rs = _channel_pair(lit)
        for r in rs:
            r.CameraXOffset = 0.5 if stereo else 0
        return rs

    # (objects stay referenced: 'delete' resets every handle's device state: ~MManager -> cudaDeviceReset)
    main, struct = pair()
    sep = [main.render(), struct.render()]
    fp, up = pair(), None
    fused = vr.VolumeRender.renderChannels(list(fp))
    monkeypatch.setenv("VR_NO_FUSED_CHANNELS", "1")
    up = pair()
    unfused = vr.VolumeRender.renderChannels(list(up))
    monkeypatch.delenv("VR_NO_FUSED_CHANNELS")
    bits = lambda x: np.asarray(x, np.float32).view(np.uint32)
    for a, b, c in zip(sep, fused, unfused):
        assert a.max() > 0 and a.shape == b.shape == c.shape
        assert np.array_equal(bits(a), bits(b))
        assert np.array_equal(bits(a), bits(c))
    # Unchanged channels of a later frame (a movie): each renders its own volumes.  (The
    # reference's textures are module globals and its upload dedup is per object,
    # mmanager.hxx:178-201: there, an unchanged object renders whatever another object bound last.)
    again = vr.VolumeRender.renderChannels([main, struct])
    for a, b in zip(again, sep):
        assert np.array_equal(bits(a), bits(b))
    for r in (main, struct) + fp + up:
        r.delete()


@pytest.mark.gpu
def test_channels_mixed_gradient_modes(monkeypatch, counter_clock):
    """A lookup-gradient channel (not marched in the fused launch) beside an on-the-fly one: each
    is rendered against its own synced textures, identical to its own render()."""
    def pair():
        main, struct = _channel_pair(True)
        gy, gx, gz = np.gradient(np.asarray(struct.VolumeEmission.Data, np.float64))
        for name, gvol in (("VolumeGradientX", gx), ("VolumeGradientY", gy), ("VolumeGradientZ", gz)):
            setattr(struct, name, vr.Volume(np.asfortranarray(gvol.astype(np.float32))))
        return main, struct

    main, struct = pair()
    sep = [main.render(), struct.render()]
    fp = pair()
    fused = vr.VolumeRender.renderChannels(list(fp))
    for r in (main, struct) + fp:
        r.delete()
    for a, b in zip(sep, fused):
        assert a.max() > 0
        assert np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.gpu
def test_channels_device_images_and_fp32_sum(counter_clock):
    """vr_render_channels_device writes each channel's image where the host variant returns it, bit
    for bit; vr_sum_channels_device adds them in channel order in fp32 (the channel sum of
    examples/example3.m:239, kept on the device)."""
    import torch
    from volume_renderer_amd import mex

    def three():
        main, struct = _channel_pair(True)
        third = ex1_renderer(vr.Volume(O.shell_volume(40)), res=(90, 70), lights=True)
        third.Color = [1, 0, 0]
        third.FactorEmission = 0.25
        return main, struct, third

    def chans(rs):
        out = []
        for r in rs:
            r._validate_volumes()
            argv = r._render_argv(np.float32(0.0), np.flip(r.ImageResolution))
            out.append((r.objectHandle, r.TimeLastMemSync,
                        [r.VolumeEmission, r.VolumeReflection, r.VolumeAbsorption], argv))
        return out

    hr = three()
    host = mex.render_channels(chans(hr))
    dr = three()
    n = host[0].size
    d = torch.zeros(3 * n, dtype=torch.float32, device="cuda")
    s = torch.zeros(n, dtype=torch.float32, device="cuda")
    mex.render_channels_device(chans(dr), d.data_ptr())
    mex.sum_channels_device(d.data_ptr(), 3, 1, n, s.data_ptr())
    torch.cuda.synchronize()
    dev = d.cpu().numpy().reshape(3, n)
    flat = [np.asarray(h, np.float32).reshape(-1, order="F") for h in host]
    for i in range(3):
        assert flat[i].max() > 0
        assert np.array_equal(dev[i].view(np.uint32), flat[i].view(np.uint32))
    want = (flat[0] + flat[1]) + flat[2]
    assert np.array_equal(s.cpu().numpy().view(np.uint32), want.view(np.uint32))
    for r in hr + dr:
        r.delete()


def test_scheduled_partition_under_a_changing_camera(monkeypatch, counter_clock):
    """The longest-first schedule of a short partitioned launch (one part of 8, depth lanes, few
    waves per wave slot) orders workgroups by the PREVIOUS launch of the same shape; under a camera
    that moves every frame that order is stale.  The image must not depend on it: every frame of
    the scheduled part equals the same part rendered unscheduled (VR_SCHED=0), bit for bit."""
    import torch
    from volume_renderer_amd import mex
    n, W, H = 64, 320, 200
    v = vr.Volume(O.shell_volume(n))
    lut = vr.Volume(vr.HenyeyGreenstein(32))
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    h = vr.volumeRender("new")
    vr.volumeRender("sync_volumes", h, np.uint64(0), v, vr.Volume(1), v)
    part = mex.partition(16, 3, 8)
    cols = mex.partition_columns(W, part)
    assert mex.depth_lanes(cols, H) > 1
    out = torch.empty(3 * cols * H, dtype=torch.float32, device="cuda")
    for k in range(6):
        R = np.flip(O.rotation(125 + 9 * k, 25 - 4 * k, 3 * k), 0).astype(np.float32)
        ra, keep = mex.render_args(lights, lut, np.float32([1, 0.4, 0.6]), np.float32([1, 1, 1]),
                                   np.uint64([H, W]), R, np.float32([0, 3, 6]), np.float32(0.9), np.float32([1, 1, 0]))
        monkeypatch.delenv("VR_SCHED", raising=False)
        mex.render_device(h, ra, out.data_ptr(), part)
        torch.cuda.synchronize()
        sched = out.cpu().numpy().copy()
        monkeypatch.setenv("VR_SCHED", "0")
        mex.render_device(h, ra, out.data_ptr(), part)
        torch.cuda.synchronize()
        plain = out.cpu().numpy()
        assert plain.max() > 0
        assert np.array_equal(sched.view(np.uint32), plain.view(np.uint32)), k
    monkeypatch.delenv("VR_SCHED", raising=False)
    vr.volumeRender("delete", h)


@pytest.mark.parametrize("tail_pct", ["0", "60"])
def test_full_frame_schedule_keeps_the_image(monkeypatch, counter_clock, tail_pct):
    """Full frames (many waves per wave slot) are measured on their first launch and every
    VR_SCHED_REMEASURE-th after; when the heaviest block would form a tail the frames follow the
    heavy-first order (VR_SCHED_TAIL_PCT=0 forces it), else no schedule.  Whatever the order, every
    frame equals the unscheduled render bit for bit, through measured, ordered and re-measured
    launches under a moving camera."""
    monkeypatch.setenv("VR_SCHED_TAIL_PCT", tail_pct)
    monkeypatch.setenv("VR_SCHED_REMEASURE", "3")
    v = vr.Volume(O.shell_volume(64))
    frames = {}
    for mode in ("sched", "plain"):
        if mode == "plain":
            monkeypatch.setenv("VR_SCHED_FULL", "0")
        else:
            monkeypatch.delenv("VR_SCHED_FULL", raising=False)
        r = ex1_renderer(v, res=(1280, 1280))
        out = []
        for k in range(7):
            r.rotate(4 if k else 0, 2 if k else 0, 0)
            out.append(r.render())
        frames[mode] = out
        r.delete()
    monkeypatch.delenv("VR_SCHED_FULL", raising=False)
    for k, (a, b) in enumerate(zip(frames["sched"], frames["plain"])):
        assert a.max() > 0
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k


def test_bounce_upload_is_bit_identical(monkeypatch, counter_clock):
    """A host volume uploaded through the pinned bounce ring (VR_UPLOAD_BOUNCE=1, vr_resources.h
    Bounce: 16 MiB pieces through 16 pinned buffers filled by 3 host threads) renders bit for bit as
    the runtime's pageable copy.  322 MB of ragged extent: 20 pieces (the ring wraps), the last one
    partial."""
    rng = np.random.default_rng(5)
    data = np.asfortranarray(rng.random((430, 433, 431), dtype=np.float32) * np.float32(0.02))
    v = vr.Volume(data)
    r = ex1_renderer(v, res=(96, 80))
    monkeypatch.setenv("VR_UPLOAD_BOUNCE", "0")
    base = r.render()
    monkeypatch.setenv("VR_UPLOAD_BOUNCE", "1")
    monkeypatch.setenv("VR_UPLOAD_THREADS", "3")
    v.touch()
    got = r.render()
    assert base.max() > 0
    assert np.array_equal(got.view(np.uint32), base.view(np.uint32))
    r.delete()
