"""CPU tests of the oracle itself (no GPU): reference-pinned known answers, sampler known-answer
tests against an independent numpy restatement, analytic compositing checks, and the committed
golden fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
import hashlib
import os

import numpy as np
import pytest

import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ---- Henyey-Greenstein LUT: pinned by the reference generator's own outputs ----

def test_hg_lut_reference_known_answers():
    lut = O.hg_lut(64, 0.8).reshape(-1, order="F")
    # values printed by the reference's HenyeyGreenstein.cc (N=64, g=0.8), SURVEY.md 8c
    assert float(lut[0]) == pytest.approx(3.580975, rel=2e-7, abs=1e-6)
    assert float(lut[1]) == pytest.approx(3.336926, rel=3e-7, abs=1e-6)
    assert float(lut[64]) == pytest.approx(3.336926, rel=3e-7, abs=1e-6)
    assert float(lut[64 ** 3 - 1]) == pytest.approx(0.004934164, rel=2e-7)


def test_hg_lut_golden_hash_and_16cube():
    lut = O.hg_lut(64, 0.8)
    h = hashlib.sha256(np.ascontiguousarray(lut.reshape(-1, order="F")).tobytes()).hexdigest()
    with open(os.path.join(GOLDEN, "hg64_g0.8.sha256")) as f:
        assert h == f.read().split()[0]
    g16 = np.load(os.path.join(GOLDEN, "hg16_g0.8.npy"))
    assert np.array_equal(O.hg_lut(16, 0.8).reshape(-1, order="F").view(np.uint32), g16.view(np.uint32))


def test_hg_lut_symmetry_and_range():
    lut = O.hg_lut(32, 0.8)
    # LUT(b, a, c) ~ LUT(a, b, c): cos(theta) = sin a sin b + cos g cos a cos b
    assert np.allclose(lut, np.transpose(lut, (1, 0, 2)), rtol=1e-5)
    assert (lut > 0).all()
    with pytest.raises(ValueError):
        O.hg_lut(8, 1.5)


# ---- sampler: CUDA linear filter, normalized coords, clamp, 8-bit weights -----

def numpy_tex3d(vol, x, y, z):
    """Independent float64 restatement of the tex3D semantics (weights quantized to 1/256)."""
    v = np.asarray(vol, np.float64)
    dims = v.shape + (1,) * (3 - v.ndim)
    v = v.reshape(dims, order="F")
    idx, ws = [], []
    for c, n in zip((x, y, z), dims):
        c = np.float32(c)
        if np.isnan(c):
            c = np.float32(0)
        xb = np.float32(c * np.float32(n)) - np.float32(0.5)
        fl = np.floor(xb)
        w = np.rint(np.float32((xb - fl) * np.float32(256))) / 256.0
        i = int(fl)
        idx.append((min(max(i, 0), n - 1), min(max(i + 1, 0), n - 1)))
        ws.append(float(w))
    out = 0.0
    for a in (0, 1):
        for b in (0, 1):
            for c in (0, 1):
                wt = (ws[0] if a else 1 - ws[0]) * (ws[1] if b else 1 - ws[1]) * (ws[2] if c else 1 - ws[2])
                out += wt * v[idx[0][a], idx[1][b], idx[2][c]]
    return out


def test_sampler_voxel_centres_and_midpoints():
    v = O.rand_volume(8)
    for (i, j, k) in [(0, 0, 0), (3, 5, 7), (7, 7, 7), (2, 0, 6)]:
        c = [(i + 0.5) / 8, (j + 0.5) / 8, (k + 0.5) / 8]
        assert O.tex3d(v, *c) == pytest.approx(float(v[i, j, k]), abs=0)
    # exact midpoint between voxels 2 and 3 along x
    got = O.tex3d(v, 3 / 8, 4.5 / 8, 4.5 / 8)
    assert got == pytest.approx(0.5 * (float(v[2, 4, 4]) + float(v[3, 4, 4])), rel=1e-6)


def test_sampler_clamp_and_nan():
    v = O.rand_volume(8)
    assert O.tex3d(v, 0.0, 0.5 / 8, 0.5 / 8) == float(v[0, 0, 0])
    assert O.tex3d(v, -3.0, 0.5 / 8, 0.5 / 8) == float(v[0, 0, 0])
    assert O.tex3d(v, 1.0, 7.5 / 8, 7.5 / 8) == float(v[7, 7, 7])
    assert O.tex3d(v, 9.0, 7.5 / 8, 7.5 / 8) == float(v[7, 7, 7])
    assert O.tex3d(v, float("nan"), 0.5 / 8, 0.5 / 8) == float(v[0, 0, 0])  # NaN -> 0 -> edge


def test_sampler_weights_are_quantized_to_8_bits():
    v = np.zeros((4, 1, 1), np.float32)
    v[1] = 1.0
    # xB = 0.3 -> frac 0.3 -> weight rint(76.8)/256 = 77/256 (not 0.3)
    x = (0.3 + 0.5) / 4
    assert O.tex3d(v, x, 0.5, 0.5) == pytest.approx(77 / 256, abs=1e-7)
    assert O.tex3d(v, x, 0.5, 0.5) != pytest.approx(0.3, abs=1e-4)


def test_sampler_random_kats_vs_numpy_restatement():
    v = O.rand_volume(32)
    rng = np.random.default_rng(7)
    pts = rng.uniform(-0.1, 1.1, size=(300, 3)).astype(np.float32)
    for p in pts:
        assert O.tex3d(v, *p) == pytest.approx(numpy_tex3d(v, *p), rel=2e-6, abs=2e-7)
        assert O.tex3d(v, *p, double=True) == pytest.approx(numpy_tex3d(v, *p), rel=1e-6, abs=1e-7)


def test_sampler_non_cubic_and_2d():
    v = O.rand_volume(12)[:, :7, :3].copy(order="F")
    rng = np.random.default_rng(3)
    for p in rng.uniform(0, 1, size=(50, 3)).astype(np.float32):
        assert O.tex3d(v, *p) == pytest.approx(numpy_tex3d(v, *p), rel=2e-6, abs=2e-7)
    flat = O.rand_volume(9)[:, :, 0].copy(order="F")
    for p in rng.uniform(0, 1, size=(20, 3)).astype(np.float32):
        assert O.tex3d(flat, *p) == pytest.approx(numpy_tex3d(flat, *p), rel=2e-6, abs=2e-7)


# ---- host arithmetic --------------------------------------------------------------------------

def test_init_render_box_and_step():
    import ctypes
    L = O.lib()
    bmin, bmax, ts = (ctypes.c_float * 3)(), (ctypes.c_float * 3)(), ctypes.c_float()
    es = (ctypes.c_float * 3)(1, 1, 1)
    L.or_init_render(1024, 1024, 1024, es, bmin, bmax, ctypes.byref(ts))
    assert list(bmax) == [1.0, 1.0, 1.0] and list(bmin) == [-1.0, -1.0, -1.0]
    assert ts.value == pytest.approx(3.1388e-4, rel=1e-4)
    L.or_init_render(64, 64, 64, es, bmin, bmax, ctypes.byref(ts))
    assert ts.value == pytest.approx(5.022e-3, rel=1e-3)
    es2 = (ctypes.c_float * 3)(2, 1, 0.5)  # kernel order (x, y, z)
    L.or_init_render(100, 50, 20, es2, bmin, bmax, ctypes.byref(ts))
    assert bmax[1] == pytest.approx(50 * 1 / (100 * 2)) and bmax[2] == pytest.approx(20 * 0.5 / (100 * 2))
    assert ts.value == pytest.approx(1 / (2.2 * np.sqrt(50 ** 2 + 20 ** 2)), rel=1e-6)


# ---- ray march ---------------------------------------------------------------------------------

def ex1_session(vol, lights=False, lut=None):
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(vol, 5)
    S.sync_volumes(h, 0, v, O.OVolume(np.ones((1, 1), np.float32), 3), v)
    R = np.flip(O.rotation(125, 25, 0), 0).astype(np.float32)
    return S, h, R


def test_c1_step_count_matches_independent_analysis():
    """SURVEY.md A.3 (numpy analysis): 64^3 @ 256^2, ex1 camera: 6.79e6 samples/frame."""
    S, h, R = ex1_session(O.shell_volume(64))
    img, steps = S.render(h, None, None, [1, 0.4, 0.6], [1, 1, 1], [256, 256], R, [0, 3, 6], 0.9, [1, 1, 0])
    assert steps == pytest.approx(6.79e6, rel=5e-3)
    assert np.isfinite(img).all() and img.max() > 0


def test_constant_volume_compositing_closed_form():
    """Homogeneous medium c, EA only, axis-aligned central ray: after n samples
    a = 1 - (1-alpha)^n, rgb = c*tstep*color*(1 - (1-alpha)^n)."""
    c = 0.8
    vol = np.full((16, 16, 16), c, np.float32)
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(vol, 5)
    S.sync_volumes(h, 0, v, v, v)
    W = H = 8
    R = np.eye(3, dtype=np.float32)
    xs, ys = np.array([4]), np.array([4])  # u = v = 0: direction +z
    fe, fa = 1.0, 2.5
    col = np.array([1.0, 0.5, 0.25])
    out, steps = S.render(h, None, None, [fe, 1, fa], [1, 1, 1], [H, W], np.flip(R, 0), [0, 3, 6], 0.999, col,
                          pixels=(xs, ys))
    n = int(steps[0])
    tstep = 1 / (2.2 * np.sqrt(2) * 16)
    assert n == pytest.approx(2 / tstep, abs=2)  # chord 2 world units
    alpha = 1 - np.exp(-fa * c * tstep)
    expect = fe * c * tstep * col * (1 - (1 - alpha) ** n)
    assert np.allclose(out[0], expect, rtol=2e-4)


def test_early_termination_bounds_opacity():
    vol = np.full((16, 16, 16), 5.0, np.float32)
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(vol, 5)
    S.sync_volumes(h, 0, v, v, v)
    out, steps = S.render(h, None, None, [1, 1, 50], [1, 1, 1], [8, 8], np.eye(3)[::-1], [0, 3, 6], 0.5,
                          [1, 1, 1], pixels=(np.array([4]), np.array([4])))
    tstep = 1 / (2.2 * np.sqrt(2) * 16)
    alpha = 1 - np.exp(-50 * 5 * tstep)
    n_exp = int(np.ceil(np.log(0.5) / np.log(1 - alpha)))  # first n with 1-(1-a)^n > 0.5
    assert int(steps[0]) == n_exp


def test_fp32_fp64_envelope_is_small():
    S, h, R = ex1_session(O.shell_volume(32))
    lut = O.OVolume(O.hg_lut(32), 7)
    L = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
    a, _ = S.render(h, L, lut, [1, 0.4, 0.6], [1, 1, 1], [48, 64], R, [0, 3, 6], 0.9, [1, 1, 0])
    b, _ = S.render(h, L, lut, [1, 0.4, 0.6], [1, 1, 1], [48, 64], R, [0, 3, 6], 0.9, [1, 1, 0], double=True)
    d = np.abs(a.astype(np.float64) - b)
    assert np.percentile(d, 99) <= 1e-3 * np.abs(b).max()


@pytest.mark.parametrize("name", ["c1_ea_64", "hg2_compute_32", "hg1_lookup_24", "stereo_right_24"])
def test_golden_fixtures(name):
    """The oracle reproduces its committed golden images bit for bit (tests/golden/make_golden.py)."""
    import golden_cases as G
    data = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    img, steps = G.CASES[name]()
    assert int(data["steps"]) == steps
    assert np.array_equal(img.view(np.uint32), data["image"].view(np.uint32))
    img64, _ = G.oracle_render(name, double=True)
    assert np.array_equal(img64.view(np.uint32), data["image64"].view(np.uint32))


def test_assumption_variants_build_and_differ():
    """The oracle's assumption variants (oracle/variants/, tools/parity_band.py) load and render;
    truncating filter weights moves the EA-only 64^3 image far outside the fp32 envelope, a fused
    sampler coordinate changes nothing on a power-of-two grid (c*N is exact there)."""
    import golden_cases as G
    sc = G.SCENES["c1_ea_64"]
    S = O.OracleSession()
    h = S.new()
    v = O.OVolume(sc["em"](), G.STAMP_EM)
    S.sync_volumes(h, 0, v, O.OVolume(np.ones((1, 1), np.float32), G.STAMP_RE), v)
    args = G.render_argv(sc, None, None)[2:]
    base, _ = S.render(h, None, None, *args, threads=4)
    vdir = os.path.join(os.path.dirname(O.LIB_PATH), "variants")
    trunc, _ = S.render(h, None, None, *args, threads=4, lib_path=os.path.join(vdir, "liboracle_trunc.so"))
    fused, _ = S.render(h, None, None, *args, threads=4, lib_path=os.path.join(vdir, "liboracle_axis_fma.so"))
    assert np.isfinite(trunc).all() and np.abs(trunc - base).max() > 1e-4 * base.max()
    assert np.array_equal(fused.view(np.uint32), base.view(np.uint32))
