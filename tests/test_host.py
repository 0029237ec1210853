"""CPU tests of the product's host side (no GPU): the C-ABI library loads and exports every
declared symbol; host-only entry points (HG LUT, timestamp, partition math, the slot state
machine) agree with the oracle's independent restatement; the Python mirror of the MATLAB API
marshals and validates like the reference; errors are loud (no CPU fallback)."""
import ctypes
import itertools
import os
import re
import time

import numpy as np
import pytest

import oracle as O
import volume_renderer_amd as vr
from volume_renderer_amd import _lib, mex, parallel
from volume_renderer_amd.volume_render import VolumeRender, _cosd, _imcrop, _sind

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "vrhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vr_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = vr.lib()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    assert {s for s, _, _ in _lib.SIGNATURES} == set(syms)
    assert b"gfx950" in L.vr_version()


def test_hip_error_log_reads_without_a_gpu():
    """vr_hip_errors (the log of HIP errors the library handled or found pending, never dropped)
    reads without touching the device: a count and well-formed lines."""
    n, lines = _lib.hip_errors()
    assert n >= 0 and len(lines) <= min(n, 32)
    for l in lines:
        assert re.match(r"^(handled|pending|pending at entry): hipError\w+ \(\d+\) at .+", l), l


def test_library_is_built_for_gfx950_only():
    out = os.popen(f"strings -a {_lib.LIB_PATH} | grep -o 'amdgcn-amd-amdhsa--gfx[0-9a-z]*' | sort -u").read()
    assert "gfx950" in out and not re.search(r"gfx9[0-4]", out.replace("gfx950", ""))


@pytest.mark.parametrize("n,g", [(64, 0.8), (16, 0.8), (20, -0.3), (7, 0.0), (1, 1.0)])
def test_hg_lut_product_matches_oracle_bitwise(n, g):
    a = vr.HenyeyGreenstein(n, g)
    b = O.hg_lut(n, g)
    assert a.shape == (n, n, n) and a.flags.f_contiguous
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_hg_lut_rejects_g_out_of_range():
    with pytest.raises(vr.VrError, match=r"g must be in interval \[-1,1\]"):
        vr.HenyeyGreenstein(8, 1.01)


def test_timestamp_is_low_32_bits_of_ms():
    t = int(vr.timestamp())
    now = int(time.time() * 1000) & 0xFFFFFFFF
    assert 0 <= t < 2 ** 32
    assert abs(((now - t + 2 ** 31) % 2 ** 32) - 2 ** 31) < 5000


@pytest.mark.parametrize("W,bc,np_", [(1920, 16, 8), (1920, 16, 1), (123, 7, 3), (5, 16, 4), (0, 4, 2)])
def test_partition_columns(W, bc, np_):
    counts = [mex.partition_columns(W, mex.partition(bc, p, np_)) for p in range(np_)]
    assert sum(counts) == W
    for p in range(np_):
        idx = parallel.partition_column_indices(W, bc, p, np_)
        assert len(idx) == counts[p]
    allc = np.concatenate([parallel.partition_column_indices(W, bc, p, np_) for p in range(np_)])
    assert np.array_equal(np.sort(allc), np.arange(W))
    assert mex.partition_columns(W, mex.partition(bc, np_, np_)) == -1


# ---- upload / slot state machine (syncWithDevice, kernel.cu:739-867) ----------------------------

def _oracle_transition(idx_in, em_obj, ab_obj, re_obj, lus):
    """Run one sync through the oracle's session model starting from slot state idx_in with all
    arrays present; objects identify volumes (same object == same ptr/last_update/size)."""
    S = O.OracleSession()
    h = S.new()
    m = S.handles[h]
    S.idx = {O.EM: idx_in[0], O.AB: idx_in[1], O.RE: idx_in[2]}
    for s in (O.EM, O.AB, O.RE):
        m.arr[s] = object()
        S.bind[s] = m.arr[s]
    vols = {k: O.OVolume(np.zeros(2, np.float32), lus[k]) for k in set((em_obj, ab_obj, re_obj))}
    # no real upload: record what happens instead
    S._sync_volume = lambda m_, tex, slot: (S.bind.__setitem__(tex, "new"), m_.arr.__setitem__(slot, "new"))
    S.sync_volumes(h, 100, vols[em_obj], vols[re_obj], vols[ab_obj])
    unbound = [S.bind[s] is None for s in (O.EM, O.AB, O.RE)]
    return [S.idx[O.EM], S.idx[O.AB], S.idx[O.RE]], unbound, vols


def test_slot_state_machine_matches_oracle():
    L = vr.lib()
    states = [(0, 0, 2), (0, 0, 0), (2, 0, 0), (2, 0, 1), (0, 0, 1), (2, 1, 2)]
    assignments = [("a", "a", "a"), ("a", "a", "b"), ("a", "b", "a"), ("a", "b", "b"), ("a", "b", "c")]
    checked = 0
    for idx_in, (e, a, r) in itertools.product(states, assignments):
        objs = sorted(set((e, a, r)))
        for lu_bits in itertools.product((50, 200), repeat=len(objs)):
            lus = dict(zip(objs, lu_bits))
            idx_o, unb_o, vols = _oracle_transition(idx_in, e, a, r, lus)
            req = {k: lus[k] > 100 for k in objs}
            i_in = (ctypes.c_int32 * 3)(*idx_in)
            i_out, u_out = (ctypes.c_int32 * 3)(), (ctypes.c_int32 * 3)()
            L.vr_debug_slot_transition(i_in, e == a, e == r, a == r, req[e], req[a], req[r], i_out, u_out)
            assert list(i_out) == idx_o, (idx_in, e, a, r, lus)
            assert [bool(x) for x in u_out] == unb_o, (idx_in, e, a, r, lus)
            checked += 1
    assert checked > 100


def test_reference_quirk_paths():
    """Absorption is never selected (idx stays emission); Em==Re sets idxRe = emission;
    the simEmAb typo path routes emission through the reflection texture."""
    L = vr.lib()

    def tr(idx, sims, reqs):
        i_in = (ctypes.c_int32 * 3)(*idx)
        o, u = (ctypes.c_int32 * 3)(), (ctypes.c_int32 * 3)()
        L.vr_debug_slot_transition(i_in, *sims, *reqs, o, u)
        return list(o), list(u)

    assert tr((0, 0, 2), (0, 0, 0), (1, 1, 1)) == ([0, 0, 2], [0, 0, 0])   # all distinct, all new
    assert tr((0, 0, 2), (1, 1, 1), (1, 1, 1))[0] == [0, 0, 0]             # all the same volume
    assert tr((0, 0, 2), (1, 0, 0), (0, 0, 1)) == ([2, 0, 2], [1, 0, 0])   # Em==Ab, only Re new


# ---- the Python mirror of the MATLAB API ---------------------------------------------------------

def test_cosd_sind_exact_at_right_angles():
    for a, s, c in [(0, 0, 1), (90, 1, 0), (180, 0, -1), (270, -1, 0), (-90, -1, 0), (450, 1, 0)]:
        assert _sind(a) == s and _cosd(a) == c
    assert _sind(30) == pytest.approx(0.5)


def test_rotate_matches_oracle_rotation():
    r = object.__new__(VolumeRender)
    object.__setattr__(r, "RotationMatrix", np.eye(3))
    r.rotate(125, 25, 0)
    r.rotate(0, 5, 0)
    expect = O.rotation(0, 5, 0, R=O.rotation(125, 25, 0))
    assert np.array_equal(r.RotationMatrix, expect)


def test_imcrop_as_used_by_stereo():
    img = np.arange(2 * 10 * 3, dtype=np.float32).reshape(2, 10, 3)
    delta = 3
    left = _imcrop(img, delta + 1, img.shape[1])
    right = _imcrop(img, 0, img.shape[1] - delta)
    assert np.array_equal(left, img[:, delta:, :]) and np.array_equal(right, img[:, :10 - delta, :])


def test_volume_grad_matches_matlab_gradient():
    d = O.rand_volume(10)[:, :7, :5].copy(order="F")
    gx, gy, gz = vr.Volume(d).grad()
    for g, o in zip((gx, gy, gz), O.matlab_gradient(d)):
        assert np.array_equal(g.Data, o)


def test_volume_is_single_column_major_and_stamped(counter_clock):
    v = vr.Volume(np.arange(24, dtype=np.float64).reshape(2, 3, 4))
    assert v.Data.dtype == np.float32 and v.Data.flags.f_contiguous
    t0 = int(v.TimeLastUpdate)
    v.Data = v.Data * 2
    assert int(v.TimeLastUpdate) > t0
    assert mex._matlab_dims(vr.Volume(1).Data) == (1, 1, 1)
    assert mex._matlab_dims(vr.Volume(np.ones((5, 6))).Data) == (5, 6, 1)


def test_light_source_validation():
    with pytest.raises(ValueError):
        vr.LightSource([1, 2], [1, 1, 1])
    ls = vr.LightSource([500, 1000, 550], [0, 1, 1])
    assert ls.Position.dtype == np.float32


def test_mex_argument_errors():
    with pytest.raises(vr.VrError, match="command string"):
        vr.volumeRender("x" * 64)
    with pytest.raises(vr.VrError, match="class instance handle"):
        vr.volumeRender("render")
    with pytest.raises(vr.VrError, match="uint64 scalar"):
        vr.volumeRender("mem_info", 5)
    with pytest.raises(vr.VrError, match="Handle not valid"):
        vr.volumeRender("mem_info", np.uint64(12345))


def test_render_args_marshalling():
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    lut = vr.Volume(vr.HenyeyGreenstein(4))
    R = O.rotation(125, 25, 0)
    ra, keep = mex.render_args(lights, lut, np.float32([1, 0.4, 0.6]), np.float32([1, 2, 3]), np.uint64([1080, 1920]),
                               np.flip(R, 0).astype(np.float32), np.float32([0, 3, 6]), np.float32(0.9),
                               np.float32([1, 1, 0]))
    assert ra.num_lights == 2 and list(ra.lights[1].position) == [0, 550, 90]
    assert list(ra.resolution) == [1080, 1920]
    assert np.allclose(list(ra.rotation_flipped), np.flip(R, 0).astype(np.float32).reshape(-1, order="F"))
    ra2, _ = mex.render_args(False, lut, *([np.float32([1, 1, 1])] * 2), np.uint64([2, 2]),
                             np.eye(3, dtype=np.float32), np.float32([0, 3, 6]), np.float32(0.9),
                             np.float32([1, 1, 1]))
    assert ra2.num_lights == -1 and not ra2.illumination


@pytest.mark.skipif(__import__("conftest").gpu_available(), reason="checks the no-GPU failure mode")
def test_no_silent_cpu_fallback_without_gpu():
    with pytest.raises(vr.VrError):
        VolumeRender()


def test_committed_traffic_matches_bench_default_workload():
    """bench.py reports roofline.traffic / .valu only when the newest profiles/<round>/traffic.json
    was measured on its default workload (the metric config); the key must match verbatim."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    path = bench._latest_traffic_json()
    with open(path) as fh:
        tj = json.load(fh)
    entries = tj.get("entries", [tj])  # round 4: one entry per BASELINE config
    want = {bench.workload_name(1024, 1920, 1080, 2, "compute"), bench.workload_name(1024, 1024, 768, 2, "compute"),
            bench.workload_name(1024, 1920, 1080, 2, "lookup"), bench.workload_name(2048, 4096, 4096, 2, "compute")}
    got = {e["workload"] for e in entries}
    assert bench.workload_name(1024, 1920, 1080, 2, "compute") in got
    if "entries" in tj:
        assert want <= got, want - got
    for e in entries:
        assert e["bytes_per_launch"] > 0 and e["kernel"].startswith("vr::fast::march_kernel<")


def test_binding_roof_names_the_largest_hardware_fraction():
    """bench.py roofline.binding: the largest of the fetched-bytes, counter-traffic and VALU
    fractions (the F-weighted sample-stream fraction is not a candidate)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    # (round 6: frac is the needed-bytes fraction; the F-weighted one is sample_stream_frac)
    rf = {"frac": 0.46, "sample_stream_frac": 1.07, "traffic": 1.0e12, "valu": {"frac": 0.62}}
    b = bench.binding_roof(rf, 0.265)  # 1 TB in 265 ms = 3.77 TB/s = 0.47 of 8 TB/s
    assert b["roof"] == "valu" and b["frac"] == 0.62
    assert abs(b["candidates"]["hbm_traffic"] - 1.0e12 / 0.265 / 8e12) < 1e-3
    b = bench.binding_roof({"frac": 0.23, "sample_stream_frac": 0.9, "traffic": 1.05e11, "valu": None}, 0.017)
    assert b["roof"] == "hbm_traffic" and set(b["candidates"]) == {"fetched", "hbm_traffic"}
    assert bench.binding_roof({"frac": 0.4, "sample_stream_frac": 0.9, "traffic": None, "valu": None},
                              0.03)["roof"] == "fetched"


def test_cpu_share_is_positive():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert 1 <= bench.cpu_share() <= (os.cpu_count() or 1)


def _gvec_brick_index(X, Y, Z, bx, by):
    """Entry of padded voxel (X, Y, Z) in the 2x2x2-brick lookup-gradient copy (vr_kernels.hip
    interleave3_kernel, DESIGN.md s5 "Lookup-gradient copy")."""
    return (((Z >> 1) * by + (Y >> 1)) * bx + (X >> 1)) * 8 + (X & 1) + 2 * (Y & 1) + 4 * (Z & 1)


@pytest.mark.parametrize("dims", [(5, 4, 3), (6, 7, 2), (2, 2, 2), (9, 5, 6)])
def test_gvec_brick_corner_offsets(dims):
    """The march's corner addressing in the bricked gradient copy (vr_sampling.h gvec_load): from the
    cell's first corner (X, Y, Z) the other seven lie at +dx, +dy, +dz and their sums, with dx = 1 or
    7, dy = 2 or row8 - 2, dz = 4 or plane8 - 4 by the corner's parity -- restated here and checked
    against the layout for every cell of padded volumes with odd and even edges, and the layout
    checked to hold every padded voxel once (bricks past an odd edge are padding)."""
    nx, ny, nz = dims
    px, py, pz = nx + 2, ny + 2, nz + 2
    bx, by, bz = (px + 1) // 2, (py + 1) // 2, (pz + 1) // 2
    row8, plane8 = 8 * bx, 8 * bx * by
    idx = {(X, Y, Z): _gvec_brick_index(X, Y, Z, bx, by)
           for X in range(px) for Y in range(py) for Z in range(pz)}
    assert len(set(idx.values())) == px * py * pz and max(idx.values()) < 8 * bx * by * bz
    for (X, Y, Z), o in idx.items():
        if X + 1 >= px or Y + 1 >= py or Z + 1 >= pz:
            continue
        dx = 7 if X & 1 else 1
        dy = row8 - 2 if Y & 1 else 2
        dz = plane8 - 4 if Z & 1 else 4
        for cx, cy, cz in itertools.product((0, 1), repeat=3):
            assert idx[(X + cx, Y + cy, Z + cz)] == o + cx * dx + cy * dy + cz * dz, (X, Y, Z, cx, cy, cz)
