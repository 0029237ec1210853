"""The MATLAB-side volume preprocessing on the device: HenyeyGreenstein,
Volume.normalize and Volume.resize (include/vrhip.h vr_*_device) against the oracle's restatements
(oracle/oracle.py resize_contributions / resize / normalize, the host LUT generator).  Parity is
unpinned for resize (no MATLAB here: the restatement follows imresize's published contributions()
algorithm) and pinned for the LUT through the host generator's known answers (test_oracle.py)."""
import numpy as np
import pytest

import oracle as O

vr = pytest.importorskip("volume_renderer_amd")
from volume_renderer_amd import mex  # noqa: E402

AXES = [(10, 20), (20, 10), (7, 3), (64, 64), (5, 17), (100, 37), (1, 4), (4, 1), (3, 200), (256, 96)]


@pytest.mark.parametrize("a,b", AXES)
def test_resize_contributions_match_oracle(a, b):
    """The product's host-side contributions (vr_resize_contributions) equal the restatement's bit
    for bit; weights sum to 1 per output; indices inside the input."""
    w, i = mex.resize_contributions(a, b)
    ow, oi = O.resize_contributions(a, b)
    assert np.array_equal(w.view(np.uint64), ow.view(np.uint64)) and np.array_equal(i, oi)
    assert np.allclose(w.sum(axis=1), 1.0, rtol=0, atol=1e-12)
    assert i.min() >= 0 and i.max() < a


def test_resize_oracle_known_answers():
    """imresize semantics the restatement must have: same size is the identity; a constant volume
    stays constant (normalised weights); doubling a ramp keeps it monotone and symmetric about its
    centre; an axis is shrunk with the antialiasing (wider) kernel."""
    rng = np.random.default_rng(3)
    d = np.asfortranarray(rng.random((6, 5, 4), dtype=np.float32))
    assert np.array_equal(O.resize(d, d.shape), d)
    c = np.full((5, 6, 7), 0.25, np.float32, order="F")
    assert np.all(O.resize(c, (9, 4, 3)) == np.float32(0.25))
    ramp = np.asfortranarray(np.tile(np.arange(8, dtype=np.float32)[:, None, None], (1, 2, 2)))
    up = O.resize(ramp, (16, 2, 2))[:, 0, 0]
    assert np.all(np.diff(up) > 0)
    assert np.allclose(up + up[::-1], up[0] + up[-1], atol=1e-5)
    w_up, _ = O.resize_contributions(20, 40)
    w_dn, _ = O.resize_contributions(40, 20)
    assert w_dn.shape[1] > w_up.shape[1]


def test_normalize_mirror_matches_oracle():
    """Volume.normalize of the Python mirror (MATLAB's single arithmetic) equals the restatement."""
    rng = np.random.default_rng(5)
    d = np.asfortranarray((rng.standard_normal((9, 8, 7)) * 3).astype(np.float32))
    d[1, 2, 3] = np.nan
    v = vr.Volume(d.copy(order="F"))
    v.normalize(-1, 2.5)
    want = O.normalize(d, -1, 2.5)
    assert np.array_equal(v.Data.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,new", [((40, 30, 20), (64, 30, 11)), ((33, 17, 9), (16, 40, 9)), ((24, 24, 24), (48, 48, 48)),
                                       ((50, 40, 30), (25, 20, 15)), ((17, 23), (40, 9)), ((8, 1, 5), (8, 3, 5))])
def test_resize_device_matches_oracle(shape, new):
    import torch
    rng = np.random.default_rng(sum(shape))
    d = np.asfortranarray(rng.random(shape, dtype=np.float32))
    dims = tuple(shape) + (1,) * (3 - len(shape))
    out_dims = tuple(new) + (1,) * (3 - len(new))
    src = torch.from_numpy(d.reshape(-1, order="F").copy()).cuda()
    dst = torch.full((int(np.prod(out_dims)),), np.nan, dtype=torch.float32, device="cuda")
    mex.resize_device(src.data_ptr(), dims, out_dims, dst.data_ptr())
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    want = O.resize(d, new).reshape(-1, order="F")
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_volume_resize_mirror(counter_clock):
    v = vr.Volume(O.shell_volume(32))
    t0 = v.TimeLastUpdate
    v.resize([48, 20, 32])
    assert v.Data.shape == (48, 20, 32) and v.TimeLastUpdate != t0
    assert np.array_equal(v.Data.view(np.uint32), O.resize(O.shell_volume(32), (48, 20, 32)).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["randn", "nan", "const", "allnan", "inplace"])
def test_normalize_device_matches_oracle(case):
    import torch
    rng = np.random.default_rng(11)
    d = (rng.standard_normal(100_003) * 7 + 2).astype(np.float32)
    if case == "nan":
        d[::997] = np.nan
        d[5] = np.inf
    elif case == "const":
        d[:] = 3.0
    elif case == "allnan":
        d[:] = np.nan
    src = torch.from_numpy(d.copy()).cuda()
    dst = src if case == "inplace" else torch.empty_like(src)
    mex.normalize_device(src.data_ptr(), d.size, 0.0, 1.0, dst.data_ptr())
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    want = O.normalize(d, 0.0, 1.0)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    m = ~np.isnan(want)
    assert np.array_equal(got[m].view(np.uint32), want[m].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,g", [(64, 0.8), (16, 0.8), (33, -0.3), (8, 0.0), (64, 1.0)])
def test_hg_lut_device_vs_host(n, g):
    """The device LUT against the host generator (bit-identical to the reference's known answers):
    the same expression with the host's sines and cosines; only the device powf can differ (measured:
    ~91 % of elements bit-identical, at most 3 ulp apart); bound stated as 4 ulp."""
    import torch
    host = vr.HenyeyGreenstein(n, g).reshape(-1, order="F")
    dev = torch.empty(n ** 3, dtype=torch.float32, device="cuda")
    mex.henyey_greenstein_device(n, g, dev.data_ptr())
    got = dev.cpu().numpy()
    assert np.array_equal(np.isfinite(got), np.isfinite(host))
    m = np.isfinite(host)
    ulp = np.abs(got[m].view(np.int32).astype(np.int64) - host[m].view(np.int32).astype(np.int64))
    print(f"HG({n},{g}) device vs host: {float((ulp == 0).mean()):.4f} bit-identical, max {int(ulp.max())} ulp")
    assert ulp.max() <= 4
