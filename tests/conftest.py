import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


class CounterClock:
    """Deterministic stand-in for the ms clock behind `timestamp` (strictly increasing)."""

    def __init__(self, start=1000):
        self.t = start

    def __call__(self):
        self.t += 1
        return self.t


@pytest.fixture
def counter_clock():
    import volume_renderer_amd as vr
    clk = CounterClock()
    vr.set_clock(clk)
    yield clk
    vr.set_clock(None)


def assert_parity(got: np.ndarray, ref32: np.ndarray, ref64: np.ndarray, what: str = ""):
    """SURVEY.md 8c tolerance: envelope E = |fp32 - fp64| of the oracle;
    |d| <= 4E + 1e-5*max(img) for >= 99.9% of pixel-channels (d = product - fp32 oracle),
    NaN masks identical, and no pixel-channel farther than 1e-2*max(img) from BOTH oracle renders.
    The cap is taken to the nearer of the two because the fp32 oracle has outliers of its own (an
    early-exit step or an acos argument that rounds past -1 flips in fp32 but not in fp64); a
    product value that agrees with the fp64 render there is not an error.  Returns a stats dict."""
    assert got.shape == ref32.shape, (got.shape, ref32.shape)
    n_got, n_ref = np.isnan(got), np.isnan(ref32)
    assert np.array_equal(n_got, n_ref), f"{what}: NaN masks differ ({n_got.sum()} vs {n_ref.sum()})"
    g = np.where(n_got, 0, got).astype(np.float64)
    r = np.where(n_ref, 0, ref32).astype(np.float64)
    r64 = np.where(np.isnan(ref64), 0, ref64).astype(np.float64)
    scale = max(float(np.abs(r).max()), 1e-30)
    d = np.abs(g - r)
    env = np.abs(r - r64)
    ok = d <= 4 * env + 1e-5 * scale
    frac = float(ok.mean()) if ok.size else 1.0
    near = np.minimum(d, np.abs(g - r64))
    stats = dict(max_abs=float(d.max()) if d.size else 0.0, max_abs_nearer=float(near.max()) if d.size else 0.0,
                 scale=scale, frac_within=frac,
                 bit_exact=float((got.view(np.uint32) == ref32.view(np.uint32)).mean()) if got.size else 1.0)
    bad = (frac < 0.999) or (stats["max_abs_nearer"] > 1e-2 * scale)
    if bad and os.environ.get("PARITY_DUMP"):
        os.makedirs(os.environ["PARITY_DUMP"], exist_ok=True)
        name = "".join(ch if ch.isalnum() else "_" for ch in (os.environ.get("PYTEST_CURRENT_TEST", "") + what))
        np.savez_compressed(os.path.join(os.environ["PARITY_DUMP"], name[-120:] + ".npz"),
                            got=got, ref32=ref32, ref64=ref64)
    assert frac >= 0.999, f"{what}: only {frac:.5f} within envelope; {stats}"
    assert stats["max_abs_nearer"] <= 1e-2 * scale, f"{what}: |d| {stats['max_abs_nearer']} > 1e-2*max from both oracles; {stats}"
    return stats
