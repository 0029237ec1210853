import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session", autouse=True)
def _test_switches():
    """The variant tests select kernels through VR_* environment switches, which the library reads
    only after vr_set_option("test_switches", 1) (include/vrhip.h; a MATLAB session never sets it)."""
    try:
        from volume_renderer_amd import mex
        mex.enable_test_switches()
    except (ImportError, OSError):
        pass  # (no library: the CPU tests that need none)
    yield


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


def assert_parity(got: np.ndarray, ref32: np.ndarray, ref64: np.ndarray, what: str = "", min_frac: float = 0.999):
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
    bad = (frac < min_frac) or (stats["max_abs_nearer"] > 1e-2 * scale)
    if bad and os.environ.get("PARITY_DUMP"):
        os.makedirs(os.environ["PARITY_DUMP"], exist_ok=True)
        name = "".join(ch if ch.isalnum() else "_" for ch in (os.environ.get("PYTEST_CURRENT_TEST", "") + what))
        np.savez_compressed(os.path.join(os.environ["PARITY_DUMP"], name[-120:] + ".npz"),
                            got=got, ref32=ref32, ref64=ref64)
    assert frac >= min_frac, f"{what}: only {frac:.5f} within envelope; {stats}"
    assert stats["max_abs_nearer"] <= 1e-2 * scale, f"{what}: |d| {stats['max_abs_nearer']} > 1e-2*max from both oracles; {stats}"
    return stats


def assert_parity_full_size(got: np.ndarray, ref32: np.ndarray, ref64: np.ndarray, what: str = "",
                            max_rms_ratio: float = 1.0):
    """SURVEY.md 8c tolerance at BASELINE sizes (rays of 4-15k samples), on a sample of pixels.

    The per-channel envelope E = |fp32 - fp64| of the oracle is one draw of a rounding random walk
    along the ray: over the lit pixel-channels of a full-size frame it is ~2e-4 of the image maximum
    in RMS, but on a few tenths of a percent of channels it is near zero by chance, and there the
    per-channel test |d| <= 4E + 1e-5 max fails for any fp32 implementation that does not round
    exactly like the oracle.  (Round 2 measured 0.4 % failing channels even for the oracle-op-sequence
    kernel; the cause was the device exponential's rounding bias, fixed in round 3 -- that kernel now
    meets the unfloored test at 100 % of sampled channels, the default fast arithmetic at 99.90-100 %,
    which test_full_size.py asserts separately.)
    So at full size the envelope is floored at its RMS over the lit sampled channels of the same
    image (E' = max(E, rms_lit(E))), and the product may be no farther from the fp32 oracle than the
    fp32 oracle is from exact (fp64) arithmetic: rms_lit(d) <= max_rms_ratio * rms_lit(E), ratio 1 by
    default (round 3: fast arithmetic 0.03-0.14 over the BASELINE configs, the oracle-op-sequence
    kernel 0.001).
    Unchanged: NaN masks equal; no channel farther than 1e-2 max from both oracle renders.  The
    unfloored SURVEY fraction is reported as `frac_within_survey`."""
    assert got.shape == ref32.shape, (got.shape, ref32.shape)
    n_got, n_ref = np.isnan(got), np.isnan(ref32)
    assert np.array_equal(n_got, n_ref), f"{what}: NaN masks differ ({n_got.sum()} vs {n_ref.sum()})"
    g = np.where(n_got, 0, got).astype(np.float64)
    r = np.where(n_ref, 0, ref32).astype(np.float64)
    r64 = np.where(np.isnan(ref64), 0, ref64).astype(np.float64)
    scale = max(float(np.abs(r).max()), 1e-30)
    d = np.abs(g - r)
    env = np.abs(r - r64)
    lit = np.abs(r) > 1e-3 * scale
    rms_e = float(np.sqrt((env[lit] ** 2).mean())) if lit.any() else 0.0
    rms_d = float(np.sqrt((d[lit] ** 2).mean())) if lit.any() else 0.0
    floored = d <= 4 * np.maximum(env, rms_e) + 1e-5 * scale
    near = np.minimum(d, np.abs(g - r64))
    stats = dict(max_abs=float(d.max()), max_abs_nearer=float(near.max()), scale=scale,
                 frac_within=float(floored.mean()), frac_within_survey=float((d <= 4 * env + 1e-5 * scale).mean()),
                 rms_d=rms_d, rms_env=rms_e, rms_ratio=rms_d / rms_e if rms_e else 0.0, lit=float(lit.mean()),
                 bit_exact=float((got.view(np.uint32) == ref32.view(np.uint32)).mean()))
    assert stats["frac_within"] >= 0.999, f"{what}: only {stats['frac_within']:.5f} within the floored envelope; {stats}"
    assert stats["max_abs_nearer"] <= 1e-2 * scale, f"{what}: |d| beyond 1e-2*max from both oracles; {stats}"
    assert stats["rms_ratio"] <= max_rms_ratio, f"{what}: product farther from the fp32 oracle than fp32 rounding; {stats}"
    return stats
