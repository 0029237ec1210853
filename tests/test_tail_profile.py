"""tools/tail_profile.py (CPU): the occupancy profile of a VR_SCHED_DUMP pair of files (block
durations and start ticks, vr_capi.hip do_render) on a synthetic launch whose answer is known."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, hdr, vals):
    with open(path, "ab") as f:
        np.asarray(hdr, np.uint32).tofile(f)
        np.asarray(vals, np.uint32).tofile(f)


def test_tail_profile_of_a_synthetic_launch(tmp_path):
    # 2 resident slots; blocks (start, duration) in 10 ns ticks: two fill the slots for 100 ticks,
    # then one runs alone for 300 more -- span 400, the last 300 at half residency
    dump = str(tmp_path / "dump")
    starts = [1000, 1000, 1100]  # absolute ticks (the tool subtracts the earliest)
    durs = [100, 100, 300]
    _write(dump, [2, 0, 1, 3], durs)
    _write(dump + ".start", [2, 0, 1, 3], starts)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tail_profile.py"), dump, "2"],
                         capture_output=True, text=True, check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    assert r["k"] == 2 and r["blocks"] == 3 and r["peak_resident"] == 2
    assert abs(r["span_ms"] - 400 / 1e5) < 1e-12
    # idle slot-time: 1 slot for 300 ticks of 2 x 400
    assert abs(r["idle_frac"] - 300 / 800) < 1e-4
    assert abs(r["ms_below_90pct"] - 300 / 1e5) < 1e-12
    assert abs(r["ramp_down_ms"] - 300 / 1e5) < 1e-12
    assert r["longest_ms"][0] == round(300 / 1e5, 3)
