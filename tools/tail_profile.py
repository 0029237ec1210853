#!/usr/bin/env python3
"""tools/tail_profile.py DUMP [slots] -- occupancy profile of timed march launches from a
VR_SCHED_DUMP run (DUMP: block durations, DUMP.start: block start ticks, both in s_memrealtime
ticks of 10 ns; written by vr_capi.hip do_render).  For each launch: span, the resident-workgroup
count over time, how long the launch runs below 90 % / 50 % of its peak residency (the ramp-down
tail), and the idle fraction of the workgroup slots over the span."""
import json
import sys

import numpy as np


def records(path):
    raw = np.fromfile(path, dtype=np.uint32)
    out, i = [], 0
    while i + 4 <= raw.size:
        k, part, parts, nb = (int(x) for x in raw[i:i + 4])
        out.append(((k, part, parts), raw[i + 4:i + 4 + nb].astype(np.int64)))
        i += 4 + nb
    return out


def main():
    path = sys.argv[1]
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    res = []
    for (hdr, dur), (_, st) in zip(records(path), records(path + ".start")):
        st = st - st.min()  # the low 32 bits of the 100 MHz clock: no wrap within a launch
        end = st + dur
        span = int(end.max())
        ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([end, -np.ones_like(end)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        t, act = ev[:, 0], np.cumsum(ev[:, 1])
        peak = int(act.max()) if not slots else slots
        dt = np.diff(np.append(t, span))
        idle = float(np.sum((peak - act) * dt)) / (peak * span) if span else 0.0
        below = lambda f: float(np.sum(dt[act < f * peak])) / 1e5  # ms (10 ns ticks)
        # the end of the last interval at >= 90 % of peak residency: everything after it is the ramp-down
        t_next = np.append(t[1:], span)
        full = t_next[act >= 0.9 * peak]
        ramp = (span - int(full.max())) / 1e5 if full.size else span / 1e5
        order = np.argsort(-dur)
        res.append({
            "k": hdr[0], "part": hdr[1], "parts": hdr[2], "blocks": int(dur.size),
            "span_ms": span / 1e5, "peak_resident": peak, "idle_frac": round(idle, 4),
            "ms_below_90pct": below(0.9), "ms_below_50pct": below(0.5), "ramp_down_ms": ramp,
            "sum_dur_over_peak_ms": float(dur.sum()) / peak / 1e5,
            "longest_ms": [round(float(dur[j]) / 1e5, 3) for j in order[:5]],
            "longest_start_ms": [round(float(st[j]) / 1e5, 3) for j in order[:5]],
            "last_starts_ms": round(float(np.sort(st)[-1]) / 1e5, 3),
            "median_ms": float(np.median(dur)) / 1e5,
        })
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
