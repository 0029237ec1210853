#!/usr/bin/env python3
"""Summarise a VR_SCHED_DUMP file (block durations of timed launches, vr_capi.hip).

Each record: uint32 header (K, part, num_parts, blocks) then `blocks` uint32 durations in
s_memrealtime ticks (100 MHz).  A block split inside its workgroup (SCHED 5) records twice its
first workgroup's duration.  Prints, per part of the last frame, the longest block, the top
quantiles and the summed block time; with --skip N the first N launches (warmup) are dropped.
"""
import argparse
import numpy as np


def read(path):
    a = np.fromfile(path, dtype=np.uint32)
    out, i = [], 0
    while i + 4 <= a.size:
        k, part, parts, nb = (int(v) for v in a[i:i + 4])
        out.append((k, part, parts, a[i + 4:i + 4 + nb].astype(np.float64) / 100.0))  # us
        i += 4 + nb
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump", nargs="+")
    ap.add_argument("--skip", type=int, default=16)
    args = ap.parse_args()
    for path in args.dump:
        recs = read(path)[args.skip:]
        print(f"{path}: {len(recs)} launches")
        by_part = {}
        for k, part, parts, c in recs:
            by_part.setdefault(part, []).append(c)
        for part in sorted(by_part):
            cs = by_part[part]
            mx = np.mean([c.max() for c in cs])
            top = np.mean([np.sort(c)[::-1][[0, 9, 99, 999]] for c in cs], axis=0)
            tot = np.mean([c.sum() for c in cs])
            print(f"  part {part}: blocks {cs[0].size} max {mx:8.1f} us  #10 {top[1]:7.1f}  #100 {top[2]:7.1f}"
                  f"  #1000 {top[3]:7.1f}  sum {tot / 1e3:8.1f} ms  median {np.mean([np.median(c) for c in cs]):6.1f}")


if __name__ == "__main__":
    main()
