#!/usr/bin/env python3
"""Print the runs of tools/ab_sweep.sh: frame ms, kernel ms, simulated per-part max."""
import glob, json, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*.json")):
    try:
        d = json.load(open(f))
    except ValueError:
        print(f, "(no result)"); continue
    s = d.get("sim_parts_kernel_ms") or {}
    print(f"{f.split('/')[-1]:28s} frame {d['ms_per_step']:8.3f}  kernel {d['roofline']['kernel_ms']:8.3f}  "
          f"part-max {s.get('max')}")
