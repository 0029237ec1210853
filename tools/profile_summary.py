#!/usr/bin/env python3
"""Summarise one measurement pass (tools/r*.sh output under gpurun_out/<run>) into profiles/<round>/:
kernel_stats.csv (rocprofv3 --kernel-trace --stats), pmc_summary.txt (per-kernel counter averages),
traffic.json (HBM bytes per launch of the march kernel, read by bench.py for roofline.traffic).

HBM bytes: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 64 B per 128 B request
(MI355X_MICROARCH.md, HBM section), so read bytes = 2 x 1024 x FETCH_SIZE.  The factor is checked
here on stats_kernel, which reads every padded voxel once (known byte count).
usage: tools/profile_summary.py gpurun_out/r13 profiles/round1 [WORKLOAD_STRING]
The workload key defaults to the bench.json line of the run (bench.py matches it verbatim against
its config.workload before it reports roofline.traffic).
Several configurations (round 4, one tools/gpupass.py pass with a bench and a pmc step per config):
  tools/profile_summary.py --configs profiles/round4 PMC_DIR:BENCH_JSON[:NAME] ...
writes traffic.json with one entry per config ({"entries": [...]}, bench.py picks the entry of its
workload and kernel) and configs.json (each config's bench line with its counter-backed fractions)."""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

if sys.argv[1] == "--configs":
    import runpy
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic_configs.py"), run_name="__main__")
    sys.exit(0)
run, out = sys.argv[1], sys.argv[2]
workload = sys.argv[3] if len(sys.argv) > 3 else None
if workload is None:
    with open(os.path.join(run, "bench.json")) as fh:
        workload = json.loads(fh.read().strip().splitlines()[-1])["config"]["workload"]
os.makedirs(out, exist_ok=True)
ks = glob.glob(os.path.join(run, "kt", "*kernel_stats.csv"))
if ks:
    shutil.copy(ks[0], os.path.join(out, "kernel_stats.csv"))

vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(os.path.join(run, "pmc", "pass*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            vals[row["Kernel_Name"]][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])

lines = []
for k in sorted(vals):
    lines.append(k)
    for c in sorted(vals[k]):
        per = vals[k][c]
        lines.append(f"  {c:28s} {sum(per.values()) / len(per):.6g}   (mean over {len(per)} dispatches)")
with open(os.path.join(out, "pmc_summary.txt"), "w") as fh:
    fh.write("\n".join(lines) + "\n")


def mean(kname, counter):
    """Per-dispatch mean of a counter over the dispatches of exactly the kernel `kname`."""
    xs = [v for k, cs in vals.items() if k.split("(")[0].replace("void ", "", 1) == kname
          for v in cs.get(counter, {}).values()]
    return sum(xs) / len(xs) if xs else None


# the kernel bench.py timed (its roofline.kernel, the exact instantiation), else the most-launched
# march kernel of the kernel trace
kname = None
try:
    with open(os.path.join(run, "bench.json")) as fh:
        kname = json.loads(fh.read().strip().splitlines()[-1])["roofline"].get("kernel")
except (OSError, ValueError, KeyError, IndexError):
    pass
if kname is None and ks:
    with open(ks[0]) as fh:
        rows = [r for r in csv.DictReader(fh) if "march_kernel<" in r["Name"]]
    if rows:
        kname = max(rows, key=lambda r: int(r["Calls"]))["Name"].split("(")[0].replace("void ", "", 1)
fetch_kb, write_kb = (mean(kname, "FETCH_SIZE"), mean(kname, "WRITE_SIZE")) if kname else (None, None)
if fetch_kb is None:
    print("no PMC dispatches of", kname)
else:
    traffic = 2 * 1024 * fetch_kb + 1024 * (write_kb or 0.0)
    extra = {c: mean(kname, c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU",
                                          "SQ_INSTS_SMEM", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                                          "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
                                          "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_ACTIVE_INST_VALU",
                                          "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU_TRANS_F32",
                                          "SQ_THREAD_CYCLES_VALU", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum",
                                          "GRBM_GUI_ACTIVE")}
    ndisp = {c: len([1 for k, cs in vals.items() if k.split("(")[0].replace("void ", "", 1) == kname
                     for _ in cs.get(c, {})]) for c in ("FETCH_SIZE", "SQ_INSTS_VALU")}
    with open(os.path.join(out, "traffic.json"), "w") as fh:
        json.dump({"workload": workload, "kernel": kname, "dispatches": ndisp,
                   "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
                   "bytes_per_launch": traffic,
                   "valu_insts_per_launch": extra["SQ_INSTS_VALU"],
                   "counters_per_launch": {k: v for k, v in extra.items() if v is not None},
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py's production "
                             "frames (the timed instantiation, matched by exact name); read bytes = "
                             "2 x 1024 x FETCH_SIZE (gfx950 64 B tally per 128 B request)"}, fh, indent=1)
    print("kernel", kname, "traffic bytes/launch", traffic)
print("\n".join(lines[:80]))
