#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-kernel counter values (sum over dispatches / dispatches)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
kfilter = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            if kfilter not in k:
                continue
            vals[k][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
for k, cs in vals.items():
    print(k[:100])
    for c, lst in sorted(cs.items()):
        per = defaultdict(float)
        for d, v in lst:
            per[d] += v
        avg = sum(per.values()) / len(per)
        print(f"  {c:40s} {avg:.6g}  (dispatches {len(per)})")
