#!/usr/bin/env python3
"""tools/parity_summary.py LOG... OUT.json -- collect the PARITY lines that tests/test_full_size.py
prints (one JSON object per checked image) from GPU test logs into one committed summary."""
import json
import sys

rows = {}
for path in sys.argv[1:-1]:
    for line in open(path, errors="replace"):
        if "PARITY {" in line:
            d = json.loads(line[line.index("{"):])
            rows[d["what"]] = d
with open(sys.argv[-1], "w") as f:
    json.dump(list(rows.values()), f, indent=1)
print(len(rows), "images ->", sys.argv[-1])
