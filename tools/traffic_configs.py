#!/usr/bin/env python3
"""tools/profile_summary.py --configs OUT PMC_DIR:BENCH_JSON[:NAME] ... (see profile_summary.py).

Per configuration: the bench line of the pass (bench.py at that config, its roofline.kernel = the
timed instantiation) and the rocprofv3 PMC passes over the same bench arguments (tools/pmc.sh).
HBM bytes per launch = 2 x 1024 x FETCH_SIZE + 1024 x WRITE_SIZE (gfx950: FETCH_SIZE tallies 64 B
per 128 B request, MI355X_MICROARCH.md).  Writes OUT/traffic.json ({"entries": [...]}) and
OUT/configs.json (each line with roofline.traffic / valu / binding filled in from its entry)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
VALU_ISSUE_PER_S = 1024 * 2.4e9 / 2
COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVES",
            "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
            "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU_TRANS_F32", "SQ_THREAD_CYCLES_VALU", "TCC_HIT_sum", "TCC_MISS_sum",
            "TCC_REQ_sum", "GRBM_GUI_ACTIVE")
METHOD = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py's production frames (the timed "
          "instantiation, matched by exact name); read bytes = 2 x 1024 x FETCH_SIZE (gfx950 64 B tally per "
          "128 B request)")


def last_json(path):
    with open(path) as fh:
        return json.loads(fh.read().strip().splitlines()[-1])


def counters(pmc_dir):
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(pmc_dir, "pass*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[row["Kernel_Name"]][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return vals


def mean(vals, kname, counter):
    xs = [v for k, cs in vals.items() if k.split("(")[0].replace("void ", "", 1) == kname
          for v in cs.get(counter, {}).values()]
    return sum(xs) / len(xs) if xs else None


def entry(pmc_dir, bench_json, name):
    line = last_json(bench_json)
    kname = line["roofline"]["kernel"]
    vals = counters(pmc_dir)
    fetch_kb, write_kb = mean(vals, kname, "FETCH_SIZE"), mean(vals, kname, "WRITE_SIZE")
    if fetch_kb is None:
        raise SystemExit(f"{name}: no PMC dispatches of {kname} in {pmc_dir}")
    extra = {c: mean(vals, kname, c) for c in COUNTERS}
    e = {"name": name, "workload": line["config"]["workload"], "kernel": kname,
         "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
         "bytes_per_launch": 2 * 1024 * fetch_kb + 1024 * (write_kb or 0.0),
         "valu_insts_per_launch": extra["SQ_INSTS_VALU"],
         "counters_per_launch": {k: v for k, v in extra.items() if v is not None}, "method": METHOD}
    return e, line


def attach(line, e, src):
    """The bench line with roofline.traffic / valu / binding from its entry (as bench.py does)."""
    rf = line["roofline"]
    t = rf["kernel_ms"] / 1e3
    rf["traffic"] = e["bytes_per_launch"]
    rf["traffic_source"] = src
    vi = e["valu_insts_per_launch"]
    if vi:
        rf["valu"] = {"insts_per_launch": vi, "achieved": round(vi / t / 1e9, 2),
                      "peak": round(VALU_ISSUE_PER_S / 1e9, 1), "unit": "G wave64-instr/s",
                      "frac": round(vi / t / VALU_ISSUE_PER_S, 4)}
    fr = rf["fetched"]["frac"] if "fetched" in rf else rf["frac"]  # (round 6: frac is the fetched fraction)
    cands = {"fetched": fr, "hbm_traffic": round(rf["traffic"] / t / 1e9 / HBM_PEAK_GBS, 4)}
    if vi:
        cands["valu"] = rf["valu"]["frac"]
    name = max(cands, key=cands.get)
    rf["binding"] = {"roof": name, "frac": cands[name], "candidates": cands}
    c = e["counters_per_launch"]
    if c.get("SQ_WAVE_CYCLES") and c.get("SQ_WAIT_INST_ANY"):
        rf["binding"]["wait_inst_any_frac_of_wave_cycles"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    if c.get("TCC_HIT_sum") and c.get("TCC_REQ_sum"):
        rf["binding"]["l2_hit"] = round(c["TCC_HIT_sum"] / c["TCC_REQ_sum"], 4)
    return line


def main():
    out = sys.argv[2]
    os.makedirs(out, exist_ok=True)
    entries, lines = [], {}
    for spec in sys.argv[3:]:
        parts = spec.split(":")
        pmc_dir, bench_json = parts[0], parts[1]
        name = parts[2] if len(parts) > 2 else os.path.basename(pmc_dir)
        e, line = entry(pmc_dir, bench_json, name)
        entries.append(e)
        lines[name] = attach(line, e, os.path.join(out, "traffic.json"))
        b = lines[name]["roofline"]["binding"]
        print(f"{name:8s} {line['ms_per_step']:9.3f} ms  traffic {e['bytes_per_launch'] / 1e9:8.2f} GB  "
              f"binding {b['roof']} {b['frac']}  {b['candidates']}")
    with open(os.path.join(out, "traffic.json"), "w") as fh:
        json.dump({"entries": entries}, fh, indent=1)
    with open(os.path.join(out, "configs.json"), "w") as fh:
        json.dump(lines, fh, indent=1)


if __name__ == "__main__":
    main()
