#!/bin/bash
# round-3 pass w: P = 2 and P = 4 part times (bench.py --sim-parts) by depth lanes and schedule
RUN=${1:-r3w}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for P in 2 4; do for e in "VR_X=1" "VR_DEPTH_LANES=2" "VR_DEPTH_LANES=4" "VR_SCHED=0" "VR_SCHED=1"; do
  echo -n "{\"P\": $P, \"env\": \"$e\", \"line\": " >> gpurun_out/$RUN/ab.jsonl
  env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipelined-streams 0 --sim-parts $P 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
  echo "}" >> gpurun_out/$RUN/ab.jsonl
done; done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); s=d['line']['sim_parts_kernel_ms']; print(d['P'], d['env'], d['line']['roofline']['kernel_ms'], s['per_part'], s['est_speedup'])
"
