#!/bin/bash
# round-3 pass y: short-launch schedule heavy-first + row-major (VR_SCHED_SHORT_DIV) vs longest-first
RUN=${1:-r3y}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for P in 2 4 8; do for e in "VR_X=1" "VR_SCHED_SHORT_DIV=2" "VR_SCHED_SHORT_DIV=4" "VR_SCHED_SHORT_DIV=8"; do
  echo -n "{\"P\": $P, \"env\": \"$e\", \"line\": " >> gpurun_out/$RUN/ab.jsonl
  env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipelined-streams 0 --sim-parts $P 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
  echo "}" >> gpurun_out/$RUN/ab.jsonl
done; done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); s=d['line']['sim_parts_kernel_ms']; print(d['P'], d['env'], d['line']['roofline']['kernel_ms'], max(s['per_part']), s['est_speedup'])
"
