#!/bin/bash
# round-3 pass x: P = 2 / 4 part times by the column block of the partition
RUN=${1:-r3x}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for spec in "2 16" "2 32" "2 64" "2 128" "4 16" "4 32" "4 64"; do
  set -- $spec
  echo -n "{\"P\": $1, \"bc\": $2, \"line\": " >> gpurun_out/$RUN/ab.jsonl
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipelined-streams 0 --sim-parts $1 --block-cols $2 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
  echo "}" >> gpurun_out/$RUN/ab.jsonl
done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); s=d['line']['sim_parts_kernel_ms']; print(d['P'], d['bc'], d['line']['roofline']['kernel_ms'], s['per_part'], s['est_speedup'])
"
