#!/bin/bash
# round-3 pass s: P = 8 part times (bench.py --sim-parts 8) by the column block of the partition
RUN=${1:-r3s}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for r in 1 2; do for bc in 16 8 4 32; do
  echo -n "{\"bc\": $bc, \"round\": $r, \"line\": " >> gpurun_out/$RUN/ab.jsonl
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipelined-streams 0 --sim-parts 8 --block-cols $bc 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
  echo "}" >> gpurun_out/$RUN/ab.jsonl
done; done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); s=d['line']['sim_parts_kernel_ms']; print(d['bc'], d['round'], d['line']['roofline']['kernel_ms'], s['max'], round(sum(s['per_part'])/8,3), s['est_speedup'])
"
