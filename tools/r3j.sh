#!/bin/bash
# round-3 pass j: P = 8 part time (bench.py --sim-parts 8) against the raised-priority block count of
# the scheduled short launch (VR_PRIO_BLOCKS; default = wave slots / 4)
RUN=${1:-r3j}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for r in 1 2; do for pb in def 0 64 128 256 512; do
  if [ $pb = def ]; then E="VR_X=1"; else E="VR_PRIO_BLOCKS=$pb"; fi
  echo -n "{\"pb\": \"$pb\", \"round\": $r, \"line\": " >> gpurun_out/$RUN/ab.jsonl
  env $E timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipelined-streams 0 --sim-parts 8 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
  echo "}" >> gpurun_out/$RUN/ab.jsonl
done; done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); s=d['line']['sim_parts_kernel_ms']; print(d['pb'], d['round'], s['max'], s['est_speedup'], s['per_part'])
"
