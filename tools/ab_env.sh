#!/bin/bash
# tools/ab_env.sh ROUNDS "ENV1" "ENV2" ... -- on the GPU box: interleaved bench.py kernel times of the
# in-tree library under environment settings ("-" = none), ROUNDS rounds each.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do i=0; for e in "$@"; do i=$((i+1))
  if [ "$e" = "-" ]; then envs=""; else envs="$e"; fi
  env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --pipelined-streams 0 \
    > gpurun_out/ab/env$i.$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab/env$i.$r.json').read().strip().splitlines()[-1]);print('$e', $r, d['roofline']['kernel_ms'])" | tee -a gpurun_out/ab/summary.txt
done; done
