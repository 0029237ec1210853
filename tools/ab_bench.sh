#!/bin/bash
# A/B timing of library variants / env switches on the GPU box (3 frames each, no CPU baseline)
cd "$GRAFT_REPO_ROOT"
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || return 1;
        python -c "import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['ms_per_step'], d['value'])" >> gpurun_out/ab_summary.txt; }
