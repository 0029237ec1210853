#!/bin/bash
# round-3 pass be: per-rank share of a P-way image partition on one GPU (bench.py --sim-parts P) with
# the round-3 kernel -- P = 2, 4, 8 at their default depth lanes, and P = 8 at K = 2 -- two rounds
RUN=${1:-r3be}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for P in 2 4 8; do
  BENCH_ARGS="--sim-parts $P" bash tools/ab_env_r3.sh gpurun_out/$RUN/p$P.jsonl 2 "p$P=VR_X=1" || exit 1
done &&
BENCH_ARGS="--sim-parts 8" bash tools/ab_env_r3.sh gpurun_out/$RUN/p8k2.jsonl 2 "p8k2=VR_DEPTH_LANES=2" &&
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/$RUN/p*.jsonl')):
    for l in open(f):
        d=json.loads(l); L=d['line']; s=L['sim_parts_kernel_ms']
        print(d['ab'], L['roofline']['kernel_ms'], 'parts', [round(x,3) for x in s['per_part']], 'max', s['max'], 'est', s['est_speedup'])
"
