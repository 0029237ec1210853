#!/bin/bash
# tools/final_r2.sh -- round-2 closing measurements on the GPU box: tools/measure.sh (GPU tests,
# bench line, kernel-trace stats, PMC passes) then the per-part times of P-way partitions.
cd "$GRAFT_REPO_ROOT" &&
bash tools/measure.sh r2f &&
for p in 2 4 8; do
  timeout -k 10 300 python bench.py --sim-parts $p --steps 5 --warmup 2 --no-cpu-baseline --pipelined-streams 0 \
    > gpurun_out/r2f/simparts_$p.json 2> gpurun_out/r2f/simparts_$p.err || exit 1
done
