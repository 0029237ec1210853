#!/bin/bash
# tools/configs_r2.sh (round 3: gpurun_out/cfg3) -- the other BASELINE configurations on one GPU (diagnostics, not bench lines)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/cfg3 &&
B="python bench.py --no-cpu-baseline --pipelined-streams 0 --steps 3 --warmup 1" &&
timeout -k 10 300 $B --width 1024 --height 768 > gpurun_out/cfg3/c2.json 2> gpurun_out/cfg3/c2.err &&
timeout -k 10 300 $B --gradient lookup > gpurun_out/cfg3/c3.json 2> gpurun_out/cfg3/c3.err &&
timeout -k 10 600 $B --volume 2048 --width 4096 --height 4096 > gpurun_out/cfg3/c5.json 2> gpurun_out/cfg3/c5.err
