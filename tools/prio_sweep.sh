#!/bin/bash
# tools/prio_sweep.sh OUT "PRIO..." "K:P ..." -- scheduled-launch wave priority sweep (GPU box)
OUT=$1; PRIOS=$2; KPS=$3
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$OUT || exit 1
for PR in $PRIOS; do for KP in $KPS; do
  K=${KP%:*}; P=${KP#*:}
  VR_PRIO_BLOCKS=$PR VR_DEPTH_LANES=$K timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --sim-parts $P > gpurun_out/$OUT/pr${PR}_k${K}p$P.json 2> gpurun_out/$OUT/pr${PR}_k${K}p$P.err || exit 1
done; done
