#!/bin/bash
# tools/ab_sweep.sh OUT "LIB..." "K:P ..." [bench args] -- on the GPU box: bench.py per library
# variant (default = the in-tree build, else build_ab/libvrhip_<name>.so) and per depth-lane count
# K / simulated partition count P; one JSON per run under gpurun_out/OUT.
OUT=$1; LIBS=$2; KPS=$3; shift 3
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$OUT || exit 1
for LIB in $LIBS; do
  if [ "$LIB" = default ]; then unset VR_LIB_PATH; else export VR_LIB_PATH=build_ab/libvrhip_$LIB.so; fi
  for KP in $KPS; do
    K=${KP%:*}; P=${KP#*:}
    VR_DEPTH_LANES=$K timeout -k 10 200 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --sim-parts $P "$@" \
      > gpurun_out/$OUT/${LIB}_k${K}p$P.json 2> gpurun_out/$OUT/${LIB}_k${K}p$P.err || exit 1
  done
done
