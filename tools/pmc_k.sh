#!/bin/bash
# tools/pmc_k.sh OUT -- one rocprofv3 PMC pass per depth-lane count K over one bench frame (GPU box)
OUT=$1
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$OUT
for K in ${KS:-2 4 8}; do
  VR_DEPTH_LANES=$K timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD \
    -d gpurun_out/$OUT/k$K -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/$OUT/k$K.log 2>&1 || exit 1
done
