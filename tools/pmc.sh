#!/bin/bash
# tools/pmc.sh OUTDIR [bench args...] -- rocprofv3 PMC passes over bench.py (run ON the GPU box).
# One counter group per pass (gfx950 slot limits, MI355X_MICROARCH.md "rocprofv3 PMC slots");
# no trace domains are combined with --pmc.

OUT=$1; shift
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
# --warmup 1: the first full frame of a shape is the timed-schedule instantiation (SCHED 2); the
# production frames that bench.py times come after it
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --pipelined-streams 0 $*"
i=0
PMCG=${PMC_GROUPS:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SMEM;SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE;FETCH_SIZE;TCC_HIT_sum,TCC_MISS_sum,TCC_REQ_sum;GRBM_GUI_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_THREAD_CYCLES_VALU"}
IFS=';' read -ra GRPS <<< "$PMCG"
for g in "${GRPS[@]}"; do
  i=$((i+1))
  grp=${g//,/ }
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$OUT/pass$i" -o pmc --output-format csv -- python bench.py $ARGS > "$OUT/pass$i.log" 2>&1 || exit 1
done
