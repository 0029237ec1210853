#!/bin/bash
# round-3 measurement pass: GPU tests, the default bench line, rocprofv3 kernel trace, PMC passes
# on the timed kernel (FETCH/WRITE, L2, SQ issue/wait, VALU/trans, L1/TA)
RUN=${1:-r3z}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -le 1 ]; } &&
timeout -k 10 400 python bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err &&
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$RUN/kt -o kt --output-format csv -- \
   python bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipelined-streams 0 > gpurun_out/$RUN/kt.log 2>&1) &&
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum,TCC_MISS_sum,TCC_REQ_sum;SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SMEM;SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE;GRBM_GUI_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_THREAD_CYCLES_VALU;TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCP_TCC_READ_REQ_LATENCY_sum,TCP_TCP_LATENCY_sum;TA_TOTAL_WAVEFRONTS_sum,TA_FLAT_READ_WAVEFRONTS_sum" \
  bash tools/pmc.sh gpurun_out/$RUN/pmc &&
grep -E "passed|failed" gpurun_out/$RUN/tests.log | tail -1 && cut -c1-300 gpurun_out/$RUN/bench.json
