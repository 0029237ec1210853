cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh && mkdir -p gpurun_out/r34 &&
PMC_GROUPS="FETCH_SIZE;TCC_HIT_sum,TCC_MISS_sum,TCC_REQ_sum" bash tools/pmc.sh gpurun_out/r34/pmc && run wg4 && run wg4b && cat gpurun_out/ab_summary.txt
