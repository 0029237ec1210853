cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 300 tools/microbench/mathcheck > gpurun_out/mathcheck.log 2>&1 ;
cat gpurun_out/mathcheck.log;
timeout -k 10 120 python tools/variant_dump.py > gpurun_out/vd.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t10.log 2>&1 ;
tail -3 gpurun_out/t10.log;
run pair && run nopair VR_NO_PAIR=1 && cat gpurun_out/ab_summary.txt
