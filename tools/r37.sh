cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/t37.log 2>&1 ; tail -1 gpurun_out/t37.log;
run grp && run prev VR_LIB_PATH=build_ab/libvrhip_prev.so && run grp2 && run prev2 VR_LIB_PATH=build_ab/libvrhip_prev.so && cat gpurun_out/ab_summary.txt
