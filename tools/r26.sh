cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variants or c1 or hg_two" > gpurun_out/t26.log 2>&1 ; tail -1 gpurun_out/t26.log;
run queue && run static VR_STATIC=1 && run prev VR_LIB_PATH=build_ab/libvrhip_prev.so && run queue2 && run static2 VR_STATIC=1 && run prev2 VR_LIB_PATH=build_ab/libvrhip_prev.so && cat gpurun_out/ab_summary.txt
