cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/t27.log 2>&1 ; tail -1 gpurun_out/t27.log;
run wg1 && run wg4 VR_LIB_PATH=build_ab/libvrhip_wg4.so && run wg2 VR_LIB_PATH=build_ab/libvrhip_wg2.so && run wg1b && run wg4b VR_LIB_PATH=build_ab/libvrhip_wg4.so && cat gpurun_out/ab_summary.txt
