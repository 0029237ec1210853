cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/t29.log 2>&1 ; tail -1 gpurun_out/t29.log;
run pipe && run prev VR_LIB_PATH=build_ab/libvrhip_prev.so && run pipe2 && run prev2 VR_LIB_PATH=build_ab/libvrhip_prev.so &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --lights 0 > gpurun_out/pl0.log 2>&1 &&
VR_LIB_PATH=build_ab/libvrhip_prev.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --lights 0 > gpurun_out/ql0.log 2>&1 && cat gpurun_out/ab_summary.txt
