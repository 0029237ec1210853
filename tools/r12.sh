cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t12.log 2>&1 ; tail -3 gpurun_out/t12.log;
run base && run even VR_LIB_PATH=build_ab/libvrhip_even.so && run nochk VR_LIB_PATH=build_ab/libvrhip_nochk.so && run a4 VR_LIB_PATH=build_ab/libvrhip_a4.so && run base2 && cat gpurun_out/ab_summary.txt
