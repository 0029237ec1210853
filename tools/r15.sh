cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t15.log 2>&1 ; tail -1 gpurun_out/t15.log;
run part && run nopart VR_LIB_PATH=build_ab/libvrhip_nopart.so && run pa4 VR_LIB_PATH=build_ab/libvrhip_pa4.so && run pa2 VR_LIB_PATH=build_ab/libvrhip_pa2.so && run part2 && cat gpurun_out/ab_summary.txt
