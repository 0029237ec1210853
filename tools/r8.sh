cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
timeout -k 10 120 python tools/variant_dump.py > gpurun_out/vd.log 2>&1 &&
run base && run c2560 VR_LIB_PATH=build_ab/libvrhip_c2560.so && run c3072 VR_LIB_PATH=build_ab/libvrhip_c3072.so &&
run c4096 VR_LIB_PATH=build_ab/libvrhip_c4096.so && run c2560a4 VR_LIB_PATH=build_ab/libvrhip_c2560a4.so &&
run c3072a4 VR_LIB_PATH=build_ab/libvrhip_c3072a4.so && run c4096a4 VR_LIB_PATH=build_ab/libvrhip_c4096a4.so && cat gpurun_out/ab_summary.txt
