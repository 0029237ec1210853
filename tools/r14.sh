cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
run base && run a4 VR_LIB_PATH=build_ab/libvrhip_a4.so && run c16 VR_LIB_PATH=build_ab/libvrhip_c16.so && run c64a5 VR_LIB_PATH=build_ab/libvrhip_c64a5.so && run base2 && cat gpurun_out/ab_summary.txt
