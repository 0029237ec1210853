cd $GRAFT_REPO_ROOT && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
for v in base u8 u16; do
  if [ $v = base ]; then L=""; else L="VR_LIB_PATH=build_ab/libvrhip_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --lights 0 > gpurun_out/l0_$v.log 2>&1 || exit 1
  run $v $L || exit 1
done; cat gpurun_out/ab_summary.txt; for v in base u8 u16; do tail -c 300 gpurun_out/l0_$v.log | grep -o '"ms_per_step": [0-9.]*' ; done
