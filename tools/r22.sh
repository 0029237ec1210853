cd $GRAFT_REPO_ROOT && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r22 && rm -f gpurun_out/ab_summary.txt && source tools/ab_bench.sh &&
for v in base ab1 ab2 ab4 ab16; do
  if [ $v = base ]; then L=""; else L="VR_LIB_PATH=build_ab/libvrhip_$v.so"; fi
  env $L timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 -d gpurun_out/r22/$v -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r22/$v.log 2>&1 || exit 1
  run $v $L || exit 1
done; cat gpurun_out/ab_summary.txt
