cd $GRAFT_REPO_ROOT && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r16 &&
for v in base ab1 ab2 ab4 ab8 ab16; do
  if [ $v = base ]; then L=""; else L="VR_LIB_PATH=build_ab/libvrhip_$v.so"; fi
  env $L timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 -d gpurun_out/r16/$v -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r16/$v.log 2>&1 || exit 1
done
