#!/bin/bash
# round-3 pass bb: GPU tests on the tree (whole-box slot test skip, zero-fill compositing, one exit
# test per depth-lane step, DPP group_any), the whole-box invariant checked by the diagnostic build
# (VR_CHECK_WHOLE=1: printf on any sample whose taps leave a whole box) over the parity tests and the
# metric frame, then a same-box A/B: HEAD library / tree / tree with the row-shift order (VR_SCHED_SHIFT)
RUN=${1:-r3bb}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/tests.log &&
{ VR_LIB_PATH=build_ab/libvrhip_check.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py \
    -q -s --timeout 200 --timeout-method thread > gpurun_out/$RUN/check.log 2>&1; echo "check rc=$?" >> gpurun_out/$RUN/check.log; } &&
VR_LIB_PATH=build_ab/libvrhip_check.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --pipelined-streams 0 > gpurun_out/$RUN/check_bench.log 2>&1 &&
echo "whole-box violations: $(cat gpurun_out/$RUN/check.log gpurun_out/$RUN/check_bench.log | grep -c VR_CHECK_WHOLE)" &&
tail -1 gpurun_out/$RUN/check.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "head=VR_LIB_PATH=build_ab/libvrhip_head.so" "tree=VR_X=1" \
  "shift10=VR_SCHED_SHIFT=10" "shift20=VR_SCHED_SHIFT=20" "shift30=VR_SCHED_SHIFT=30" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append((d['line']['ms_per_step'], d['line']['roofline']['kernel_ms'], d['line'].get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
"
