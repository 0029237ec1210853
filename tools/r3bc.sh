#!/bin/bash
# round-3 pass bc: the whole-box rule (tame, staged, not partial, not clamped at a volume face) checked
# by the diagnostic build over every GPU test and the metric frame (VR_CHECK_WHOLE=1: counts samples
# the per-sample slot test would have sent elsewhere, prints the first ones), the GPU tests on the tree,
# and a same-box A/B of the HEAD library and the tree
RUN=${1:-r3bc}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ VR_LIB_PATH=build_ab/libvrhip_check.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 200 \
    --timeout-method thread > gpurun_out/$RUN/check.log 2>&1; echo "check rc=$?" >> gpurun_out/$RUN/check.log; } &&
VR_LIB_PATH=build_ab/libvrhip_check.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --pipelined-streams 0 > gpurun_out/$RUN/check_bench.log 2>&1 &&
echo "whole-box violation lines: $(cat gpurun_out/$RUN/check.log gpurun_out/$RUN/check_bench.log | grep -c VR_CHECK_WHOLE)" &&
grep -m 12 VR_CHECK_WHOLE gpurun_out/$RUN/check.log gpurun_out/$RUN/check_bench.log; tail -2 gpurun_out/$RUN/check.log &&
{ timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/tests.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "head=VR_LIB_PATH=build_ab/libvrhip_head.so" "tree=VR_X=1" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append((d['line']['ms_per_step'], d['line']['roofline']['kernel_ms'], d['line'].get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
"
