#!/bin/bash
# round-3 pass e: same-box A/B of the TAME sample path (in-tree) against the previous commit's
# library and a 5-waves/EU variant, the exp rounding microbench, then the GPU test suite with the
# full-size parity lines (-s) captured for tools/parity_summary.py
RUN=${1:-r3e}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 2 "abcd=VR_LIB_PATH=build_ab/libvrhip_abcd.so" \
  "tree=VR_X=1" "eu5=VR_LIB_PATH=build_ab/libvrhip_eu5.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
" > gpurun_out/$RUN/ab.txt && cat gpurun_out/$RUN/ab.txt &&
timeout -k 10 120 tools/microbench/exp_check > gpurun_out/$RUN/exp_check.txt 2>&1 &&
{ timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -le 1 ]; } &&
grep -E "passed|failed" gpurun_out/$RUN/tests.log | tail -3
