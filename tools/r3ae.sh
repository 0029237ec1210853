#!/bin/bash
# round-3 pass ae: skipping the group compositing of all-zero wave samples (tree) vs always (nozc)
RUN=${1:-r3ae}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/t.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/t.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/t.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "tree=VR_X=1" "nozc=VR_LIB_PATH=build_ab/libvrhip_nozc.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
"
