#!/bin/bash
# round-3 pass af: host-side single-voxel reflection constant (tree) vs the per-sample load (head)
RUN=${1:-r3af}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/t.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/t.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/t.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "tree=VR_X=1" "head=VR_LIB_PATH=build_ab/libvrhip_head.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
"
