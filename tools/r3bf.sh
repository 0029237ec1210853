#!/bin/bash
# round-3 pass bf: GPU tests on the tree (adaptive first chunk length, VR_ADAPTIVE_S), a same-box A/B
# against 04d5f8b, then the P-way partition shares (tools/r3be.sh)
RUN=${1:-r3bf}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/tests.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "head=VR_LIB_PATH=build_ab/libvrhip_head.so" "tree=VR_X=1" "pk=VR_LIB_PATH=build_ab/libvrhip_pk.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); L=d['line']; r[d['ab']].append((L['ms_per_step'], L['roofline']['kernel_ms'], L.get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
" && bash tools/r3be.sh ${RUN}_parts
