#!/bin/bash
# round-3 pass v: LUT lookups from the yz-quad copy (A/B build, VR_LUT_QUAD=1) vs the z-paired copy
RUN=${1:-r3v}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ VR_LIB_PATH=build_ab/libvrhip_quad.so VR_LUT_QUAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "variants or exact_shading or hg_two" --timeout 200 --timeout-method thread > gpurun_out/$RUN/t.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/t.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/t.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "zpair=VR_X=1" "quad=VR_LIB_PATH=build_ab/libvrhip_quad.so VR_LUT_QUAD=1" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
"
