#!/bin/bash
# round-3 pass d: same-box A/B of sample-path micro-optimizations (libraries under build_ab/) and of
# the row-ordered full-frame schedule (in-tree library)
RUN=${1:-r3d}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 2 "base=VR_LIB_PATH=build_ab/libvrhip_base.so" \
  "abc=VR_LIB_PATH=build_ab/libvrhip_abc.so" "abcd=VR_LIB_PATH=build_ab/libvrhip_abcd.so" \
  "rows=VR_SCHED_ROWS=1" "tree=VR_X=1" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
"
