#!/bin/bash
# round-3 pass bj: same-box A/B of the final build against 12-sample chunks per depth lane
# (VR_CHUNK_PER_LANE=12, smaller boxes: more of them whole) and 6 KiB slots (VR_LDS_CAP=1536)
RUN=${1:-r3bj}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "tree=VR_X=1" "cpl12=VR_LIB_PATH=build_ab/libvrhip_cpl12.so" \
  "c1536=VR_LIB_PATH=build_ab/libvrhip_c1536.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); L=d['line']; r[d['ab']].append((L['ms_per_step'], L['roofline']['kernel_ms'], L.get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
"
