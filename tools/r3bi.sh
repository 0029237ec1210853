#!/bin/bash
# round-3 pass bi: same-box A/B of the final build (5 waves per SIMD) against 4 waves per SIMD
# (dropped: at 84 VGPRs it builds the same kernel) and against 8 staging loads in flight per lane (VR_STAGE_UNROLL=8)
RUN=${1:-r3bi}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "tree=VR_X=1" \
  "u8=VR_LIB_PATH=build_ab/libvrhip_u8.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); L=d['line']; r[d['ab']].append((L['ms_per_step'], L['roofline']['kernel_ms'], L.get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
"
