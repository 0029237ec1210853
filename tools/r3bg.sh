#!/bin/bash
# round-3 pass bg: occupancy vs slot size after the whole-box kernel -- same-box A/B of the tree
# (6.5 KiB slots, 6 waves per SIMD), 5 waves per SIMD with the same slots (VR_MARCH_MIN_EU=5: 96
# VGPRs, no spills), and 5 waves with 7.9 KiB slots (VR_LDS_CAP=2016: 5 workgroups per CU by LDS too)
RUN=${1:-r3bg}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "tree=VR_X=1" "eu5=VR_LIB_PATH=build_ab/libvrhip_eu5.so" \
  "c2016=VR_LIB_PATH=build_ab/libvrhip_c2016.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); L=d['line']; r[d['ab']].append((L['ms_per_step'], L['roofline']['kernel_ms'], L.get('image_sha256','')[:12]))
for k,v in r.items(): print(k, v)
"
