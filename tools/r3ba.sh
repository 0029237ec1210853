#!/bin/bash
# round-3 pass ba: occupancy profile of the metric frame (block start + duration of the timed
# row-major frame, tools/tail_profile.py) and a same-box A/B of the full-frame tail: forced
# heavy-first order (VR_SCHED_TAIL_PCT=0) at heavy thresholds 1/8, 1/2, 1/32 of the longest block,
# and non-temporal staging loads (build_ab/libvrhip_nt.so)
RUN=${1:-r3ba}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
VR_SCHED_DUMP=gpurun_out/$RUN/dump VR_SCHED_REMEASURE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 0 \
  --no-cpu-baseline --pipelined-streams 0 > gpurun_out/$RUN/dump.json 2>&1 &&
python3 tools/tail_profile.py gpurun_out/$RUN/dump > gpurun_out/$RUN/tail.jsonl &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "def=VR_X=1" "heavy8=VR_SCHED_TAIL_PCT=0" \
  "heavy2=VR_SCHED_TAIL_PCT=0 VR_SCHED_HEAVY_DIV=2" "heavy32=VR_SCHED_TAIL_PCT=0 VR_SCHED_HEAVY_DIV=32" \
  "nt=VR_LIB_PATH=build_ab/libvrhip_nt.so" &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append((d['line']['ms_per_step'], d['line']['roofline']['kernel_ms']))
for k,v in r.items(): print(k, v)
" && cut -c1-400 gpurun_out/$RUN/tail.jsonl
