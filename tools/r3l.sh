#!/bin/bash
# round-3 pass l: 7 waves per SIMD (72-VGPR cap, 5.5 KiB slots so that 7 workgroups fit the LDS)
# against the default 6 (80 VGPRs, 6.5 KiB) -- metric frame and the P = 8 part
RUN=${1:-r3l}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for r in 1 2; do
  for spec in "tree|VR_X=1" "eu7|VR_LIB_PATH=build_ab/libvrhip_eu7.so"; do
    IFS='|' read name envs <<< "$spec"
    echo -n "{\"ab\": \"$name\", \"round\": $r, \"line\": " >> gpurun_out/$RUN/ab.jsonl
    env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --pipelined-streams 0 --sim-parts 8 \
      2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
    echo "}" >> gpurun_out/$RUN/ab.jsonl
  done
done &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append((d['line']['roofline']['kernel_ms'], d['line']['sim_parts_kernel_ms']['max']))
for k,v in r.items(): print(k, v)
"
