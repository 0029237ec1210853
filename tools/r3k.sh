#!/bin/bash
# round-3 pass k: where the metric kernel's time goes -- diagnostic ablation builds (wrong images):
# a1 no LUT fetch, a2 no angles (acospi), a3 both, a4 no gradient taps; and the light count
RUN=${1:-r3k}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for r in 1 2; do
  for spec in "tree|VR_X=1|" "a1|VR_LIB_PATH=build_ab/libvrhip_a1.so|" "a2|VR_LIB_PATH=build_ab/libvrhip_a2.so|" \
              "a3|VR_LIB_PATH=build_ab/libvrhip_a3.so|" "a4|VR_LIB_PATH=build_ab/libvrhip_a4.so|" \
              "l0|VR_X=1|--lights 0" "l1|VR_X=1|--lights 1"; do
    IFS='|' read name envs args <<< "$spec"
    echo -n "{\"ab\": \"$name\", \"round\": $r, \"line\": " >> gpurun_out/$RUN/ab.jsonl
    env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --pipelined-streams 0 $args \
      2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
    echo "}" >> gpurun_out/$RUN/ab.jsonl
  done
done &&
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); r[d['ab']].append(d['line']['roofline']['kernel_ms'])
for k,v in r.items(): print(k, v, 'min', min(v))
"
