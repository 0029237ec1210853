#!/bin/bash
# round-3 pass ag: the slab kernel at 5 waves per SIMD (VR_SLAB_MIN_EU=5: no VGPR cap of 80, fewer
# spills) vs 6 -- one tile and 4 tiles on one rank (tools/sort_last_bench.py)
RUN=${1:-r3ag}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for r in 1 2; do for spec in "tree|VR_X=1" "slab5|VR_LIB_PATH=build_ab/libvrhip_slab5.so"; do
  IFS='|' read name envs <<< "$spec"
  for a in "--tiles 1" "--tiles 4 --streams 2"; do
    echo -n "{\"ab\": \"$name\", \"args\": \"$a\", \"line\": " >> gpurun_out/$RUN/ab.jsonl
    env $envs timeout -k 10 300 python tools/sort_last_bench.py $a 2>/dev/null | tail -1 | tr -d '\n' >> gpurun_out/$RUN/ab.jsonl || exit 1
    echo "}" >> gpurun_out/$RUN/ab.jsonl
  done
done; done &&
python3 -c "
import json
for l in open('gpurun_out/$RUN/ab.jsonl'):
    d=json.loads(l); print(d['ab'], d['args'], d['line']['ms_per_frame'])
"
