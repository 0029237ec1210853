#!/bin/bash
# round-3 pass m: sort-last cost on one MI355X (tools/sort_last_bench.py, one rank): the whole
# volume as one slab with the frame as 1 / 4 column tiles, and the volume as 4 chained slabs; the
# plain render beside it (bench.py kernel time)
RUN=${1:-r3m}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --pipelined-streams 0 > gpurun_out/$RUN/plain.json 2>/dev/null &&
for a in "--tiles 1" "--tiles 4 --streams 2" "--tiles 4 --streams 2 --check" "--tiles 1 --slabs 4 --check"; do
  timeout -k 10 300 python tools/sort_last_bench.py $a >> gpurun_out/$RUN/sl.jsonl 2> gpurun_out/$RUN/sl.err || exit 1
done &&
VR_DEPTH_LANES=2 timeout -k 10 300 python tools/sort_last_bench.py --tiles 4 --streams 2 >> gpurun_out/$RUN/sl.jsonl 2>> gpurun_out/$RUN/sl.err &&
python3 -c "
import json
p=json.load(open('gpurun_out/$RUN/plain.json'))['roofline']['kernel_ms']
print('plain kernel ms', p)
for l in open('gpurun_out/$RUN/sl.jsonl'):
    d=json.loads(l); print(d.get('tiles'), d.get('streams'), d.get('slabs_one_process'), d.get('depth_lanes_env'), d.get('ms_per_frame'), round(d.get('ms_per_frame')/p,3), d.get('check'))
"
