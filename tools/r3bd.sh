#!/bin/bash
# round-3 pass bd: GPU tests on the tree (the depth-lane sample loop compiled separately for whole
# chunks), then a same-box A/B of HEAD-of-round (943d9bb) / e6ebbd5 / the tree: full frames, and the
# P = 8 part (bench.py --sim-parts 8)
RUN=${1:-r3bd}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -eq 0 ]; } && tail -2 gpurun_out/$RUN/tests.log &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab.jsonl 3 "head=VR_LIB_PATH=build_ab/libvrhip_head.so" \
  "e6=VR_LIB_PATH=build_ab/libvrhip_e6.so" "tree=VR_X=1" &&
BENCH_ARGS="--sim-parts 8" bash tools/ab_env_r3.sh gpurun_out/$RUN/ab8.jsonl 2 "head=VR_LIB_PATH=build_ab/libvrhip_head.so" \
  "tree=VR_X=1" &&
python3 -c "
import json,collections
for f in ('ab','ab8'):
    r=collections.defaultdict(list)
    for l in open('gpurun_out/$RUN/%s.jsonl' % f):
        d=json.loads(l); L=d['line']
        r[d['ab']].append((L['ms_per_step'], L['roofline']['kernel_ms'], L.get('image_sha256','')[:12],
                           L.get('sim_parts_kernel_ms', {}).get('max')))
    for k,v in r.items(): print(f, k, v)
"
