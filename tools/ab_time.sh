#!/bin/bash
# tools/ab_time.sh ROUNDS lib1 lib2 ... -- on the GPU box: interleaved bench.py kernel times of
# library builds (build_ab/libvrhip_<name>.so; "cur" = the in-tree library), ROUNDS rounds each.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do for n in "$@"; do
  lib=volume_renderer_amd/libvrhip.so; [ "$n" != cur ] && lib=build_ab/libvrhip_$n.so
  VR_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --pipelined-streams 0 \
    > gpurun_out/ab/$n.$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab/$n.$r.json').read().strip().splitlines()[-1]);print('$n', $r, d['roofline']['kernel_ms'])" | tee -a gpurun_out/ab/summary.txt
done; done
