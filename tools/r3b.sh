#!/bin/bash
# round-3 diagnostics: C4 structure-channel parity variants, heavy-first schedule A/B, P=8 parts
RUN=${1:-r3b}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
ABL_SCENES=c4_struct timeout -k 10 600 python -u tools/shade_ablation.py gpurun_out/$RUN/c4diag.json base=default \
  nolds=default:VR_NO_LDS=1 k1=default:VR_DEPTH_LANES=1 exact=default:VR_EXACT_SHADE=1 \
  exactnolds=default:VR_EXACT_SHADE=1,VR_NO_LDS=1 noskip=default:VR_NO_EMPTY_SKIP=1 > gpurun_out/$RUN/c4diag.log 2>&1 &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab_sched.jsonl 2 "default=VR_X=0" "heavy8=VR_SCHED_TAIL_PCT=0" \
  "heavy4=VR_SCHED_TAIL_PCT=0 VR_SCHED_HEAVY_DIV=4" "heavy16=VR_SCHED_TAIL_PCT=0 VR_SCHED_HEAVY_DIV=16" &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipelined-streams 0 --sim-parts 8 > gpurun_out/$RUN/sim8.json 2>/dev/null &&
cat gpurun_out/$RUN/sim8.json
