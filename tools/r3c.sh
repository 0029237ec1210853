#!/bin/bash
# round-3 pass c: exp rounding microbench, GPU tests, C4 / C2 / metric parity ablation, bench,
# schedule A/B at the metric camera, P = 8 part times
RUN=${1:-r3c}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
timeout -k 10 120 tools/microbench/exp_check > gpurun_out/$RUN/exp_check.txt 2>&1 &&
{ timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -le 1 ]; } &&
timeout -k 10 400 python bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err &&
timeout -k 10 600 python -u tools/shade_ablation.py gpurun_out/$RUN/ablation.json base=default \
  exact=default:VR_EXACT_SHADE=1 nolds=default:VR_NO_LDS=1 > gpurun_out/$RUN/ablation.log 2>&1 &&
bash tools/ab_env_r3.sh gpurun_out/$RUN/ab_sched.jsonl 2 "default=VR_X=0" "heavy8=VR_SCHED_TAIL_PCT=0" \
  "heavy16=VR_SCHED_TAIL_PCT=0 VR_SCHED_HEAVY_DIV=16" &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipelined-streams 0 --sim-parts 8 > gpurun_out/$RUN/sim8.json 2>/dev/null &&
cat gpurun_out/$RUN/exp_check.txt && tail -2 gpurun_out/$RUN/tests.log
