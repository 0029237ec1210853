#!/bin/bash
# tools/ab_env_r3.sh OUT ROUNDS NAME1="ENV=.. ENV=.." NAME2="..." -- interleaved same-box A/B of bench.py
# runs under environment switches (serial frames, no CPU baseline); one JSON line per run in OUT.
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    echo -n "{\"ab\": \"$name\", \"round\": $r, \"line\": " >> "$OUT"
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --pipelined-streams 0 $BENCH_ARGS \
      2>/dev/null | tail -1 | tr -d '\n' >> "$OUT" || exit 1
    echo "}" >> "$OUT"
  done
done
