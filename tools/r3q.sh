#!/bin/bash
# round-3 pass q: the whole GPU suite (stale-HIP-error tracing on, full-size parity lines kept) and
# the default bench line
RUN=${1:-r3q}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ VR_TRACE_STALE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -le 1 ]; } &&
timeout -k 10 400 python bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err &&
grep -E "passed|failed" gpurun_out/$RUN/tests.log | tail -2; grep -c VR_TRACE_STALE gpurun_out/$RUN/tests.log; cut -c1-400 gpurun_out/$RUN/bench.json
