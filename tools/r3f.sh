#!/bin/bash
# round-3 pass f: the GPU parity file with stale-HIP-error tracing and the runtime's error log
# (diagnosis of capture-status errors seen in pass e), then the whole GPU suite
RUN=${1:-r3f}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
{ VR_TRACE_STALE=1 AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread > gpurun_out/$RUN/parity.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/parity.log; [ $rc -le 1 ]; } &&
{ timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/$RUN/tests.log 2>&1;
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/tests.log; [ $rc -le 1 ]; } &&
grep -E "passed|failed" gpurun_out/$RUN/parity.log gpurun_out/$RUN/tests.log | tail -4
