#!/bin/bash
# tools/gpu.sh TAG 'commands...' -- run commands on the MI355X box via gpurun, logs in gpurun_out/TAG.*
# Each GPU step must carry its own `timeout -k 10 N`; steps are chained with && by the caller.
TAG=$1; shift
/usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-900} -- "export TMPDIR=/tmp; $*" > gpurun_out/$TAG.call 2>&1
rc=$?
tail -3 gpurun_out/$TAG.call
exit $rc
