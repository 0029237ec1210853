cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t35.log 2>&1 ; tail -3 gpurun_out/t35.log
