cd $GRAFT_REPO_ROOT &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "gradient_device or variants" > gpurun_out/t36.log 2>&1 ; tail -1 gpurun_out/t36.log;
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --gradient lookup > gpurun_out/c3.json 2> gpurun_out/c3.err &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --width 1024 --height 768 > gpurun_out/c2.json 2> gpurun_out/c2.err &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --n 2048 --width 4096 --height 4096 > gpurun_out/c5.json 2> gpurun_out/c5.err;
for f in c3 c2 c5; do tail -c 400 gpurun_out/$f.err; done
