#!/bin/bash
# round-3 pass h: host upload through the pinned bounce ring (VR_UPLOAD_BOUNCE=1, 4/8/16 filler
# threads) against the runtime's pageable copy: upload alone and the overlapped movie
RUN=${1:-r3h}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$RUN &&
for cfg in "VR_UPLOAD_BOUNCE=0" "VR_UPLOAD_BOUNCE=1 VR_UPLOAD_THREADS=4" "VR_UPLOAD_BOUNCE=1 VR_UPLOAD_THREADS=8" "VR_UPLOAD_BOUNCE=1 VR_UPLOAD_THREADS=16"; do
  echo "== $cfg" >> gpurun_out/$RUN/upload.log
  env $cfg VR_UPLOAD_TIMING=1 timeout -k 10 200 python tools/e2e_bench.py --upload-only --reps 5 >> gpurun_out/$RUN/upload.log 2>&1 || exit 1
done &&
for cfg in "VR_UPLOAD_BOUNCE=0" "VR_UPLOAD_BOUNCE=1 VR_UPLOAD_THREADS=8" "VR_UPLOAD_BOUNCE=1 VR_UPLOAD_THREADS=16"; do
  echo "== $cfg" >> gpurun_out/$RUN/movie.log
  env $cfg VR_UPLOAD_TIMING=1 timeout -k 10 300 python tools/e2e_bench.py --movie-only >> gpurun_out/$RUN/movie.log 2>&1 || exit 1
done && grep -v "^VR_UPLOAD_TIMING\|amdgpu.ids" gpurun_out/$RUN/upload.log gpurun_out/$RUN/movie.log
