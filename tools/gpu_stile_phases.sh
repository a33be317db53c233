#!/bin/bash
# Cumulative cost of the stile phases (O3DX_TILE_DEBUG=1 staging, 2 +histogram,
# 3 +list scan, 4 +moments, 0: full kernel) at a block shape (default 3).
# Usage (via gpurun): bash tools/gpu_stile_phases.sh [shape]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export O3DX_STILE_SHAPE=${1:-3}
: > gpurun_out/phases.txt
for dbg in 1 2 3 4 0; do
  if [ $dbg = 0 ]; then unset O3DX_TILE_DEBUG; else export O3DX_TILE_DEBUG=$dbg; fi
  timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --steps 20 \
    > gpurun_out/ph_$dbg.json 2> gpurun_out/ph_$dbg.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ph_$dbg.json')); print('$dbg', d['extra']['kernels']['normals_stile']['avg_ms'])" >> gpurun_out/phases.txt
done
cat gpurun_out/phases.txt
