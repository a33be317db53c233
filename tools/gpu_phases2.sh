#!/bin/bash
# Cumulative stile phase costs (O3DX_TILE_DEBUG 1..4, 0 = full) for the
# mirrored and the symmetric stencil (stile form).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/phases.txt
export O3DX_STILE_FORM=stile
for st in mirror sym; do
  export O3DX_STILE_STENCIL=$st
  for dbg in 1 2 3 4 0; do
    if [ $dbg = 0 ]; then unset O3DX_TILE_DEBUG; else export O3DX_TILE_DEBUG=$dbg; fi
    timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --c5-n 0 --steps 20 \
      > gpurun_out/ph_$dbg.json 2> gpurun_out/ph_$dbg.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ph_$dbg.json')); print('$st', '$dbg', d['extra']['kernels']['normals_stile']['avg_ms'])" >> gpurun_out/phases.txt
  done
done
cat gpurun_out/phases.txt
