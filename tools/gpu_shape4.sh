#!/bin/bash
# A/B of O3DX_STILE_SHAPE=4 (2x3 waves) against the default 2x2: the normals
# parity tests under shape 4, then the headline bench per shape.
# Usage (via gpurun): bash tools/gpu_shape4.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O3DX_STILE_SHAPE=4 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "normal" > gpurun_out/shape4_tests.log 2>&1 || { tail -30 gpurun_out/shape4_tests.log; exit 1; }
tail -1 gpurun_out/shape4_tests.log
for sh in 3 4 3 4; do
  O3DX_STILE_SHAPE=$sh timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --steps 20 \
    > gpurun_out/shape4_$sh.json 2> gpurun_out/shape4_$sh.err || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/shape4_$sh.json'));print('$sh',d['ms_per_step'],d['extra']['kernels']['normals_stile']['avg_ms'])"
done
