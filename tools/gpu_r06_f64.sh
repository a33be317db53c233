#!/bin/bash
# float64 normals tiles: parity tests, then the f64 chain timing (tiles vs the lane form)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_f64.py -k "normals or knn" > gpurun_out/r06_f64_tests.log 2>&1 || { tail -40 gpurun_out/r06_f64_tests.log; exit 1; }
tail -4 gpurun_out/r06_f64_tests.log
timeout -k 10 300 python tools/f64_time.py 2>/dev/null | tee gpurun_out/r06_f64_time.txt || exit 1
O3DX_F64_NO_TILES=1 timeout -k 10 300 python tools/f64_time.py 2>/dev/null | sed -n 1p | sed "s/^/no_tiles /" | tee -a gpurun_out/r06_f64_time.txt
