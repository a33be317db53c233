#!/bin/bash
# Round-2 close-out: the whole -m gpu suite, the bench line, the rocprofv3
# kernel stats of the bench, and the plain dense voxel path for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/parity_report.jsonl
export O3DX_PARITY_LOG=$PWD/gpurun_out/parity_report.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
unset O3DX_PARITY_LOG
O3DX_VOXEL_PLAIN=1 timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --c5-n 0 --steps 20 \
  > gpurun_out/plain_voxel.json 2> gpurun_out/plain_voxel.err || exit $?
bash tools/gpu_r02_bench.sh
