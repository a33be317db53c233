#!/bin/bash
# the sharded ICP device loop with the sorts' own bounds: its GPU tests, then
# the one-rank RCCL bench leg again
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_distributed.py \
  -k "sharded_icp or c5_pipeline or icp" > gpurun_out/r06_shard_tests.log 2>&1 || { tail -30 gpurun_out/r06_shard_tests.log; exit 1; }
tail -3 gpurun_out/r06_shard_tests.log
bash tools/gpu_r06_rccl1.sh
