#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29534 tools/rccl_selftest.py > gpurun_out/r06_rccl_selftest.json 2> gpurun_out/r06_rccl_selftest.log \
  || { tail -30 gpurun_out/r06_rccl_selftest.log; exit 1; }
cat gpurun_out/r06_rccl_selftest.json
