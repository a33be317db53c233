#!/bin/bash
# Multi-GPU path rehearsal on a one-GPU box: bench.py under torchrun with N
# ranks sharing cuda:0 (gloo, O3DX_BENCH_SHARED_GPU=1) — C4 headline, sharded
# ICP and the C5 sharded pipeline at reduced sizes ($1 = ranks, default 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-2}
export O3DX_BENCH_SHARED_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$R" --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus "$R" --steps 10 --warmup 3 --c4-n 50000000 --c5-n ${C5N:-40000000} \
  --icp-n 2000000 > gpurun_out/rehearsal_$R.json 2> gpurun_out/rehearsal_$R.log
rc=$?
tail -c 3000 gpurun_out/rehearsal_$R.json
exit $rc
