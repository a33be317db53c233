#!/bin/bash
# Round-2 checkpoint: distributed GPU tests, the default bench line (C2 + CPU
# legs + C3/C4/C5), and a 2-rank rehearsal of the N>1 headline on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -3 gpurun_out/dist_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err || { tail -30 gpurun_out/bench_r02a.err; exit 1; }
cat gpurun_out/bench_r02a.json
O3DX_BENCH_SHARED_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --c4-n 20000000 \
  > gpurun_out/bench_r02a_2r.json 2> gpurun_out/bench_r02a_2r.err || { tail -30 gpurun_out/bench_r02a_2r.err; exit 1; }
cat gpurun_out/bench_r02a_2r.json
