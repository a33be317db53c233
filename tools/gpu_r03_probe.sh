#!/bin/bash
# Round-3 probe: raw C3 normals breakdown (sorted-grid path, search stats)
# and the 2-rank shared-GPU rehearsal of the multi-GPU bench (host/kernel split).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python tools/raw_normals_time.py > gpurun_out/raw_normals.json 2> gpurun_out/raw_normals.err || { tail -20 gpurun_out/raw_normals.err; exit 1; }
cat gpurun_out/raw_normals.json
bash tools/gpu_rehearsal.sh 2
