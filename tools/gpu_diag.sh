#!/bin/bash
# Normals parity diagnostic + the default bench line, in one GPU call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/normals_diag.py gpurun_out/normals_diag.json > gpurun_out/normals_diag.log 2>&1 || { tail -20 gpurun_out/normals_diag.log; exit 1; }
cat gpurun_out/normals_diag.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_diag.json 2> gpurun_out/bench_diag.err || exit $?
cat gpurun_out/bench_diag.json
