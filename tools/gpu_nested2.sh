#!/bin/bash
# nested-grid trigger: dense-cell query counts on the surface and the planted-plane clouds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export O3DX_NESTED_VERBOSE=1
timeout -k 10 200 python tools/surface_normals_time.py > gpurun_out/surf.jsonl 2> gpurun_out/surf.err || { tail gpurun_out/surf.err; exit 1; }
timeout -k 10 200 python tools/raw_normals_time.py > gpurun_out/raw.jsonl 2> gpurun_out/raw.err || { tail gpurun_out/raw.err; exit 1; }
cat gpurun_out/surf.jsonl gpurun_out/raw.jsonl; sort -u gpurun_out/surf.err gpurun_out/raw.err | grep nested
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "nested or raw_planted" > gpurun_out/nested2_tests.log 2>&1 || { tail -30 gpurun_out/nested2_tests.log; exit 1; }
tail -2 gpurun_out/nested2_tests.log
