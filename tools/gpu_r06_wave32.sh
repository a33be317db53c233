#!/bin/bash
# the sorted-grid tiles' hand-offs through the exact-key wave form
# (k_normals_knn64_wave<float>): the whole -m gpu suite, then raw C3 and box-
# surface normals against the former wave form (O3DX_WAVE32_OLD=1), twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06_wave32_tests.log 2>&1 || { tail -30 gpurun_out/r06_wave32_tests.log; exit 1; }
tail -2 gpurun_out/r06_wave32_tests.log
: > gpurun_out/r06_wave32_ab.txt
for i in 1 2; do
  for mode in new old; do
    if [ $mode = old ]; then export O3DX_WAVE32_OLD=1; else unset O3DX_WAVE32_OLD; fi
    echo "== $mode" >> gpurun_out/r06_wave32_ab.txt
    timeout -k 10 200 python tools/raw_normals_time.py >> gpurun_out/r06_wave32_ab.txt 2>/dev/null || exit 1
    timeout -k 10 200 python tools/surface_normals_time.py >> gpurun_out/r06_wave32_ab.txt 2>/dev/null || exit 1
  done
done
cat gpurun_out/r06_wave32_ab.txt
