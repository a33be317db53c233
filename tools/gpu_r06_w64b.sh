#!/bin/bash
# float64 hand-off wave form (ballot-counted member selection, 4 waves/SIMD)
# and the skip step without its mpos read: the f64 + ICP tests, then the
# float64 normals A/B against the lane form, and C5's ICP stage in parts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64.py \
  tests/test_gpu_kernels.py tests/test_gpu_scale.py -k "f64 or icp" > gpurun_out/r06_w64b_tests.log 2>&1 \
  || { tail -40 gpurun_out/r06_w64b_tests.log; exit 1; }
tail -2 gpurun_out/r06_w64b_tests.log
: > gpurun_out/r06_f64_wave_ab.txt
for i in 1 2; do
  for v in wave lane; do
    if [ $v = lane ]; then export O3DX_F64_NO_WAVE=1; else unset O3DX_F64_NO_WAVE; fi
    timeout -k 10 200 python tools/f64_normals_ab.py >> gpurun_out/r06_f64_wave_ab.txt 2>/dev/null || exit 1
  done
done
unset O3DX_F64_NO_WAVE
cat gpurun_out/r06_f64_wave_ab.txt
timeout -k 10 300 python tools/c5_icp_parts.py 200000000 > gpurun_out/r06_c5_icp_parts_b.txt 2>/dev/null || exit 1
cat gpurun_out/r06_c5_icp_parts_b.txt
