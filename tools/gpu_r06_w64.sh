#!/bin/bash
# float64 hand-off wave form: the f64 suite on the in-tree build, A/B of the
# in-tree build against the 4-waves/SIMD variant (wpe4) and the lane form
# (O3DX_F64_NO_WAVE), then the full -m gpu suite + smoke (gpu_final.sh tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64.py \
  > gpurun_out/r06_w64_tests.log 2>&1 || { tail -40 gpurun_out/r06_w64_tests.log; exit 1; }
tail -2 gpurun_out/r06_w64_tests.log
: > gpurun_out/r06_w64_ab.txt
for i in 1 2; do
  for v in in-tree wpe4 lane; do
    unset O3DX_LIB O3DX_F64_NO_WAVE
    if [ $v = wpe4 ]; then export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_wpe4.so; fi
    if [ $v = lane ]; then export O3DX_F64_NO_WAVE=1; fi
    timeout -k 10 200 python tools/f64_normals_ab.py >> gpurun_out/r06_w64_ab.txt 2>/dev/null || exit 1
  done
done
unset O3DX_LIB O3DX_F64_NO_WAVE
cat gpurun_out/r06_w64_ab.txt
bash tools/gpu_final.sh tests
