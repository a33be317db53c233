#!/bin/bash
# float64 lane-form batching A/B (in-tree = 2 loads in flight; b1, b4), tiles and lane form each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f64.py -k "normals or knn" > gpurun_out/r06_f64_tests.log 2>&1 || { tail -40 gpurun_out/r06_f64_tests.log; exit 1; }
tail -2 gpurun_out/r06_f64_tests.log
for v in in-tree b1 b4; do
  if [ $v = in-tree ]; then unset O3DX_LIB; else export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_$v.so; fi
  timeout -k 10 200 python tools/f64_normals_ab.py 2>/dev/null | tee -a gpurun_out/r06_f64_b.txt || exit 1
  O3DX_F64_NO_TILES=1 timeout -k 10 200 python tools/f64_normals_ab.py 2>/dev/null | tee -a gpurun_out/r06_f64_b.txt || exit 1
done
