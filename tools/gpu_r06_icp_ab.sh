set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py -k "sharded_icp or c5_pipeline" > gpurun_out/r06_b_tests.log 2>&1 || { tail -30 gpurun_out/r06_b_tests.log; exit 1; }
tail -12 gpurun_out/r06_b_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "icp or skip" > gpurun_out/r06_c_icp_tests.log 2>&1 || { tail -30 gpurun_out/r06_c_icp_tests.log; exit 1; }
tail -3 gpurun_out/r06_c_icp_tests.log
for lib in base in-tree base in-tree; do
  if [ $lib = base ]; then export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_base.so; else unset O3DX_LIB; fi
  timeout -k 10 200 python tools/icp_loop_ab.py 10000000 30 5 2>/dev/null | tee -a gpurun_out/r06_icp_ab.txt || exit 1
done
