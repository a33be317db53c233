#!/bin/bash
# ICP 1-NN walk: parity tests, then the C3 ICP leg with the row walk
# (default) and with the shell walk (O3DX_ICP_SHELL=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${1:-icp}" \
  > gpurun_out/r02d_tests.log 2>&1 || { tail -30 gpurun_out/r02d_tests.log; exit 1; }
tail -2 gpurun_out/r02d_tests.log
for mode in ${ICP_MODES:-rows shell}; do
  if [ $mode = shell ]; then export O3DX_ICP_SHELL=1; fi
  timeout -k 10 200 python bench.py --no-cpu --c4-n 0 --c5-n 0 --steps 5 > gpurun_out/icp_$mode.json \
    2> gpurun_out/icp_$mode.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/icp_$mode.json')); print('$mode', d['extra']['icp'])"
done
unset O3DX_ICP_SHELL
# target-grid settings under the row walk
: > gpurun_out/icp_sweep_rows.txt
for kv in ${ICP_SWEEP:-O3DX_ICP_MINH_DIV=20 O3DX_ICP_MINH_DIV=24 O3DX_ICP_MINH_DIV=32}; do
  env "$kv" timeout -k 10 200 python bench.py --no-cpu --c4-n 0 --c5-n 0 --steps 2 --warmup 1 \
    > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/sweep_one.json'))['extra']['icp']
print('$kv', d['iters_per_s'], d['match_kernel_ms'], d['accumulate_kernel_ms'], d['fitness'], d['T_err_vs_gt_inverse'])" \
    >> gpurun_out/icp_sweep_rows.txt
done
cat gpurun_out/icp_sweep_rows.txt
