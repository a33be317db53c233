#!/bin/bash
# Round-4 iteration: GPU tests matching $1 (pytest -k; "all" runs the whole
# -m gpu suite, "none" skips it), then the cumulative stile phase costs and one
# bench line (no CPU legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K="$1"
if [ "$K" != none ]; then
  KA=(-k "$K")
  [ "$K" = all ] && KA=()
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" \
    > gpurun_out/iter_tests.log 2>&1 || { tail -30 gpurun_out/iter_tests.log; exit 1; }
  tail -2 gpurun_out/iter_tests.log
fi
[ "$2" = nophase ] || bash tools/gpu_stile_phases.sh 3 || exit $?
timeout -k 10 300 python bench.py --no-cpu --c5-n 0 > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || exit $?
python -c "
import json; d=json.load(open('gpurun_out/iter_bench.json')); e=d['extra']
print('step_ms', d['ms_per_step'], 'stile', e['kernels']['normals_stile']['avg_ms'], 'c4', e.get('c4_single_gpu',{}).get('ms'))
print('icp', e.get('icp',{}).get('iters_per_s'), 'ransac', e.get('ransac',{}).get('ms'))"
