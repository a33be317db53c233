#!/bin/bash
# Round-4 ICP iteration: the ICP GPU tests, the bench line (no CPU legs, no
# C4/C5), then PMC passes over the converged step kernel (prof_kernels icp).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or registration" \
  > gpurun_out/icp_tests.log 2>&1 || { tail -30 gpurun_out/icp_tests.log; exit 1; }
tail -2 gpurun_out/icp_tests.log
timeout -k 10 300 python bench.py --no-cpu --c4-n 0 --c5-n 0 > gpurun_out/icp_bench.json 2> gpurun_out/icp_bench.err || exit $?
python -c "
import json; d=json.load(open('gpurun_out/icp_bench.json')); e=d['extra']
print('step_ms', d['ms_per_step'], 'icp', json.dumps(e.get('icp')), 'ransac', e.get('ransac',{}).get('ms'))"
if [ "$1" = pmc ]; then
  rm -rf gpurun_out/pmc_icp
  bash tools/pmc.sh gpurun_out/pmc_icp -- python tools/prof_kernels.py ${PMC_WHAT:-icp_loop} > gpurun_out/pmc_icp.log 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_icp gpurun_out/pmc_icp.json > /dev/null || exit $?
  python -c "
import json; e=json.load(open('gpurun_out/pmc_icp.json'))['kernels']
for k, v in e.items():
    if 'icp' in k: print(k, {kk: (round(vv/ v.get('SQ_WAVES', 1), 1) if kk.startswith('SQ_') and kk != 'SQ_WAVES' else vv) for kk, vv in v.items()})"
fi
