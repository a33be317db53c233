#!/bin/bash
# Round-end evidence in one GPU call: the full -m gpu suite, the PMC passes over
# the normals (profiles/pmc_traffic.json refreshed for bench.py's roofline),
# the default bench line, and the rocprofv3 kernel trace + stats of the bench.
# Usage (via gpurun): bash tools/gpu_final.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r01_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r01_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r01_gpu_tests.log
rm -rf gpurun_out/pmc
bash tools/pmc.sh gpurun_out/pmc -- python tools/prof_kernels.py normals > gpurun_out/pmc.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_summary.json || exit $?
python - <<'EOF' || exit $?
import json
old = json.load(open("profiles/pmc_traffic.json"))
new = json.load(open("gpurun_out/pmc_summary.json"))
old["kernels"].update(new["kernels"])
for p in ("profiles/pmc_traffic.json", "gpurun_out/pmc_traffic.json"):
    with open(p, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
EOF
timeout -k 10 400 python bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err || exit $?
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --no-cpu > gpurun_out/r01_prof_bench.log 2>&1 || exit $?
cat gpurun_out/r01_bench.json
