#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_check.json 2> gpurun_out/r06_bench_check.err || { tail -20 gpurun_out/r06_bench_check.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06_bench_check.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['scaling'],d['roofline']['frac'],d['cpu_baseline']['value'])"
