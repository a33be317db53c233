#!/bin/bash
# Round-end evidence (ROUND, default r06), in two GPU calls:
#   bash tools/gpu_final.sh tests   — the full -m gpu suite + smoke(), every normal
#                                     row's parity logged to profiles-bound gpurun_out/\${R}_parity_report.jsonl
#   bash tools/gpu_final.sh bench   — PMC passes (profiles/pmc_traffic.json refreshed
#                                     for bench.py's roofline), the default bench line,
#                                     and the rocprofv3 kernel trace + stats of the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r06}
if [ "$1" = tests ]; then
  export O3DX_PARITY_LOG=$PWD/gpurun_out/${R}_parity_report.jsonl
  rm -f "$O3DX_PARITY_LOG"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${R}_gpu_tests.log; exit 1; }
  tail -2 gpurun_out/${R}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/${R}_smoke.log 2>&1 || { cat gpurun_out/${R}_smoke.log; exit 1; }
  tail -3 gpurun_out/${R}_smoke.log
  exit 0
fi
rm -rf gpurun_out/pmc
bash tools/pmc.sh gpurun_out/pmc -- python tools/prof_kernels.py ${PMC_WHAT:-all} > gpurun_out/pmc.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_summary.json || exit $?
python - <<'PYEOF' || exit $?
import json, os
old = json.load(open("profiles/pmc_traffic.json"))
new = json.load(open("gpurun_out/pmc_summary.json"))
old["kernels"].update(new["kernels"])
old["round"] = os.environ.get("ROUND", "r06")
for p in ("profiles/pmc_traffic.json", "gpurun_out/pmc_traffic.json"):
    with open(p, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
PYEOF
timeout -k 10 500 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
cat gpurun_out/${R}_bench.json
# C2 only (the headline step, no secondary legs): its own kernel stats, so
# the roofline recomputes from profiles/ without other configs' launches
rm -rf gpurun_out/prof_${R}_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_c2 -o run --output-format csv -- \
  python bench.py --no-cpu --no-secondary > gpurun_out/${R}_prof_c2.log 2>&1 || exit $?
[ -n "$NO_FULL_PROF" ] && { echo FINAL_DONE; exit 0; }
rm -rf gpurun_out/prof_${R}
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R} -o run --output-format csv -- \
  python bench.py --no-cpu > gpurun_out/${R}_prof_bench.log 2>&1 || exit $?
echo FINAL_DONE
