#!/bin/bash
# C5's ICP stage (target grid build, source sort, 30-iteration loop) under a
# rocprofv3 kernel trace: where the build and the sort spend their time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_c5icp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5icp -o run --output-format csv -- \
  python tools/c5_icp_parts.py 200000000 > gpurun_out/r06_c5_icp_parts.txt 2>&1 || { tail -20 gpurun_out/r06_c5_icp_parts.txt; exit 1; }
grep '^{' gpurun_out/r06_c5_icp_parts.txt
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_c5icp/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  {int(r["Calls"]):5d}  {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
