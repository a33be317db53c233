#!/bin/bash
# Stile stencil A/B: parity of every variant, then bench + PMC per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/parity_report.jsonl
export O3DX_PARITY_LOG=$PWD/gpurun_out/parity_report.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "dense_voxel_table or 10m_voxel_table" > gpurun_out/stencil_tests.log 2>&1 || { tail -30 gpurun_out/stencil_tests.log; exit 1; }
tail -2 gpurun_out/stencil_tests.log
for v in "mirror vlist" "sym vlist" "mirror stile"; do
  set -- $v
  O3DX_STILE_STENCIL=$1 O3DX_STILE_FORM=$2 timeout -k 10 200 python bench.py --no-cpu --no-secondary \
    > gpurun_out/st_$1_$2.json 2> gpurun_out/st_$1_$2.err || exit 1
  python - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/st_{sys.argv[1]}_{sys.argv[2]}.json"))
print(sys.argv[1], sys.argv[2], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["extra"]["kernels"].items()})
PY
done
for st in mirror sym; do
  rm -rf gpurun_out/pmc_$st
  O3DX_STILE_STENCIL=$st O3DX_STILE_FORM=vlist bash tools/pmc.sh gpurun_out/pmc_$st -- python tools/prof_kernels.py normals > gpurun_out/pmc_$st.log 2>&1 || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_$st gpurun_out/pmc_$st.json > /dev/null || exit 1
  python - $st <<'PY'
import json, sys
e = json.load(open(f"gpurun_out/pmc_{sys.argv[1]}.json"))["kernels"]["normals_stile"]
print(sys.argv[1], {k: round(e[k]) for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE", "hbm_bytes_per_launch") if k in e})
PY
done
