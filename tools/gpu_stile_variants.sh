#!/bin/bash
# Normals on the voxel table: parity tests with the merged histogram/list pass
# on, then the headline bench per variant "SHAPE:MERGED" (O3DX_STILE_SHAPE,
# O3DX_STILE_MERGED).  Usage (via gpurun): bash tools/gpu_stile_variants.sh [variants...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O3DX_STILE_MERGED=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "normals" > gpurun_out/variant_tests.log 2>&1
rc=$?
tail -3 gpurun_out/variant_tests.log
[ $rc -eq 0 ] || exit $rc
vars=("$@")
[ ${#vars[@]} -eq 0 ] && vars=(3:0 2:1 1:1)
: > gpurun_out/variant_bench.txt
for v in "${vars[@]}"; do
  sh=${v%%:*}; mg=${v##*:}
  O3DX_STILE_SHAPE=$sh O3DX_STILE_MERGED=$mg timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 \
    --steps 20 > gpurun_out/variant.json 2> gpurun_out/variant.err || exit $?
  python - "$v" >> gpurun_out/variant_bench.txt <<'EOF'
import json, sys
d = json.load(open("gpurun_out/variant.json"))
k = d["extra"]["kernels"]
print(sys.argv[1], d["ms_per_step"], {n: v["avg_ms"] for n, v in k.items()})
EOF
done
cat gpurun_out/variant_bench.txt
