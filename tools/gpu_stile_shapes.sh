#!/bin/bash
# Normals-on-voxel-table block shapes: parity tests for the stile path, then
# the headline bench per O3DX_STILE_SHAPE (1: one wave per 4^3 block;
# 2: 2x2 waves sharing one box; 3: 2x2 allocated for 3 waves/SIMD).
# Usage (via gpurun): bash tools/gpu_stile_shapes.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "normals" \
  > gpurun_out/shape_tests.log 2>&1
rc=$?
tail -3 gpurun_out/shape_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/shape_bench.txt
for sh in 1 2 3; do
  O3DX_STILE_SHAPE=$sh timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --steps 20 \
    > gpurun_out/shape_$sh.json 2> gpurun_out/shape_$sh.err || exit $?
  python - "$sh" >> gpurun_out/shape_bench.txt <<'EOF'
import json, sys
sh = sys.argv[1]
d = json.load(open(f"gpurun_out/shape_{sh}.json"))
k = d["extra"]["kernels"]
print(sh, d["ms_per_step"], {n: v["avg_ms"] for n, v in k.items()})
EOF
done
cat gpurun_out/shape_bench.txt
