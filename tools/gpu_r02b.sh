#!/bin/bash
# Round-2b: parity of the given pytest -k selection, then the headline bench
# per O3DX_STILE_SHAPE listed in $2 (default "3 5 6").
# Usage (via gpurun): bash tools/gpu_r02b.sh "<pytest -k expr>" "3 5 6"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$1" \
  > gpurun_out/r02b_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r02b_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r02b_shapes.txt
for sh in ${2:-3 5 6}; do
  O3DX_STILE_SHAPE=$sh timeout -k 10 180 python bench.py --no-cpu --no-secondary --c4-n 0 --steps 20 \
    > gpurun_out/shape_$sh.json 2> gpurun_out/shape_$sh.err || exit $?
  python - "$sh" >> gpurun_out/r02b_shapes.txt <<'PY'
import json, sys
sh = sys.argv[1]
d = json.load(open(f"gpurun_out/shape_{sh}.json"))
k = d["extra"]["kernels"]
print(sh, d["ms_per_step"], {n: v["avg_ms"] for n, v in k.items()})
PY
done
cat gpurun_out/r02b_shapes.txt
