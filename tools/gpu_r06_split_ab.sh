#!/bin/bash
# Variant build (_lib/var/libo3dx_${1:-split}.so): the stile's split launch
# (shell blocks + their hand-off tail on a side stream beside the interior
# blocks) and the dense start table filled from the runs.  The whole -m gpu
# suite on it, then A/B: the C2 step with and without the split
# (O3DX_STILE_NO_SPLIT), C5's ICP stage and the float64 normals with and
# without the run fill (O3DX_GRID_SCAN_STARTS: the count + scan form).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_${1:-split}.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06_split_tests.log 2>&1 || { tail -30 gpurun_out/r06_split_tests.log; exit 1; }
tail -2 gpurun_out/r06_split_tests.log
: > gpurun_out/r06_split_ab.txt
for i in 1 2; do
  for mode in split nosplit; do
    if [ $mode = nosplit ]; then export O3DX_STILE_NO_SPLIT=1; else unset O3DX_STILE_NO_SPLIT; fi
    timeout -k 10 200 python bench.py --no-cpu --no-secondary > gpurun_out/r06_split_$mode.json 2>/dev/null || exit 1
    python - "$mode" >> gpurun_out/r06_split_ab.txt <<'PYEOF' || exit 1
import json, sys
d = json.loads(open(f"gpurun_out/r06_split_{sys.argv[1]}.json").read().strip().splitlines()[-1])
k = d.get("extra", {}).get("kernels", {})
print(sys.argv[1], "ms_per_step", d["ms_per_step"], "value", d["value"],
      {n: k.get(n) for n in ("normals_stile", "normals_wave", "normals_knn")})
PYEOF
  done
done
unset O3DX_STILE_NO_SPLIT
for mode in fill scan; do
  if [ $mode = scan ]; then export O3DX_GRID_SCAN_STARTS=1; else unset O3DX_GRID_SCAN_STARTS; fi
  echo "== starts: $mode" >> gpurun_out/r06_split_ab.txt
  timeout -k 10 300 python tools/c5_icp_parts.py 200000000 >> gpurun_out/r06_split_ab.txt 2>/dev/null || exit 1
  timeout -k 10 200 python tools/f64_normals_ab.py >> gpurun_out/r06_split_ab.txt 2>/dev/null || exit 1
done
unset O3DX_GRID_SCAN_STARTS
echo "== f64 hand-offs to the lane form (O3DX_F64_NO_WAVE)" >> gpurun_out/r06_split_ab.txt
O3DX_F64_NO_WAVE=1 timeout -k 10 200 python tools/f64_normals_ab.py >> gpurun_out/r06_split_ab.txt 2>/dev/null || exit 1
cat gpurun_out/r06_split_ab.txt
