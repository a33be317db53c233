#!/bin/bash
# ICP device loop at C3 (10M, 30 iterations): the in-tree build against MODE 2
# at 8 waves/SIMD (w8) and 512 accumulator copies (c512), alternated twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_icp_ab2.txt
for lib in in-tree w8 c512 in-tree w8 c512; do
  if [ $lib = in-tree ]; then unset O3DX_LIB; else export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_$lib.so; fi
  echo "== $lib" >> gpurun_out/r06_icp_ab2.txt
  timeout -k 10 200 python tools/icp_loop_ab.py 10000000 30 5 2>/dev/null >> gpurun_out/r06_icp_ab2.txt || exit 1
done
cat gpurun_out/r06_icp_ab2.txt
