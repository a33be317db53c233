#!/bin/bash
# A/B of library variants on the surface-normals path (10M box surface,
# tools/surface_normals_time.py): the in-tree build, then each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in in-tree "$@" in-tree "$@"; do
  if [ $lib = in-tree ]; then unset O3DX_LIB; else export O3DX_LIB=$PWD/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_$lib.so; fi
  echo "== $lib"
  timeout -k 10 200 python tools/surface_normals_time.py "" 2>/dev/null | tee -a gpurun_out/r06_surface_ab.txt || exit 1
done
