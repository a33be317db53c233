#!/bin/bash
# A/B against a git revision: csrc/ of REV built in /tmp as
# open3dpypro/_lib/var/libo3dx_NAME.so (load with O3DX_LIB=<path>).
# Usage: tools/build_rev.sh NAME REV
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1 REV=$2
W=/tmp/o3dx_rev_$NAME
rm -rf "$W" && mkdir -p "$W/x/csrc" "$W/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" open3d-py-extension_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$W/x/csrc/$(basename "$f")"
done
git -C "$ROOT" show "$REV:include/o3dx.h" > "$W/include/o3dx.h"
make -s -j8 -C "$W/x/csrc" OUT="$W/out" > /dev/null
mkdir -p "$ROOT/open3d-py-extension_amd/open3dpypro/_lib/var"
cp "$W/out/libo3dx.so" "$ROOT/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_$NAME.so"
echo "built _lib/var/libo3dx_$NAME.so from $REV"
