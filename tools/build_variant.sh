#!/bin/bash
# A/B kernel variants: a copy of csrc/ with a sed script applied to one
# source, built in-tree as open3dpypro/_lib/var/libo3dx_NAME.so (load it with
# O3DX_LIB=<path>).  Usage: tools/build_variant.sh NAME FILE 'sed script'
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1 FILE=$2 SED=$3
SRC=$ROOT/open3d-py-extension_amd/csrc
W=/tmp/o3dx_var_$NAME
rm -rf "$W" && mkdir -p "$W/x/csrc" "$W/include"
cp "$SRC"/*.hip "$SRC"/*.hpp "$SRC"/Makefile "$W/x/csrc/"
cp "$ROOT"/include/o3dx.h "$W/include/"
sed -i "$SED" "$W/x/csrc/$FILE"
diff -q "$SRC/$FILE" "$W/x/csrc/$FILE" > /dev/null && { echo "sed changed nothing"; exit 1; }
make -s -j8 -C "$W/x/csrc" OUT="$W/out" > /dev/null
mkdir -p "$ROOT/open3d-py-extension_amd/open3dpypro/_lib/var"
cp "$W/out/libo3dx.so" "$ROOT/open3d-py-extension_amd/open3dpypro/_lib/var/libo3dx_$NAME.so"
echo "built _lib/var/libo3dx_$NAME.so"
