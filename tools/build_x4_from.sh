#!/bin/bash
# Build libmvn_hip.so with unproject_x4.hip replaced by another source file (A/B of kernel
# versions, e.g. one taken from git history) into tools/bin/<name>.so; the other objects come
# from the in-tree build.   tools/build_x4_from.sh name path/to/unproject_x4_variant.hip [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG="$ROOT/learnable-triangulation-pytorch_amd"
name=$1; src=$2; shift 2
mkdir -p "$ROOT/tools/bin"
make -s -C "$PKG"
tmp="$PKG/csrc/_variant_${name}.hip"; cp "$src" "$tmp"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics -I$ROOT/include -I$PKG/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$tmp" -o "$ROOT/tools/bin/$name.unproject_x4.o"
rm -f "$tmp"
objs=$(ls "$PKG"/build/*.o | grep -v unproject_x4.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$ROOT/tools/bin/$name.unproject_x4.o" -o "$ROOT/tools/bin/$name.so"
