#!/bin/bash
# Build libmvn_hip.so with extra -D flags on ONE source file into tools/bin/<name>.so (A/B
# variants for tools/ab_step.py / ab_x4.py / ab_softargmax.py; the other objects come from
# the in-tree build).
#   tools/build_variant.sh name source.hip [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG="$ROOT/learnable-triangulation-pytorch_amd"
name=$1; src=$2; shift 2
base=$(basename "$src" .hip)
# src: a file name in csrc/, or a path to another version of one (e.g. from git show)
if [ -f "$src" ]; then srcpath=$src; else srcpath="$PKG/csrc/$base.hip"; fi
mkdir -p "$ROOT/tools/bin"
make -s -C "$PKG"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics -I$ROOT/include -I$PKG/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$srcpath" -o "$ROOT/tools/bin/$name.$base.o"
objs=$(ls "$PKG"/build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$ROOT/tools/bin/$name.$base.o" -o "$ROOT/tools/bin/$name.so"
