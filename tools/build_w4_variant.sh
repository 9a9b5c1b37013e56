#!/bin/bash
# Build libmvn_hip.so with extra -D flags on the wave-autonomous unprojection (unproject_w4.hip)
# into tools/bin/<name>.so (A/B variants for tools/ab_lib.py).
#   tools/build_w4_variant.sh name [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG="$ROOT/learnable-triangulation-pytorch_amd"
name=$1; shift
mkdir -p "$ROOT/tools/bin"
make -s -C "$PKG"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics -I$ROOT/include -I$PKG/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$PKG/csrc/unproject_w4.hip" -o "$ROOT/tools/bin/$name.unproject_w4.o"
objs=$(ls "$PKG"/build/*.o | grep -v unproject_w4.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$ROOT/tools/bin/$name.unproject_w4.o" -o "$ROOT/tools/bin/$name.so"
rm -f "$ROOT/tools/bin/$name.unproject_w4.o"
