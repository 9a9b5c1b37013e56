#!/bin/bash
# Build the unprojection arithmetic-floor microbenchmark (tools/micro/unproject_floor.hip)
# into tools/bin/unproject_floor.so (same flags as the product build).
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG="$ROOT/learnable-triangulation-pytorch_amd"
mkdir -p "$ROOT/tools/bin"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -I"$ROOT/include" -I"$PKG/csrc" "$ROOT/tools/micro/unproject_floor.hip" -o "$ROOT/tools/bin/unproject_floor.so"
