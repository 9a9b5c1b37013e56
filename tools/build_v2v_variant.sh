#!/bin/bash
# Build csrc/v2v_front.hip alone into tools/bin/<name>.so with extra -D flags (A/B variants).
#   tools/build_v2v_variant.sh name [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$ROOT/tools/bin"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -I"$ROOT/include" -I"$ROOT/learnable-triangulation-pytorch_amd/csrc" "$@" \
  "$ROOT/learnable-triangulation-pytorch_amd/csrc/v2v_front.hip" -o "$ROOT/tools/bin/$name.so"
