#!/bin/bash
# One SQ/GRBM pass (cycles, waits, MFMA busy, clock) per build of the V2V conv.
#   tools/pmc_cycles.sh <outdir> lib1.so lib2.so ...
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex v2v --output-format csv \
      -d "$out/$n" -o pmc -- python3 tools/ab_v2v.py --rounds 1 "$lib" > "$out/$n.log" 2>&1
  echo "== $n"; python3 tools/pmc_dump.py "$out/$n"
done
