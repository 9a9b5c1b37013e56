#!/bin/bash
# SQ-only PMC passes (instruction mix and wave-state split).  Usage: tools/pmc_sq.sh <outdir> <regex> <cmd...>
set -e
out=$1; regex=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for counters in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
                "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_TRANS_F32" \
                "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "$regex" --output-format csv \
      -d "$out/p$i" -o pmc -- "$@" > "$out/p$i.log" 2>&1
done
echo "sq passes: $i"
