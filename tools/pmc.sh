#!/bin/bash
# PMC passes over one workload (MI355X_MICROARCH.md: separate --pmc passes, no tracing
# domains combined with counters).  Usage: tools/pmc.sh <outdir> <kernel-regex> <cmd...>
set -e
out=$1; regex=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "$regex" --output-format csv \
      -d "$out/p$i" -o pmc -- "$@" > "$out/p$i.log" 2>&1
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_TRANS_F32
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum
LIST
echo "pmc passes: $i"
