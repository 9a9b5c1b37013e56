#!/bin/bash
# Memory-pipe PMC passes (TA / TD / TCP / LDS / L2) over one workload, one rocprofv3 run per
# line (block limits: TA 2, TD 2, TCP 4, TCC 4, SQ 8, GRBM 2).
#   tools/pmc_mem.sh <outdir> <kernel-regex> <cmd...>
set -e
out=$1; regex=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $counters --kernel-include-regex "$regex" --output-format csv \
      -d "$out/p$i" -o pmc -- "$@" > "$out/p$i.log" 2>&1
done <<'LIST'
GRBM_GUI_ACTIVE GRBM_TA_BUSY TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES
TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum
TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
LIST
echo "pmc passes: $i"
