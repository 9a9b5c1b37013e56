#!/bin/bash
# PMC passes over the V2V front conv alone (tools/ab_v2v.py, one build), one rocprofv3 run
# per counter line.   tools/pmc_v2v.sh <outdir> <lib.so>
set -e
out=$1; lib=$2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters --kernel-include-regex v2v --output-format csv \
      -d "$out/p$i" -o pmc -- python3 tools/ab_v2v.py --rounds 1 "$lib" > "$out/p$i.log" 2>&1
done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VALU
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum
LIST
echo "pmc passes: $i"
