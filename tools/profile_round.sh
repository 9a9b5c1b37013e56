#!/bin/bash
# One round's profiles (run on the GPU box):  tools/profile_round.sh <round-tag>
#   1. rocprofv3 --kernel-trace --stats over bench.py (all configs; then configs 2, 3, 4 one per run)
#   2. PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: separate passes) per config
#   3. SQ instruction-mix passes on config 2
# Raw output under gpurun_out/<tag>/; tools/profile_summary.py turns it into profiles/.
set -e
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-in-kernel-coords > "$out/kt.log" 2>&1
echo "kernel trace done"
# one config per process: a kernel that serves several configs gets one mean per config
for cfg in 2 3 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_cfg$cfg" -o kt -- \
      python3 bench.py --config $cfg --steps 20 --warmup 5 --no-secondary --no-cpu-baseline \
      > "$out/kt_cfg$cfg.log" 2>&1
done
# the fast arithmetic, configs 2 and 3
for cfg in 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_cfg${cfg}_fast" -o kt -- \
      python3 bench.py --config $cfg --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --precision fast \
      > "$out/kt_cfg${cfg}_fast.log" 2>&1
done
echo "per-config kernel traces done"
for cfg in 2 3 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex 'mvn' --output-format csv \
        -d "$out/pmc_${c}_cfg$cfg" -o pmc -- python3 tools/prof_unproject.py $cfg 5 > "$out/pmc_${c}_cfg$cfg.log" 2>&1
  done
done
for cfg in 2 3 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex 'unproject' --output-format csv \
        -d "$out/pmc_${c}_cfg${cfg}_fast" -o pmc -- python3 tools/prof_unproject.py $cfg 5 fast \
        > "$out/pmc_${c}_cfg${cfg}_fast.log" 2>&1
  done
done
echo "traffic passes done"
bash tools/pmc_sq.sh "$out/sq_cfg2" 'unproject_x4' python3 tools/prof_unproject.py 2 5
bash tools/pmc_sq.sh "$out/sq_cfg3" 'unproject_x4' python3 tools/prof_unproject.py 3 5
bash tools/pmc_sq.sh "$out/sq_cfg3_fast" 'unproject_x4' python3 tools/prof_unproject.py 3 5 fast
echo "sq passes done"
# memory pipe (TA / TD / TCP / L2 hit-miss) of the config-3 and config-4 unprojections, both arithmetics
for cfg in 3 4; do
  bash tools/pmc_mem.sh "$out/mem_cfg$cfg" 'unproject_x4' python3 tools/prof_unproject.py $cfg 5
  bash tools/pmc_mem.sh "$out/mem_cfg${cfg}_fast" 'unproject_x4' python3 tools/prof_unproject.py $cfg 5 fast
done
echo "memory-pipe passes done"
timeout -k 10 120 python3 tools/repack_cost.py > "$out/repack_cost.txt" 2>&1
python3 tools/step_gaps.py "$out/kt_cfg2/kt_kernel_trace.csv" > "$out/step_gaps_cfg2.txt" 2>&1 || true
python3 tools/step_gaps.py "$out/kt_cfg3/kt_kernel_trace.csv" > "$out/step_gaps_cfg3.txt" 2>&1 || true
bash tools/pmc_cycles.sh "$out/v2v_cycles" learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so > "$out/v2v_cycles.txt" 2>&1
echo "v2v cycle pass done"
