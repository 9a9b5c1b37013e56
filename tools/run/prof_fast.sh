# SQ + memory-pipe PMC passes of the config-3 unprojection in fast arithmetic
set -e
bash tools/pmc_sq.sh gpurun_out/sq3_fast2 'unproject_x4' python3 tools/prof_unproject.py 3 5 fast
python3 tools/sq_summary.py gpurun_out/sq3_fast2 > gpurun_out/sq3_fast2.txt
bash tools/pmc_mem.sh gpurun_out/mem3_fast 'unproject_x4' python3 tools/prof_unproject.py 3 5 fast
bash tools/pmc_mem.sh gpurun_out/mem3_exact 'unproject_x4' python3 tools/prof_unproject.py 3 5 exact
python3 tools/sq_summary.py gpurun_out/mem3_fast > gpurun_out/mem3_fast.txt
python3 tools/sq_summary.py gpurun_out/mem3_exact > gpurun_out/mem3_exact.txt
cat gpurun_out/sq3_fast2.txt gpurun_out/mem3_fast.txt gpurun_out/mem3_exact.txt
