# SQ instruction-mix passes of the config-3 unprojection, exact and fast arithmetic
set -e
bash tools/pmc_sq.sh gpurun_out/sq3_exact 'unproject_x4' python3 tools/prof_unproject.py 3 5 exact
bash tools/pmc_sq.sh gpurun_out/sq3_fast 'unproject_x4' python3 tools/prof_unproject.py 3 5 fast
python3 tools/sq_summary.py gpurun_out/sq3_exact > gpurun_out/sq3_exact.txt
python3 tools/sq_summary.py gpurun_out/sq3_fast > gpurun_out/sq3_fast.txt
cat gpurun_out/sq3_exact.txt gpurun_out/sq3_fast.txt
