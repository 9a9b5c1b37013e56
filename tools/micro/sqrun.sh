set -e
for v in base corner; do
  MVN_HIP_LIB=$PWD/tools/bin/$v.so timeout -k 10 400 bash tools/pmc_sq.sh gpurun_out/sq_$v unproject_x4 python tools/prof_unproject.py 3 3
  python tools/sq_summary.py gpurun_out/sq_$v > gpurun_out/sq_$v.txt
done
