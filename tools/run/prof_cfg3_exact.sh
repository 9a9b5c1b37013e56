# rocprof kernel trace of config 3 (exact), and its HBM traffic passes
set -e
out=gpurun_out/r21b; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_cfg3 -o kt -- \
    python3 bench.py --config 3 --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $out/kt_cfg3.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --kernel-include-regex 'unproject' --output-format csv \
      -d $out/pmc_${c}_cfg3 -o pmc -- python3 tools/prof_unproject.py 3 5 > $out/pmc_${c}_cfg3.log 2>&1
done
find $out -name "*kernel_stats.csv" | head -3
