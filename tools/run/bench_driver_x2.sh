# two back-to-back driver-shape bench runs (N = 1): run-to-run spread of this round's final build
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final_$i.json 2> gpurun_out/bench_final_$i.err || exit $?
  python3 tools/bench_brief.py gpurun_out/bench_final_$i.json
done
