# the driver's bench shape, N = 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err; rc=$?
tail -c 3000 gpurun_out/bench_driver.err; python3 tools/bench_brief.py gpurun_out/bench_driver.json; exit $rc
