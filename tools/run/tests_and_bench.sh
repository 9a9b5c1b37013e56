# GPU suite, then the driver's bench shape (N = 1); stops at the first failure
bash tools/run/tests.sh && bash tools/run/bench_driver.sh
