timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t1.log; tail -8 gpurun_out/t1.log; exit $rc
