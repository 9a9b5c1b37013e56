# GPU suite, the fast-variant A/B and the timing-events A/B
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t1.log; tail -5 gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/run/ab_fast.sh || exit $?
bash tools/run/events_ab.sh
