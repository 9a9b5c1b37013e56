# the GPU suite's unprojection files on the debug build (device-side assertions)
MVN_HIP_LIB=$PWD/learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip_debug.so timeout -k 10 600 \
  python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_x4.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_debug.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_debug.log; tail -5 gpurun_out/tests_debug.log; exit $rc
