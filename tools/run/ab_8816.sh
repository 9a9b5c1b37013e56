# 8x8x16 tiles of 1024 threads (one block per CU at 4 waves per SIMD): f32 exact (f8816) and bf16 exact (b8816)
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 400 python -u tools/ab_lib.py $P tools/bin/f8816.so tools/bin/b8816.so > gpurun_out/ab_8816.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_8816.log; exit $rc
