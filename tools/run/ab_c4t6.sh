# 8-view kernel on a 6x8x8 tile of 384 threads (2 blocks per CU at 3 waves per SIMD)
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
AB_ONLY=cfg4 AB_CFG4=1 timeout -k 10 300 python -u tools/ab_lib.py $P tools/bin/c4t6.so > gpurun_out/ab_c4t6.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_c4t6.log; exit $rc
