# exact bf16 unprojection on an 8x8x8 tile at 4 waves (2 blocks of 512 per CU)
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 300 python -u tools/ab_lib.py $P tools/bin/e888w4.so > gpurun_out/ab_e888w4.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_lib.py $P tools/bin/e888w4.so > gpurun_out/ab_e888w4b.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_e888w4.log gpurun_out/ab_e888w4b.log | grep cfg3; exit $rc
