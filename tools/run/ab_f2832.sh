# f32 4-view kernel on a 2x8x32 tile (128-byte z-runs of f32 output)
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 300 python -u tools/ab_lib.py $P tools/bin/f2832.so > gpurun_out/ab_f2832.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_f2832.log | grep cfg2; exit $rc
