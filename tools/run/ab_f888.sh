# f32 4-view kernel on the 8x8x8 tile (2 blocks of 512 per CU), non-temporal and default output stores
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 300 python -u tools/ab_lib.py $P tools/bin/f888nt.so tools/bin/f888d.so > gpurun_out/ab_f888.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_step.py $P tools/bin/f888nt.so tools/bin/f888d.so > gpurun_out/ab_f888_step.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_f888.log gpurun_out/ab_f888_step.log | grep cfg2; exit $rc
