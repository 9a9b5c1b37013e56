# region words laundered per use (RegionSet::get), fast bf16 at 6 and 8 waves: fast and exact A/B
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 400 python -u tools/ab_fast.py $P tools/bin/launder.so tools/bin/launder_w8.so > gpurun_out/ab_launder_fast.log 2>&1 && \
AB_CFG4=1 timeout -k 10 400 python -u tools/ab_lib.py $P tools/bin/launder.so > gpurun_out/ab_launder_exact.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_launder_fast.log gpurun_out/ab_launder_exact.log; exit $rc
