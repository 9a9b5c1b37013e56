# soft-argmax in MALL-sized frame groups (MVN_SA_GROUP_MB), standalone and inside the bench step
P=learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so
timeout -k 10 300 python -u tools/ab_softargmax.py $P tools/bin/sag48.so tools/bin/sag96.so tools/bin/sag160.so > gpurun_out/ab_sa_groups.log 2>&1 && \
timeout -k 10 400 python -u tools/ab_step.py $P tools/bin/sag48.so tools/bin/sag96.so tools/bin/sag160.so > gpurun_out/ab_sa_groups_step.log 2>&1
rc=$?; grep -hv amdgpu.ids gpurun_out/ab_sa_groups.log gpurun_out/ab_sa_groups_step.log; exit $rc
