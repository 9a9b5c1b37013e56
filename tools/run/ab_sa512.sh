timeout -k 10 300 python -u tools/ab_softargmax.py tools/bin/base.so tools/bin/sa512.so > gpurun_out/ab_sa512.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_sa512.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_step.py tools/bin/base.so tools/bin/sa512.so --no8 > gpurun_out/ab_sa512_step.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_sa512_step.log; exit $rc
