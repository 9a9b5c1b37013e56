timeout -k 10 300 python -u tools/micro/unproject_floor.py > gpurun_out/floor.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/floor.log; exit $rc
