timeout -k 10 200 python tools/ablate.py --config c3 --bits 0 2048 128 64 2112 > gpurun_out/abl_c3.log 2>&1; grep -v amdgpu.ids gpurun_out/abl_c3.log
timeout -k 10 200 python tools/ablate.py --config c2 --bits 0 2048 128 > gpurun_out/abl_c2.log 2>&1; grep -v amdgpu.ids gpurun_out/abl_c2.log
