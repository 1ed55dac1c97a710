timeout -k 10 200 python tools/ablate.py --config c3 --bits 0 512 1024 128 > gpurun_out/abl_c3.log 2>&1 && grep -v amdgpu.ids gpurun_out/abl_c3.log
