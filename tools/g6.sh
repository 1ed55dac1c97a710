timeout -k 10 200 env CWF_VERBOSE=1 python tools/ablate.py --config c3 > gpurun_out/abl_c3.log 2>&1; cat gpurun_out/abl_c3.log | grep -v "^$" | tail -8 &&
timeout -k 10 200 env CWF_VERBOSE=1 python tools/ablate.py --config c2 > gpurun_out/abl_c2.log 2>&1; cat gpurun_out/abl_c2.log | tail -8
