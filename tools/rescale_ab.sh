set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rescale.py tests/test_gpu_keyswitch.py tests/test_cpp_host.py > gpurun_out/t5.log 2>&1
for i in 1 2; do
timeout -k 10 100 python3 tools/rescale_bw.py >> gpurun_out/rs6.log 2>&1
RS_LIB=upmem--openfhe_amd/lib/variants/libofhe_hip_nofuse.so timeout -k 10 100 python3 tools/rescale_bw.py >> gpurun_out/rs6.log 2>&1
done
