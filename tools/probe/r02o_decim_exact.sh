set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "mfma or direct or fir" > $O/pytest_fir.log 2>&1 && echo tests ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 2 > $O/cliff_d2.log 2>&1 && echo cliff2 ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 4 > $O/cliff_d4.log 2>&1 && echo cliff4 ok &&
DECIMS=1,2,4 timeout -k 10 200 python -u tools/probe/lib_ab.py build/ab/libnsh_hip_head.so newsched_amd/lib/libnsh_hip.so > $O/lib_ab.log 2>&1 && echo ab ok &&
cp build/ab/libnsh_hip_head.so newsched_amd/lib/libnsh_hip.so &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 2 > $O/cliff_d2_before.log 2>&1 && echo cliff2b ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 4 > $O/cliff_d4_before.log 2>&1 && echo cliff4b ok
