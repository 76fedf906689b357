# A/B: exact-path tap loads as constant-offset scalar loads below the last tap block vs clamped
# loads everywhere (build/ab/libnsh_hip_prev.so): main paths (lib_ab, bit-identity), exact-path
# bit-identity tests, cliffs for decim 1 and 4.
set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "mfma or direct or fir" > $O/pytest_fir.log 2>&1 && echo tests ok &&
DECIMS=1,2,4 timeout -k 10 200 python -u tools/probe/lib_ab.py build/ab/libnsh_hip_prev.so newsched_amd/lib/libnsh_hip.so > $O/lib_ab.log 2>&1 && echo ab ok &&
timeout -k 10 200 python -u tools/probe/cliff.py > $O/cliff_d1.log 2>&1 && echo cliff1 ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 4 > $O/cliff_d4.log 2>&1 && echo cliff4 ok
