# A/B: k_fir_mfma12 chunk order, address order (base) vs groups of 4 rotated (NSH_V12_ROT=1):
# main path (lib_ab, bit-identity), and the exact-path cost curve with the variant swapped in.
set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
DECIMS=1 ROUNDS=20 timeout -k 10 200 python -u tools/probe/lib_ab.py build/ab/libnsh_hip_base.so build/ab/libnsh_hip_rot.so > $O/lib_ab.log 2>&1 && echo ab ok &&
cp build/ab/libnsh_hip_rot.so newsched_amd/lib/libnsh_hip.so &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "mfma or fir" > $O/pytest_rot.log 2>&1 && echo tests ok &&
timeout -k 10 300 python -u tools/probe/cliff.py --kinds spike --ks 0,32,16,8,6,4,3,2,1 > $O/cliff_rot.log 2>&1 && echo cliff ok
