# A/B: D = 2 exact path as a non-inlined shared-input pair call (NSH_DECIM2_SHARED=2,
# build/ab/libnsh_hip_d2c.so) vs the inlined one-output form: main path, bit-identity tests, cliff.
set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
DECIMS=2 ROUNDS=20 timeout -k 10 200 python -u tools/probe/lib_ab.py build/ab/libnsh_hip_base.so build/ab/libnsh_hip_d2c.so > $O/lib_ab.log 2>&1 && echo ab ok &&
cp build/ab/libnsh_hip_d2c.so newsched_amd/lib/libnsh_hip.so &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "exact_path_bit_identical or decim" > $O/pytest_d2c.log 2>&1 && echo tests ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 2 --kinds nan > $O/cliff_d2c.log 2>&1 && echo cliff ok
