# A/B: D = 2 exact path one output at a time (default) vs the shared-input pair form looped once
# per pair (-DNSH_DECIM2_SHARED=1, build/ab/libnsh_hip_d2s.so): main-path time (lib_ab), the
# exact-path bit-identity tests and the cliff with the variant swapped in (box copy only).
set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
DECIMS=2,4 timeout -k 10 200 python -u tools/probe/lib_ab.py newsched_amd/lib/libnsh_hip.so build/ab/libnsh_hip_d2s.so > $O/lib_ab.log 2>&1 && echo ab ok &&
cp build/ab/libnsh_hip_d2s.so newsched_amd/lib/libnsh_hip.so &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "exact_path_bit_identical or decim" > $O/pytest_d2s.log 2>&1 && echo tests ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 2 > $O/cliff_d2s.log 2>&1 && echo cliff ok
