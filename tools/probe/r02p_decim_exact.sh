# D = 4 shared-input exact path, D = 2 back on the one-output form: FIR tests, lib A/B against
# the build before the decimator change (build/ab/libnsh_hip_head.so), exact-path cliffs, bench.
set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "mfma or direct or fir" > $O/pytest_fir.log 2>&1 && echo tests ok &&
DECIMS=1,2,4 timeout -k 10 200 python -u tools/probe/lib_ab.py build/ab/libnsh_hip_head.so newsched_amd/lib/libnsh_hip.so > $O/lib_ab.log 2>&1 && echo ab ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 2 > $O/cliff_d2.log 2>&1 && echo cliff2 ok &&
timeout -k 10 200 python -u tools/probe/cliff.py --decim 4 > $O/cliff_d4.log 2>&1 && echo cliff4 ok &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && echo bench ok
