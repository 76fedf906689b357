#!/bin/bash
# round 5: fft1024 / channelizer in the even/odd form with 16-B frame accesses (p1, NSH_FFT_PAIRS=1)
# vs the radix-16/16/4 form with 8-B accesses (p0); GPU FFT + channelizer tests on the default (p1)
# build first, then both orders for the channelizer and fft1024, and the configs binary's C4 lines.
set -o pipefail
O=gpurun_out/r05zc; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "fft or chan" --timeout 120 --timeout-method thread > $O/pytest_fft.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_cpp_runtime.py -q -x -k "hip_flowgraphs" --timeout 240 --timeout-method thread > $O/pytest_cpp.log 2>&1 &&
KIND=chan ROUNDS=10 timeout -k 10 240 python -u tools/probe/chan_libs_ab.py build/abl/nsh_fft_p1.so build/abl/nsh_fft_p0.so > $O/chan.log 2>&1 &&
KIND=chan ROUNDS=10 timeout -k 10 240 python -u tools/probe/chan_libs_ab.py build/abl/nsh_fft_p0.so build/abl/nsh_fft_p1.so > $O/chan_rev.log 2>&1 &&
KIND=fft ROUNDS=10 timeout -k 10 240 python -u tools/probe/chan_libs_ab.py build/abl/nsh_fft_p1.so build/abl/nsh_fft_p0.so > $O/fft.log 2>&1 &&
KIND=fft ROUNDS=10 timeout -k 10 240 python -u tools/probe/chan_libs_ab.py build/abl/nsh_fft_p0.so build/abl/nsh_fft_p1.so > $O/fft_rev.log 2>&1
echo "rc=$?"
