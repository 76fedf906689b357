#!/bin/bash
# round 5: 1024-point transforms in the 32 x 32 form (two frames per wave, one LDS exchange,
# NSH_FFT_2X=1) vs the 16 x 16 x 4 form (NSH_FFT_2X=0): channelizer and fft1024, both orders;
# then the FFT / channelizer parity tests on the new form
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan timeout -k 10 200 python tools/probe/fftlib_ab.py ${L}_old.so ${L}_x2.so > $O/chan_1.log 2>&1 || exit 1
KIND=chan timeout -k 10 200 python tools/probe/fftlib_ab.py ${L}_x2.so ${L}_old.so > $O/chan_2.log 2>&1 || exit 1
KIND=fft timeout -k 10 200 python tools/probe/fftlib_ab.py ${L}_old.so ${L}_x2.so > $O/fft_1.log 2>&1 || exit 1
echo ab-ok
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "fft or chan" > $O/pytest_fft.log 2>&1 || exit 1
timeout -k 10 300 build/tests/qa_hip_flowgraph > $O/qa_hip.log 2>&1 || exit 1
echo tests-ok
