#!/bin/bash
# round 5: the channelizer with the next frame prefetched into registers (p1: 150 VGPRs, still 3
# waves per SIMD) at 16384 / 8192 / 24576 workgroups vs without (p0, the default); both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zz; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_p0.so ${L}_p1.so ${L}_p1g8.so ${L}_p1g24.so > $O/chan1.log 2>&1 &&
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_p1g24.so ${L}_p1g8.so ${L}_p1.so ${L}_p0.so > $O/chan2.log 2>&1
echo "rc=$?"
