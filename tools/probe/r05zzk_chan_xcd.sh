#!/bin/bash
# round 5: the channelizer with an XCD-contiguous lockstep walk (each XCD its own eighth of the frame
# groups) at 16384 / 8192 / 32768 workgroups vs the grid-stride walk (x0, default); both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zzk; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_x0.so ${L}_x1.so ${L}_x1g8.so ${L}_x1g32.so > $O/chan1.log 2>&1 &&
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_x1g32.so ${L}_x1g8.so ${L}_x1.so ${L}_x0.so > $O/chan2.log 2>&1
echo "rc=$?"
