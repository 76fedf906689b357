#!/bin/bash
# round 5: the channelizer's frames (waves) per workgroup with the larger grid: f4 = 4 (16384
# workgroups, the default), f2 = 2 (32768), f8 = 8 (8192), f4g8 = 4 with 8192; A/B both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zw; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_f4.so ${L}_f2.so ${L}_f8.so ${L}_f4g8.so > $O/chan1.log 2>&1 &&
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_f4g8.so ${L}_f8.so ${L}_f2.so ${L}_f4.so > $O/chan2.log 2>&1
echo "rc=$?"
