#!/bin/bash
# round 5: the channelizer's (and fft1024's) grid cap -- 4096 workgroups (committed), 8192, 16384
# (the frame copy's best, r05zn), 65536 (one frame per wave); A/B both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zt; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g4k.so ${L}_g8k.so ${L}_g16k.so ${L}_g64k.so > $O/chan1.log 2>&1 &&
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g64k.so ${L}_g16k.so ${L}_g8k.so ${L}_g4k.so > $O/chan2.log 2>&1 &&
KIND=fft LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g4k.so ${L}_g16k.so ${L}_g64k.so > $O/fft1.log 2>&1
echo "rc=$?"
