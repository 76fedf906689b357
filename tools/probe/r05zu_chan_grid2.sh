#!/bin/bash
# round 5: the channelizer's / fft1024's grid cap refined around r05zt's 16384 (12288, 16384, 24576,
# 32768 workgroups); A/B both orders for each kernel.
export TMPDIR=/tmp
O=gpurun_out/r05zu; mkdir -p $O
L=build/abl/nsh_fft
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g12k.so ${L}_g16k.so ${L}_g24k.so ${L}_g32k.so > $O/chan1.log 2>&1 &&
KIND=chan LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g32k.so ${L}_g24k.so ${L}_g16k.so ${L}_g12k.so > $O/chan2.log 2>&1 &&
KIND=fft LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g12k.so ${L}_g16k.so ${L}_g24k.so ${L}_g32k.so > $O/fft1.log 2>&1 &&
KIND=fft LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/chan_libs_ab.py ${L}_g32k.so ${L}_g24k.so ${L}_g16k.so ${L}_g12k.so > $O/fft2.log 2>&1
echo "rc=$?"
