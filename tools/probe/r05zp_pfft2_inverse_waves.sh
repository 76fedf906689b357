#!/bin/bash
# round 5: k_fir_pfft2's inverse on waves 0..3 (b0, committed), 4..7 (b4; r05zo: 2-3 % faster), 8..11
# (b8) or 12..15 (b12), before the wave's row loads; A/B both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zp; mkdir -p $O
L=build/abl/pfft
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_b0.so ${L}_b4.so ${L}_b8.so ${L}_b12.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_b12.so ${L}_b8.so ${L}_b4.so ${L}_b0.so > $O/ab2.log 2>&1
echo "rc=$?"
