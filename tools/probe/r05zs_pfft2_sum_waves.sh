#!/bin/bash
# round 5: k_fir_pfft2's phase-sum waves (inverse on 4..7): s0 = 0..7 (committed), s1 = 4..11,
# s2 = 0..3 + 8..11, s3 = 0..3 + 12..15; A/B both orders, then s0 vs the best two-library style.
export TMPDIR=/tmp
O=gpurun_out/r05zs; mkdir -p $O
L=build/abl/pfft
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_s0.so ${L}_s1.so ${L}_s2.so ${L}_s3.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_s3.so ${L}_s2.so ${L}_s1.so ${L}_s0.so > $O/ab2.log 2>&1
echo "rc=$?"
