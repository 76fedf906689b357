#!/bin/bash
# round 5: k_fir_pfft2's inverse placement -- i0 = waves 0..3 before the wave's row loads (the
# committed form), il = after them, ih = waves 4..7 (1.8k cycles of slack at B2 in the phase trace),
# ihl = waves 4..7 after the loads; A/B both orders (outputs must be bit-identical).
export TMPDIR=/tmp
O=gpurun_out/r05zo; mkdir -p $O
L=build/abl/pfft
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_i0.so ${L}_il.so ${L}_ih.so ${L}_ihl.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_ihl.so ${L}_ih.so ${L}_il.so ${L}_i0.so > $O/ab2.log 2>&1
echo "rc=$?"
