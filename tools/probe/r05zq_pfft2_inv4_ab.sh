#!/bin/bash
# round 5: k_fir_pfft2's inverse on waves 4..7 (b4) vs 0..3 (b0, committed): two libraries only,
# four A/Bs alternating the order, 12 rounds each.
export TMPDIR=/tmp
O=gpurun_out/r05zq; mkdir -p $O
L=build/abl/pfft
for i in 1 2; do
  LOG2N=28 ROUNDS=12 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_b0.so ${L}_b4.so > $O/ab_${i}a.log 2>&1 &&
  LOG2N=28 ROUNDS=12 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_b4.so ${L}_b0.so > $O/ab_${i}b.log 2>&1 || exit 1
done
echo "rc=$?"
