#!/bin/bash
# round 5: k_fir_pfft2's cost per row-load instruction -- timing-only builds with 4 (the product),
# 3, 2, 1 and 0 of the four 16-B row loads per lane and frame (the rest register constants: wrong
# outputs), both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zl; mkdir -p $O
L=build/abl/pfft
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_n4.so ${L}_n3.so ${L}_n2.so ${L}_n1.so ${L}_n0.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 200 python -u tools/probe/pfft_ab.py ${L}_n0.so ${L}_n1.so ${L}_n2.so ${L}_n3.so ${L}_n4.so > $O/ab2.log 2>&1
echo "rc=$?"
