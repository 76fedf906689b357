#!/bin/bash
# round 5: the split inverse's wave roles: s0 no split; s1 split, sum by waves 8..15, inverse on
# waves 0..3; s2 split, sum 0..7, inverse 0..3; s3 split, sum 0..7, inverse 12..15; s4 split, sum
# 8..15, inverse 12..15. Timing (outputs bit-identical across s*).
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_s0.so build/abl/pfft_s1.so build/abl/pfft_s2.so build/abl/pfft_s3.so build/abl/pfft_s4.so > $O/ab.log 2>&1 &&
ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_s4.so build/abl/pfft_s3.so build/abl/pfft_s2.so build/abl/pfft_s1.so build/abl/pfft_s0.so > $O/ab_rev.log 2>&1
echo "rc=$?"
