#!/bin/bash
# round 5: k_fir_pfft2 with waves 12..15 (priority 3) and 8..11 (2) issuing their row loads ahead of
# the older waves (q4), against no priority change (q0); NSH_PFFT_FORM=2, both orders.
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_q0.so build/abl/pfft_q4.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_q4.so build/abl/pfft_q0.so > $O/ab_rev.log 2>&1
echo "rc=$?"
