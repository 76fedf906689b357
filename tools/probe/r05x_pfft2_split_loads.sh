#!/bin/bash
# round 5: k_fir_pfft2 row loads split by wave: waves 8..15 at the frame top, 0..7 after B1 (l2),
# with the inverse wave at priority 3 (l2p3), against p0 (all after B1) and p3; NSH_PFFT_FORM=2.
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_p0.so build/abl/pfft_l2.so build/abl/pfft_p3.so build/abl/pfft_l2p3.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_l2p3.so build/abl/pfft_p3.so build/abl/pfft_l2.so build/abl/pfft_p0.so > $O/ab_rev.log 2>&1
echo "rc=$?"
