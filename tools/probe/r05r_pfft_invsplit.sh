#!/bin/bash
# round 5: k_fir_pfft<16,1> with the inverse split over two frames (its pass 1 in phase B, the rest
# after B2; s1, NSH_PFFT_INVSPLIT=1) vs the whole inverse after B2 (s0); parity suite first.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 &&
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_s1.so build/abl/pfft_s0.so > $O/ab.log 2>&1 &&
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_s0.so build/abl/pfft_s1.so > $O/ab_rev.log 2>&1
echo "rc=$?"
