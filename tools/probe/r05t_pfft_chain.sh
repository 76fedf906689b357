#!/bin/bash
# round 5: k_fir_pfft<16,1> with the phase sum accumulated in place by four fixed-order wave chains
# (c1, NSH_PFFT_CHAIN=1: no product set, phase B = ring stores) vs the product images + phase-B
# reduction (c0); parity suite on the default (c1) first, then both build orders.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 &&
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_c1.so build/abl/pfft_c0.so > $O/ab.log 2>&1 &&
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_c0.so build/abl/pfft_c1.so > $O/ab_rev.log 2>&1
echo "rc=$?"
