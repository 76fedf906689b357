#!/bin/bash
# round 5: k_fir_pfft2 with a hop of whole 64-row blocks (V = 384 at C5), the last 2 blocks of a
# frame kept in registers as the next frame's first (3 row loads a frame instead of 4): the pfft
# parity suite on the new build, then A/B against the committed build (build/abl/pfft_base.so)
# in both orders.
set -o pipefail
O=gpurun_out/r05zd; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 && echo "pfft tests ok" &&
LOG2N=28 ROUNDS=10 timeout -k 10 120 python -u tools/probe/pfft_ab.py build/abl/pfft_base.so build/abl/pfft_reuse.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 120 python -u tools/probe/pfft_ab.py build/abl/pfft_reuse.so build/abl/pfft_base.so > $O/ab2.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 120 python -u tools/probe/pfft_ab.py build/abl/pfft_base.so build/abl/pfft_reuse.so > $O/ab3.log 2>&1
echo "rc=$?"
