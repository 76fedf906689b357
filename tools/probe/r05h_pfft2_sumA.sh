#!/bin/bash
# round 5: k_fir_pfft2 with the phase sum of frame f - 1 and the inverse of frame f - 2 inside
# frame f's phase A (Z double-buffered, a dedicated inverse image): parity suite (both forms),
# form A/B at 2^28, and row loads default-policy vs nontemporal (build/abl/pfft_{def,nt}.so).
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/ab28.log 2>&1 &&
ROUNDS=8 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_def.so build/abl/pfft_nt.so > $O/ld_aux.log 2>&1 &&
ROUNDS=8 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_nt.so build/abl/pfft_def.so > $O/ld_aux_rev.log 2>&1
echo "rc=$?"
