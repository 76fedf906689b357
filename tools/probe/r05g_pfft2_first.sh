#!/bin/bash
# round 5: first run of k_fir_pfft2 (ring-less C5 form): form A/B at 2^22 and 2^28, then the pfft
# parity suite on the default form (2).
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
LOG2N=22 ROUNDS=3 timeout -k 10 120 python -u tools/probe/pfft_form_ab.py > $O/ab22.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/ab28.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_pfft.py -q --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1
echo "rc=$?"
