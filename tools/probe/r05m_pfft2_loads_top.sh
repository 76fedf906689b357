#!/bin/bash
# round 5: k_fir_pfft2 with next-frame loads issued at the frame top;
# parity suite (both forms), form A/B at 2^28, phase trace.
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/ab28.log 2>&1 &&
TRACE_OUT=$O/trace2.npy timeout -k 10 180 python -u tools/probe/pfft2_trace.py build/abl/pfft_trace.so > $O/trace2.log 2>&1
echo "rc=$?"
