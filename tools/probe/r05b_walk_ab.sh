#!/bin/bash
# round 5: decimator lockstep walk with queued exact chunks (k_fir_mfma13 + k_fir_exact13) vs the
# contiguous walk (k_fir_mfma11): decimator parity tests (both walks), then walk_ab at D = 4 / 2
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "decim or exact_paths or odd_sample or null_history" > $O/pytest_decim.log 2>&1 || exit 1
echo tests-ok
DECIM=4 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4.log 2>&1 || exit 1
DECIM=4 MASKS=16,0 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_rev.log 2>&1 || exit 1
DECIM=4 INPUT=spike64 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_spike64.log 2>&1 || exit 1
DECIM=4 INPUT=spike4 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_spike4.log 2>&1 || exit 1
DECIM=2 MASKS=0,4 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2.log 2>&1 || exit 1
DECIM=2 MASKS=0,4 INPUT=spike64 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2_spike64.log 2>&1 || exit 1
echo ab-ok
