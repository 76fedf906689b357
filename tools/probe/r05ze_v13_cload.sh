#!/bin/bash
# round 5: k_fir_mfma13 (D = 4) with contiguous chunk loads (NSH_V13_CLOAD: each load instruction
# 1 KiB contiguous, lane pairs exchange by DPP before the split stores) vs the strided loads (c0 =
# the committed form), default and nontemporal load policy; decimator tests on the new build first.
export TMPDIR=/tmp
O=gpurun_out/r05ze; mkdir -p $O
L=build/abl/nsh_fir_mfma
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "decim" --timeout 120 --timeout-method thread > $O/pytest_decim.log 2>&1 && echo "decim tests ok" &&
DECIM=4 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1.so ${L}_c1nt.so > $O/d4_1.log 2>&1 &&
DECIM=4 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c1nt.so ${L}_c1.so ${L}_c0.so > $O/d4_2.log 2>&1 &&
DECIM=4 INPUT=spike64 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1.so > $O/d4_spike64.log 2>&1 &&
DECIM=2 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1.so > $O/d2.log 2>&1
echo "rc=$?"
