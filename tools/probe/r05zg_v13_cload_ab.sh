#!/bin/bash
# round 5: k_fir_mfma13 D = 4, the committed strided loads (c0) vs contiguous loads default policy
# (c1) and nontemporal (c1nt), three orders x 20 rounds (r05ze and r05zf disagreed across boxes)
export TMPDIR=/tmp
O=gpurun_out/r05zg; mkdir -p $O
L=build/abl/nsh_fir_mfma
DECIM=4 ROUNDS=20 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1nt.so ${L}_c1.so > $O/d4_1.log 2>&1 &&
DECIM=4 ROUNDS=20 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c1nt.so ${L}_c1.so ${L}_c0.so > $O/d4_2.log 2>&1 &&
DECIM=4 ROUNDS=20 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c1.so ${L}_c0.so ${L}_c1nt.so > $O/d4_3.log 2>&1
echo "rc=$?"
