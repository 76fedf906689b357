#!/bin/bash
# round 5: k_fir_mfma13 (D = 4) build variants in one process (lib_abn, ABAB / BABA):
# b0 = default; nt4 = nontemporal chunk loads; xw = one global lockstep row (XCD x takes window
# 8 i + x); st0 = default-policy output stores
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
L=build/abl/nsh_fir_mfma
DECIM=4 timeout -k 10 300 python tools/probe/lib_abn.py ${L}_b0.so ${L}_nt4.so ${L}_xw.so ${L}_st0.so > $O/d4_1.log 2>&1 || exit 1
DECIM=4 timeout -k 10 300 python tools/probe/lib_abn.py ${L}_st0.so ${L}_xw.so ${L}_nt4.so ${L}_b0.so > $O/d4_2.log 2>&1 || exit 1
echo ok
