#!/bin/bash
# round 5: k_fir_mfma11 (the contiguous walk: D = 2 default, D = 4 with NSH_DEC_WALK_MASK=0) with
# k_fir_mfma13's whole-line nontemporal chunk loads (c: NSH_V11_CLOAD=1) vs the strided loads (b);
# lib_abn both orders, synth and every-4th-chunk-exact input (outputs must be bit-identical).
export TMPDIR=/tmp
O=gpurun_out/r05zzf; mkdir -p $O
L=build/abl/nsh_fir_mfma
DECIM=2 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_b.so ${L}_c.so > $O/d2_a.log 2>&1 &&
DECIM=2 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c.so ${L}_b.so > $O/d2_b.log 2>&1 &&
DECIM=2 INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_b.so ${L}_c.so > $O/d2_spike4.log 2>&1 &&
NSH_DEC_WALK_MASK=0 DECIM=4 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_b.so ${L}_c.so > $O/d4_a.log 2>&1 &&
NSH_DEC_WALK_MASK=0 DECIM=4 INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_b.so ${L}_c.so > $O/d4_spike4.log 2>&1
echo "rc=$?"
