#!/bin/bash
# round 4: k_fir_mfma12 with the exact chunks in a follow-up kernel (split) vs the single kernel
# (base) and the no-exact timing probe (nx); the decimators the same way (split11: k_fir_mfma11 +
# k_fir_exact11; split: exact forms inside k_fir_mfma11; v11nx: no exact code, timing only)
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; B=build/abl/nsh_fir_mfma_split.so; C=build/abl/nsh_fir_mfma_nx.so
timeout -k 10 150 python tools/probe/lib_abn.py $A $B $C > $O/ab_synth1.log 2>&1 &&
timeout -k 10 150 python tools/probe/lib_abn.py $C $B $A > $O/ab_synth2.log 2>&1 &&
INPUT=spike4 timeout -k 10 150 python tools/probe/lib_abn.py $A $B > $O/ab_spike4.log 2>&1 &&
INPUT=spike1 ROUNDS=6 timeout -k 10 150 python tools/probe/lib_abn.py $A $B > $O/ab_spike1.log 2>&1 &&
E=build/abl/nsh_fir_mfma_split11.so; F=build/abl/nsh_fir_mfma_v11nx.so
DECIM=2 timeout -k 10 150 python tools/probe/lib_abn.py $B $E $F > $O/ab_d2_1.log 2>&1 &&
DECIM=2 timeout -k 10 150 python tools/probe/lib_abn.py $F $E $B > $O/ab_d2_2.log 2>&1 &&
DECIM=4 timeout -k 10 150 python tools/probe/lib_abn.py $B $E $F > $O/ab_d4_1.log 2>&1 &&
DECIM=4 timeout -k 10 150 python tools/probe/lib_abn.py $F $E $B > $O/ab_d4_2.log 2>&1 &&
DECIM=2 INPUT=spike4 timeout -k 10 150 python tools/probe/lib_abn.py $B $E > $O/ab_d2_spike4.log 2>&1 &&
DECIM=4 INPUT=spike4 timeout -k 10 150 python tools/probe/lib_abn.py $B $E > $O/ab_d4_spike4.log 2>&1 &&
P=build/abl/nsh_fir_mfma_p64.so; X=build/abl/nsh_fir_mfma_x2.so
timeout -k 10 150 python tools/probe/lib_abn.py $E $P > $O/ab_p64_1.log 2>&1 &&
timeout -k 10 150 python tools/probe/lib_abn.py $P $E > $O/ab_p64_2.log 2>&1 &&
INPUT=spike1 ROUNDS=4 timeout -k 10 150 python tools/probe/lib_abn.py $E $X > $O/ab_x2_spike1.log 2>&1 &&
timeout -k 10 300 python -u tools/probe/cliff.py --reps 5 > $O/cliff.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
