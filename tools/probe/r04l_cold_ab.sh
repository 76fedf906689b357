#!/bin/bash
# round 4: k_fir_mfma12 with the exact forms in an early-returning cold branch (cold) against the
# queue + k_fir_exact12 form (x5), the single-kernel form with shared staging (base) and no exact
# code (nx, timing only); ordinary stream in both orders, exact-heavy streams
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; X5=build/abl/x5.so; C=build/abl/nsh_fir_mfma_cold.so; NX=build/abl/nsh_fir_mfma_nx.so
timeout -k 10 200 python tools/probe/lib_abn.py $A $C $X5 $NX > $O/ab_synth_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $NX $X5 $C $A > $O/ab_synth_2.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $X5 $A $NX $C > $O/ab_synth_3.log 2>&1 &&
INPUT=spike1 ROUNDS=4 timeout -k 10 200 python tools/probe/lib_abn.py $A $C $X5 > $O/ab_spike1.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $C $A $X5 > $O/ab_spike4.log 2>&1 &&
INPUT=spike64 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $X5 $C $A > $O/ab_spike64.log 2>&1
