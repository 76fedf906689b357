#!/bin/bash
# round 4: k_fir_mfma12's chunk-order rotation (NSH_V12_ROT) once the exact chunks left the kernel
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
A=build/abl/nsh_fir_mfma_cur.so; B=build/abl/nsh_fir_mfma_rot0.so
timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_2.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $A $B > $O/ab_spike4.log 2>&1
