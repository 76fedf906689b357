#!/bin/bash
# round 4: k_fir_pfft's exchange 2 in registers (permlane / DPP swaps, NSH_PFFT_REGX2) on top of the
# ring-order window, ABAB / BABA after lib_abn's 2 s warm-up, C5's chain over 2^28 inputs
export TMPDIR=/tmp
O=gpurun_out/r04za; mkdir -p $O
A=build/abl/nsh_fir_pfft_rx0.so; B=build/abl/nsh_fir_pfft_rx2.so
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_1.log 2>&1 &&
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_2.log 2>&1
