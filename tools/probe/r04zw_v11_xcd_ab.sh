#!/bin/bash
# round 4: the decimators' chunk walk -- one contiguous range per persistent workgroup (c0, the
# kept form) vs XCD-interleaved with rotated windows at D = 4 (x4: NSH_V11_XCD=4); lib_abn after
# its 2 s warm-up, ABAB / BABA, D = 4 (and D = 2, where both builds run the contiguous walk);
# ordinary input and every 64th / 4th chunk exact (spike64, spike4)
export TMPDIR=/tmp
O=gpurun_out/r04zw; mkdir -p $O
A=build/abl/nsh_fir_mfma_c0.so; B=build/abl/nsh_fir_mfma_x4.so
DECIM=4 timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/b_d4_1.log 2>&1 || exit 1
DECIM=4 timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/b_d4_2.log 2>&1 || exit 1
DECIM=4 INPUT=spike64 timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/b_d4_spike64.log 2>&1 || exit 1
DECIM=4 INPUT=spike4 timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/b_d4_spike4.log 2>&1 || exit 1
DECIM=2 timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/b_d2_1.log 2>&1 || exit 1
