#!/bin/bash
# round 4: the decimators' register prefetch one chunk deeper (NSH_V11_DEPTH=4: chunk ch+2's
# scale reduction waits on loads issued two steps earlier instead of one), ABAB / BABA after
# lib_abn's 2 s warm-up, D = 2 and 4, 127 taps
export TMPDIR=/tmp
O=gpurun_out/r04zh; mkdir -p $O
A=build/abl/nsh_fir_mfma_d3.so; B=build/abl/nsh_fir_mfma_d4.so
for D in 4 2; do
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_d${D}_1.log 2>&1 || exit 1
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_d${D}_2.log 2>&1 || exit 1
done
