#!/bin/bash
# round 4: what the decimators' exact forms cost k_fir_mfma11 on ordinary input (timing probe with them
# compiled out), ABAB / BABA after lib_abn's 2 s warm-up, D = 2 and 4
export TMPDIR=/tmp
O=gpurun_out/r04y; mkdir -p $O
A=build/abl/nsh_fir_mfma_v11cur.so; B=build/abl/nsh_fir_mfma_v11nx.so
for D in 2 4; do
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_d${D}_1.log 2>&1 || exit 1
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_d${D}_2.log 2>&1 || exit 1
done
