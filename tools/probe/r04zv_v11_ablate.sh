#!/bin/bash
# round 4, timing only: what bounds k_fir_mfma11 -- probe builds with NSH_V11_ABLATE = 1 (no MFMA
# tile), 2 (no LDS staging of the next chunk), 4 (no output stores), 3 (neither MFMA nor staging)
# vs the product form (a0); lib_abn after its 2 s warm-up, D = 4 and 2, two orders
export TMPDIR=/tmp
O=gpurun_out/r04zv; mkdir -p $O
B=build/abl/nsh_fir_mfma
for D in 4 2; do
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py ${B}_a0.so ${B}_a1.so ${B}_a2.so ${B}_a4.so ${B}_a3.so ${B}_a0.so > $O/ab_d${D}_1.log 2>&1 || exit 1
  DECIM=$D timeout -k 10 200 python tools/probe/lib_abn.py ${B}_a0.so ${B}_a3.so ${B}_a4.so ${B}_a2.so ${B}_a1.so ${B}_a0.so > $O/ab_d${D}_2.log 2>&1 || exit 1
done
