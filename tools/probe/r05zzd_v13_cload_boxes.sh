#!/bin/bash
# round 5: k_fir_mfma13 D = 4, whole-line chunk loads + nt (c1nt, profiles/r05ze_v13_cload.patch.txt) vs
# the committed strided loads (c0) on another box: four two-library A/Bs alternating the order.
export TMPDIR=/tmp
O=gpurun_out/r05zzd; mkdir -p $O
L=build/abl/nsh_fir_mfma
for i in 1 2; do
  DECIM=4 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1nt.so > $O/d4_${i}a.log 2>&1 &&
  DECIM=4 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c1nt.so ${L}_c0.so > $O/d4_${i}b.log 2>&1 || exit 1
done
echo "rc=$?"
