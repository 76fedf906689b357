#!/bin/bash
# round 5: k_fir_mfma12's tap-fragment LDS reads -- a0 = the product build, ab = timing-only build
# with the B fragments as register values (no LDS reads; wrong outputs); lib_abn both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zza; mkdir -p $O
L=build/abl/nsh_fir_mfma
DECIM=1 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_a0.so ${L}_ab.so > $O/ab1.log 2>&1 &&
DECIM=1 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_ab.so ${L}_a0.so > $O/ab2.log 2>&1
echo "rc=$?"
