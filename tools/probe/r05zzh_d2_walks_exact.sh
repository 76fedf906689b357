#!/bin/bash
# round 5: decim 2 walks with exact chunks -- every 64th / every 4th 2048-input chunk holds a 2^40
# spike (the exact path): k_fir_mfma11 (mask 0) vs k_fir_mfma13 (mask 4), both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zzh; mkdir -p $O
DECIM=2 INPUT=spike64 MASKS=0,4:2 ROUNDS=8 timeout -k 10 200 python tools/probe/walk_ab.py > $O/s64a.log 2>&1 &&
DECIM=2 INPUT=spike64 MASKS=4:2,0 ROUNDS=8 timeout -k 10 200 python tools/probe/walk_ab.py > $O/s64b.log 2>&1 &&
DECIM=2 INPUT=spike4 MASKS=0,4:2 ROUNDS=6 timeout -k 10 200 python tools/probe/walk_ab.py > $O/s4a.log 2>&1 &&
DECIM=2 INPUT=spike4 MASKS=4:2,0 ROUNDS=6 timeout -k 10 200 python tools/probe/walk_ab.py > $O/s4b.log 2>&1
echo "rc=$?"
