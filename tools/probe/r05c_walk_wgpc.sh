#!/bin/bash
# round 5: k_fir_mfma13's lockstep row width -- 2, 3 or 4 resident workgroups per CU (NSH_WALK_WGPC)
# against k_fir_mfma11, D = 4 and 2, both orders
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
DECIM=4 MASKS=0,16:2,16:3,16:4 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4.log 2>&1 || exit 1
DECIM=4 MASKS=16:4,16:3,16:2,0 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_rev.log 2>&1 || exit 1
DECIM=2 MASKS=0,4:2,4:3 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2.log 2>&1 || exit 1
DECIM=4 INPUT=spike64 MASKS=0,16:2,16:3 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_spike64.log 2>&1 || exit 1
echo ok
