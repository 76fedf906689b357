#!/bin/bash
# round 5: decim 1 on k_fir_mfma13's lockstep walk (NSH_DEC_WALK_MASK bit 1: the polyphase form with
# one phase = Toeplitz on 16-sample blocks, K = 144 for 127 taps, 16x16x32 MFMAs, taps in VGPRs,
# persistent workgroups) vs k_fir_mfma12 (mask 0), 2 / 3 workgroups per CU, both orders, and with
# every 64th chunk exact.
export TMPDIR=/tmp
O=gpurun_out/r05zk; mkdir -p $O
DECIM=1 MASKS=0,18:2,18:3 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d1.log 2>&1 &&
DECIM=1 MASKS=18:3,18:2,0 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d1_rev.log 2>&1 &&
DECIM=1 INPUT=spike64 MASKS=0,18:2 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d1_spike64.log 2>&1
echo "rc=$?"
