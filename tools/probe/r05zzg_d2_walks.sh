#!/bin/bash
# round 5: decim 2 -- the contiguous walk (k_fir_mfma11, mask 0, the default) vs the lockstep walk
# with whole-line chunk loads (k_fir_mfma13, mask 4) on the in-tree build; four A/Bs alternating.
export TMPDIR=/tmp
O=gpurun_out/r05zzg; mkdir -p $O
for i in 1 2; do
  DECIM=2 MASKS=0,4:2 ROUNDS=12 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2_${i}a.log 2>&1 &&
  DECIM=2 MASKS=4:2,0 ROUNDS=12 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2_${i}b.log 2>&1 || exit 1
done
echo "rc=$?"
