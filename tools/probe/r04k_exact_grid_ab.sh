#!/bin/bash
# round 4: k_fir_exact12's occupancy / prefetch on exact-heavy streams (spike1: every chunk on the
# fp32 tile; nan1 via cliff) against the single-kernel form (base), and the empty follow-up's cost
# on the ordinary stream (x1: 256 workgroups; x5 (default): 1280)
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; X5=build/abl/x5.so; X4P=build/abl/nsh_fir_mfma_x4pf.so; X6=build/abl/nsh_fir_mfma_x6.so; X1=build/abl/nsh_fir_mfma_x1.so; NX=build/abl/nsh_fir_mfma_nx.so
INPUT=spike1 ROUNDS=4 timeout -k 10 200 python tools/probe/lib_abn.py $A $X5 $X4P $X6 > $O/ab_spike1_1.log 2>&1 &&
INPUT=spike1 ROUNDS=4 timeout -k 10 200 python tools/probe/lib_abn.py $X6 $X4P $X5 $A > $O/ab_spike1_2.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $A $X5 $X4P $X6 > $O/ab_spike4_1.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $X6 $X4P $X5 $A > $O/ab_spike4_2.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $NX $X5 $X1 $A > $O/ab_synth_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $A $X1 $X5 $NX > $O/ab_synth_2.log 2>&1 &&
timeout -k 10 300 python -u tools/probe/cliff.py --reps 5 > $O/cliff.log 2>&1
