#!/bin/bash
# round 4: k_fir_exact12's cost on ordinary input (empty queue) against its grid: 5 (kept), 2 and 1
# workgroups per CU (NSH_X12_PER_CU probe builds), lib_abn over the three builds under
# rocprofv3 --kernel-trace (the follow-up's duration per build, told apart by grid size)
export TMPDIR=/tmp
O=gpurun_out/r04zu; mkdir -p $O
A=build/abl/nsh_fir_mfma_x5.so; B=build/abl/nsh_fir_mfma_x1.so; C=build/abl/nsh_fir_mfma_x2.so
ROUNDS=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o t -- python3 tools/probe/lib_abn.py $A $B $C $A $B $C > $O/ab.log 2>&1 || exit 1
