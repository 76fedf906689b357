#!/bin/bash
# round 4: the exact queue split into 64 sub-queues (q64) against one counter (x5), the single-kernel
# form (base) and no exact code (nx); then the FIR GPU tests on the in-tree build
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; X5=build/abl/x5.so; Q=build/abl/q64.so; NX=build/abl/nsh_fir_mfma_nx.so
timeout -k 10 200 python tools/probe/lib_abn.py $A $Q $X5 $NX > $O/ab_synth_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $NX $X5 $Q $A > $O/ab_synth_2.log 2>&1 &&
INPUT=spike1 ROUNDS=4 timeout -k 10 200 python tools/probe/lib_abn.py $A $Q $X5 > $O/ab_spike1.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $Q $A $X5 > $O/ab_spike4.log 2>&1 &&
INPUT=spike64 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $X5 $Q $A > $O/ab_spike64.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fir" > $O/pytest_fir.log 2>&1
