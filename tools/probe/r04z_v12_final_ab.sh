#!/bin/bash
# round 4, final: k_fir_mfma12 + k_fir_exact12 (cur: two counter sets; any: + the one-word "anything
# queued" flag) against the round-3 single kernel (base) and the no-exact-code timing probe (nx),
# both orders after lib_abn's 2 s warm-up; exact-heavy inputs for any vs base
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; B=build/abl/cur.so; Y=build/abl/any.so; N=build/abl/nsh_fir_mfma_nx.so
timeout -k 10 200 python tools/probe/lib_abn.py $A $B $Y $N > $O/ab_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $N $Y $B $A > $O/ab_2.log 2>&1 &&
INPUT=spike256 timeout -k 10 200 python tools/probe/lib_abn.py $A $Y > $O/ab_spike256.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $A $Y > $O/ab_spike4.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fir" > $O/pytest_fir.log 2>&1
