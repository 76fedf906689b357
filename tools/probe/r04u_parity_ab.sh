#!/bin/bash
# round 4: the exact queue as two parity sets, k_fir_exact12 zeroing the next launch's counters
# (par) against the done-counter reset (q64), the single kernel (base) and no exact code (nx);
# rocprof of par on the 1-in-256 stream; then the exact-path GPU tests
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
A=build/abl/nsh_fir_mfma_base.so; Q=build/abl/q64.so; P=build/abl/par.so; NX=build/abl/nsh_fir_mfma_nx.so
timeout -k 10 200 python tools/probe/lib_abn.py $A $P $Q $NX > $O/ab_synth_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/lib_abn.py $NX $Q $P $A > $O/ab_synth_2.log 2>&1 &&
INPUT=spike256 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $A $P $Q > $O/ab_spike256.log 2>&1 &&
INPUT=spike64 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $Q $P $A > $O/ab_spike64.log 2>&1 &&
INPUT=spike4 ROUNDS=6 timeout -k 10 200 python tools/probe/lib_abn.py $P $A $Q > $O/ab_spike4.log 2>&1 &&
INPUT=spike1 ROUNDS=4 timeout -k 10 200 python tools/probe/lib_abn.py $A $P > $O/ab_spike1.log 2>&1 &&
INPUT=spike256 ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s256 -o run --output-format csv -- python3 tools/probe/lib_abn.py $P > $O/s256.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fir" > $O/pytest_fir.log 2>&1
