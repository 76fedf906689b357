#!/bin/bash
# round 5: the in-tree build with NSH_V13_CLOAD + nontemporal chunk loads (the r05ze winner) --
# decimator tests, then the walks (k_fir_mfma11 mask 0 vs k_fir_mfma13) at D = 4 / 2, both orders,
# and D = 4 with every 64th chunk exact; the committed form (build/abl c0) beside it at D = 4.
export TMPDIR=/tmp
O=gpurun_out/r05zf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "decim" --timeout 120 --timeout-method thread > $O/pytest_decim.log 2>&1 && echo "decim tests ok" &&
DECIM=4 MASKS=0,16:2 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4.log 2>&1 &&
DECIM=2 MASKS=0,4:2 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2.log 2>&1 &&
DECIM=2 MASKS=4:2,0 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d2_rev.log 2>&1 &&
DECIM=4 INPUT=spike64 MASKS=0,16:2 timeout -k 10 200 python tools/probe/walk_ab.py > $O/d4_spike64.log 2>&1 &&
DECIM=4 timeout -k 10 200 python tools/probe/lib_abn.py build/abl/nsh_fir_mfma_c0.so newsched_amd/lib/libnsh_hip.so > $O/d4_lib.log 2>&1
echo "rc=$?"
