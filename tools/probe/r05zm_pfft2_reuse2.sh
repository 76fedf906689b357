#!/bin/bash
# round 5: k_fir_pfft2 with the frame hop of whole 64-row blocks again (V = 384 at C5, the last two
# blocks kept in registers: 3 row loads per lane and frame), now on the load-k = blocks 2k, 2k+1
# mapping (r05zj) with every remaining load nontemporal; r0 = NSH_PFFT2_REUSE=0 (the committed
# form), r1 = reuse (the in-tree build). pfft suite on the in-tree build first; A/B both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zm; mkdir -p $O
L=build/abl/pfft
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 && echo "pfft tests ok" &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_r0.so ${L}_r1.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_r1.so ${L}_r0.so > $O/ab2.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_r0.so ${L}_r1.so > $O/ab3.log 2>&1
echo "rc=$?"
