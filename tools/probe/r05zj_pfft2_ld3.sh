#!/bin/bash
# round 5: k_fir_pfft2 with load k holding row blocks 2k, 2k+1 (the next frame's overlap rows all
# in load 3): ld3 = loads 0..2 nontemporal, load 3 default (the in-tree build); ld3d = the same
# mapping, default policy everywhere; base = HEAD; lo2 = HEAD's mapping with loads 0, 1 nt (r05zi).
# The pfft suite on the in-tree build, A/B both orders, PMC of the in-tree build.
export TMPDIR=/tmp
O=gpurun_out/r05zj; mkdir -p $O
L=build/abl/pfft
timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pfft.log 2>&1 && echo "pfft tests ok" &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_base.so ${L}_ld3.so ${L}_ld3d.so ${L}_lo2.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_lo2.so ${L}_ld3d.so ${L}_ld3.so ${L}_base.so > $O/ab2.log 2>&1 &&
tools/pmc_fir.sh $O/pmc --algo casc > /dev/null && python3 tools/pmc_summary.py $O/pmc $((1<<25)) $O/pmc.json > /dev/null
echo "rc=$?"
