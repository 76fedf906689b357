#!/bin/bash
# round 5: k_fir_pfft2's row-load cache policy -- b0 = default policy on all four loads (committed),
# lo2 = nontemporal on loads 0, 1 (rows never read again), all2 = nontemporal on all four: timing
# A/B both orders, then HBM bytes per input (PMC passes) for each build (swapped in as the in-tree
# library in this scratch copy of the tree).
export TMPDIR=/tmp
O=gpurun_out/r05zi; mkdir -p $O
L=build/abl/pfft
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_b0.so ${L}_lo2.so ${L}_all2.so > $O/ab1.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 150 python -u tools/probe/pfft_ab.py ${L}_all2.so ${L}_lo2.so ${L}_b0.so > $O/ab2.log 2>&1 || exit 1
for v in b0 lo2 all2; do
  cp ${L}_$v.so newsched_amd/lib/libnsh_hip.so &&
  tools/pmc_fir.sh $O/pmc_$v --algo casc > /dev/null && python3 tools/pmc_summary.py $O/pmc_$v $((1<<25)) $O/pmc_$v.json > /dev/null || exit 1
done
echo "rc=$?"
