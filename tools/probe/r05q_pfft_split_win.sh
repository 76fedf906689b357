#!/bin/bash
# round 5: k_fir_pfft's ring-order window reads as single ds_read_b64 (w1, NSH_PFFT_SPLIT_WIN=1) vs
# paired ds_read2st64_b64 (w0, round 4), both orders; PMC of the default build (w1) on the fused chain.
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_w1.so build/abl/pfft_w0.so > $O/ab.log 2>&1 &&
ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_w0.so build/abl/pfft_w1.so > $O/ab_rev.log 2>&1 &&
tools/pmc_fir.sh $O/pmc_casc --algo casc && python3 tools/pmc_summary.py $O/pmc_casc $((1<<25)) $O/pmc_casc.json > /dev/null
echo "rc=$?"
