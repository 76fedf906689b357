#!/bin/bash
# round 5, timing only: k_fir_pfft2 (loads at the frame top) vs row-load instructions of one
# contiguous 1 KiB (wrong rows) vs no row loads at all; both build orders.
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
ROUNDS=8 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_def.so build/abl/pfft_contig.so build/abl/pfft_noload.so > $O/ab.log 2>&1 &&
ROUNDS=8 timeout -k 10 180 python -u tools/probe/pfft_ab.py build/abl/pfft_noload.so build/abl/pfft_contig.so build/abl/pfft_def.so > $O/ab_rev.log 2>&1
echo "rc=$?"
