#!/bin/bash
# round 4, timing only: k_fir_pfft<16,1> whose per-frame row loads always fetch the same rows
# (NSH_PFFT_ABLATE=256: L2 hits, same issue cost, no HBM latency; outputs wrong) vs the product
# kernel -- does phase B wait on the next rows' HBM latency?
export TMPDIR=/tmp
O=gpurun_out/r04zl; mkdir -p $O
A=build/abl/pfft_base.so; B=build/abl/pfft_l2hit.so
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_1.log 2>&1 || exit 1
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_2.log 2>&1 || exit 1
