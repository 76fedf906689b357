#!/bin/bash
# round 4: k_fir_pfft with the next window's rows requested in phase B right after the previous
# rows went into the ring (NSH_PFFT_LOAD_IN_B=1) vs at the top of the transform phase; C5's chain
# (KIND=casc), lib_abn after its 2 s warm-up, ABAB / BABA
export TMPDIR=/tmp
O=gpurun_out/r04zk; mkdir -p $O
A=build/abl/pfft_base.so; B=build/abl/pfft_lib.so
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_1.log 2>&1 || exit 1
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_2.log 2>&1 || exit 1
