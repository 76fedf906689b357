#!/bin/bash
# round 4: k_fir_pfft phase B in 16-B LDS accesses -- the phase sum from ds_read_b128 (M/2 threads,
# two bins each; NSH_PFFT_SUM128) and the next rows' ring stores as ds_write_b128 (NSH_PFFT_RING128);
# C5's chain (KIND=casc), lib_abn after its 2 s warm-up, two orders
export TMPDIR=/tmp
O=gpurun_out/r04zj; mkdir -p $O
A=build/abl/pfft_base.so; S=build/abl/pfft_s128.so; R=build/abl/pfft_r128.so; B=build/abl/pfft_both.so
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $A $S $R $B $A > $O/ab_1.log 2>&1 || exit 1
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $B $R $S $A $B > $O/ab_2.log 2>&1 || exit 1
