#!/bin/bash
# round 4: k_fir_pfft reading each window in ring order (rotated; ro1) against window order (ro0),
# C5's chain over 2^28 inputs, both build orders; then the pfft / cascade GPU tests on ro1 (in-tree)
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
A=build/abl/nsh_fir_pfft_ro0.so; B=build/abl/nsh_fir_pfft_ro1.so
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $A $B $A $B > $O/ab_1.log 2>&1 &&
KIND=casc timeout -k 10 200 python tools/probe/lib_abn.py $B $A $B $A > $O/ab_2.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_pfft.py -x -q --timeout 200 --timeout-method thread > $O/pytest_pfft.log 2>&1
