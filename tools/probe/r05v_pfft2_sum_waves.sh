#!/bin/bash
# round 5: k_fir_pfft2 (loads after B1) with the phase sum on waves 8..15 (u0, default) or on
# waves 0..7 (u1: the low-priority waves that wait longest at load issue then carry no sum);
# parity of u1's form 2 first (the pfft suite against build/abl/pfft_u1.so via NSH_HIP_LIB).
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
NSH_HIP_LIB=build/abl/pfft_u1.so NSH_PFFT_FORM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x -k form2 --timeout 120 --timeout-method thread > $O/pytest_u1.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_u0.so build/abl/pfft_u1.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_u1.so build/abl/pfft_u0.so > $O/ab_rev.log 2>&1
echo "rc=$?"
