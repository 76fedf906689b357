#!/bin/bash
# round 5: k_fir_pfft2 row loads split over phase A: v1 half after B1 and half after pass 2, v2 the
# same for waves 8..15 only, v0 all after B1 (default); parity of v1 and v2 (form 2) first.
set -o pipefail
O=gpurun_out/r05zb; mkdir -p $O
NSH_HIP_LIB=build/abl/pfft_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x -k form2 --timeout 120 --timeout-method thread > $O/pytest_v1.log 2>&1 &&
NSH_HIP_LIB=build/abl/pfft_v2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pfft.py -q -x -k form2 --timeout 120 --timeout-method thread > $O/pytest_v2.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_v0.so build/abl/pfft_v1.so build/abl/pfft_v2.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=10 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_v2.so build/abl/pfft_v1.so build/abl/pfft_v0.so > $O/ab_rev.log 2>&1
echo "rc=$?"
