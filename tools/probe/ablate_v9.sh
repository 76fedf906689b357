#!/bin/bash
# v9 ablations (built by hand into build/abl/lib_<mask>.so, NSH_FIR_ABLATE masks: 256 no MFMA,
# 512 no split VALU, 768 both, 1024 no global loads, 2048 one store per lane-chunk), each
# A/B'd in one process against the real library at 2^28 samples.
set -o pipefail
mkdir -p gpurun_out/abl
for m in 256 512 768 1024 2048; do
  DECIMS=1 ROUNDS=8 timeout -k 10 100 python -u tools/probe/lib_ab.py newsched_amd/lib/libnsh_hip.so build/abl/lib_$m.so > gpurun_out/abl/m$m.log 2>&1 || exit 1
  grep "D=1" gpurun_out/abl/m$m.log | sed "s/^/mask=$m /"
done
