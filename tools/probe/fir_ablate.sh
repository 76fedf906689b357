#!/bin/bash
# Build (here) the FIR ablation probes: one binary per NSH_FIR_ABLATE mask, linked against
# the library sources compiled with that mask. Run them on the GPU box: fir_ablate_<mask>.
set -e
cd "$(dirname "$0")/../.."
for m in ${MASKS:-0 1 2 4 8 3 9 6}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DNSH_FIR_ABLATE=$m \
    newsched_amd/csrc/nsh_runtime.hip newsched_amd/csrc/nsh_stream.hip newsched_amd/csrc/nsh_fir.hip \
    newsched_amd/csrc/nsh_fir_mfma.hip tools/probe/fir_ablate.cpp -o tools/probe/fir_ablate_$m &
done
wait
