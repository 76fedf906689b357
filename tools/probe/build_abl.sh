#!/bin/bash
# Timing-only ablation builds of libnsh_hip.so (NSH_FIR_ABLATE masks, see nsh_fir_mfma.hip):
# build/abl/lib_<mask>.so for each mask given. Run on the CPU (hipcc cross-compiles).
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/abl
for m in "$@"; do
  mkdir -p build/abl/o_$m
  for f in newsched_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -DNSH_FIR_ABLATE=$m \
      -c $f -o build/abl/o_$m/$(basename $f .hip).o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/lib_$m.so build/abl/o_$m/*.o
done
