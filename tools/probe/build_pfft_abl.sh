#!/bin/bash
# Builds of libnsh_hip.so that differ only in nsh_fir_pfft.hip's compile flags:
# build/abl/pfft_<tag>.so for each "tag:FLAGS" argument (e.g. "a1:-DNSH_PFFT_ABLATE=1").
# Needs `make hip` first (reuses the other objects). Run on the CPU.
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/abl
OTHERS=$(ls build/obj/hip/*.o | grep -v nsh_fir_pfft.o)
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude $flags \
    -c newsched_amd/csrc/nsh_fir_pfft.hip -o build/abl/pfft_$tag.o &
done
wait
for spec in "$@"; do
  tag=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/pfft_$tag.so $OTHERS build/abl/pfft_$tag.o
done
