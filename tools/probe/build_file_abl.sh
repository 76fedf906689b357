#!/bin/bash
# Builds of libnsh_hip.so that differ only in one source file's compile flags:
# build/abl/<stem>_<tag>.so for each "tag:FLAGS" argument. Usage:
#   tools/probe/build_file_abl.sh nsh_fir_mfma "p0:" "p4k:-DNSH_V12_LDS_PAD=4096"
# Needs `make hip` first (reuses the other objects). Run on the CPU.
set -e
cd "$(dirname "$0")/../.."
stem=$1; shift
mkdir -p build/abl
OTHERS=$(ls build/obj/hip/*.o | grep -v "/$stem.o")
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude $flags \
    -c newsched_amd/csrc/$stem.hip -o build/abl/${stem}_$tag.o &
done
wait
for spec in "$@"; do
  tag=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/${stem}_$tag.so $OTHERS build/abl/${stem}_$tag.o
done
