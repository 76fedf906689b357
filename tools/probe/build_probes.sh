#!/bin/bash
# Build the standalone probe binaries next to their sources (git-ignored; gfx950 only).
# Usage: tools/probe/build_probes.sh [name ...]   (default: every tools/probe/*.hip)
set -e
cd "$(dirname "$0")"
names=("$@")
[ ${#names[@]} -eq 0 ] && names=($(ls *.hip | sed 's/\.hip$//'))
for n in "${names[@]}"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o "$n" "$n.hip"
done
