#!/bin/bash
# The clock each kernel ran at, measured: one rocprofv3 pass with the GRBM counters and the kernel
# trace (no other tracing domain), summarised by tools/clock_summary.py as
# GRBM_GUI_ACTIVE / 8 XCDs / kernel duration per dispatch (MI355X_MICROARCH.md, DVFS give-back).
# Usage (on the GPU box): tools/pmc_clock.sh OUTDIR [fir_one.py args...]
set -e
OUT=${1:-gpurun_out/clock}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/p" -o run --output-format csv \
  -- python3 tools/fir_one.py "$@" > "$OUT/run.log" 2>&1
python3 tools/clock_summary.py "$OUT/p" > "$OUT/clock.json"
cat "$OUT/clock.json"
