#!/bin/bash
# Separate rocprofv3 --pmc passes (never combined with tracing domains) over tools/fir_one.py.
# Usage (on the GPU box): tools/pmc_fir.sh OUTDIR [fir_one.py args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 tools/fir_one.py "$@" > "$OUT/p$i.log" 2>&1
done
echo "pmc passes done: $i"
