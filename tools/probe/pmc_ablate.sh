#!/bin/bash
# PMC passes over the FIR ablation probes (fir_ablate.sh). Usage on the GPU box:
#   tools/probe/pmc_ablate.sh OUTDIR MASK...
set -e
OUT=$1; shift
export TMPDIR=/tmp
for m in "$@"; do
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d "$OUT/m$m/p$i" -o run --output-format csv -- tools/probe/fir_ablate_$m $m > "$OUT/m$m/p$i.log" 2>&1 || { echo "pass $i mask $m failed"; exit 1; }
  done
done
echo done
