#!/bin/bash
# round 5: PMC passes (tools/pmc_fir.sh) on the fused C5 chain, k_fir_pfft2 (default) and
# k_fir_pfft (NSH_PFFT_FORM=1): HBM bytes per input sample (are the re-read overlap rows L2 hits?)
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
tools/pmc_fir.sh $O/pmc2 --algo casc && python3 tools/pmc_summary.py $O/pmc2 $((1<<25)) $O/pmc2.json > /dev/null &&
NSH_PFFT_FORM=1 tools/pmc_fir.sh $O/pmc1 --algo casc && python3 tools/pmc_summary.py $O/pmc1 $((1<<25)) $O/pmc1.json > /dev/null
echo "rc=$?"
