#!/bin/bash
# round 5: k_fir_pfft2 phase trace (build/abl/pfft_trace.so, -DNSH_PFFT_TRACE=1) and the PMC passes
# of tools/pmc_fir.sh on the fused chain for form 2 (default) and form 1 (NSH_PFFT_FORM=1).
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
TRACE_OUT=$O/trace2.npy timeout -k 10 180 python -u tools/probe/pfft2_trace.py build/abl/pfft_trace.so > $O/trace2.log 2>&1 &&
tools/pmc_fir.sh $O/pmc2 --algo casc && python3 tools/pmc_summary.py $O/pmc2 $((1<<25)) $O/pmc2.json > /dev/null &&
NSH_PFFT_FORM=1 tools/pmc_fir.sh $O/pmc1 --algo casc && python3 tools/pmc_summary.py $O/pmc1 $((1<<25)) $O/pmc1.json > /dev/null
echo "rc=$?"
