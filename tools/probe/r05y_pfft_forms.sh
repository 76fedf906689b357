#!/bin/bash
# round 5: the two C5 forms of the current build (k_fir_pfft2: phase sum on waves 0..7, loads after
# B1), 3 x 10 interleaved rounds at 2^28; the form-2 phase trace (build/abl/pfft_trace.so).
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
for i in 1 2 3; do LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/forms_$i.log 2>&1 || exit 1; done &&
NSH_PFFT_FORM=2 TRACE_OUT=$O/trace2.npy timeout -k 10 180 python -u tools/probe/pfft2_trace.py build/abl/pfft_trace.so > $O/trace2.log 2>&1
echo "rc=$?"
