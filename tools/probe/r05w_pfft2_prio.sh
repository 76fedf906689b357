#!/bin/bash
# round 5: k_fir_pfft2 (phase sum on waves 0..7, loads after B1) with s_setprio in phase A:
# p0 none; p1 waves 8..15 at 1; p2 waves 12..15 at 2, 8..11 at 1; p3 the inverse wave at 3 for its
# inverse. NSH_PFFT_FORM=2; both orders. Then both forms of the default build.
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_p0.so build/abl/pfft_p1.so build/abl/pfft_p2.so build/abl/pfft_p3.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_p3.so build/abl/pfft_p2.so build/abl/pfft_p1.so build/abl/pfft_p0.so > $O/ab_rev.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/forms.log 2>&1
echo "rc=$?"
