#!/bin/bash
# round 5: k_fir_pfft2's row loads -- at the frame top (t0) or after B1 (t1), default policy or
# nontemporal (nt); NSH_PFFT_FORM=2 for every plan; then both forms of the default build.
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_t0.so build/abl/pfft_t0nt.so build/abl/pfft_t1.so build/abl/pfft_t1nt.so > $O/ab.log 2>&1 &&
NSH_PFFT_FORM=2 ROUNDS=8 timeout -k 10 240 python -u tools/probe/pfft_ab.py build/abl/pfft_t1nt.so build/abl/pfft_t1.so build/abl/pfft_t0nt.so build/abl/pfft_t0.so > $O/ab_rev.log 2>&1 &&
LOG2N=28 ROUNDS=10 timeout -k 10 180 python -u tools/probe/pfft_form_ab.py > $O/forms.log 2>&1
echo "rc=$?"
