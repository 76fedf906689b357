#!/bin/bash
# round 4: does pacing the copy's stores move its rate? k_copy_v4 with s_sleep N (64 N cycles)
# between a step's loads and its stores (NSH_COPY_SLEEP probe builds) vs the kept form, with the
# 4-stage multiply_const chain (same shape, VALU between loads and stores) beside it;
# tools/probe/stream_ab.py. Run 1 (ab_1, ab_2): 4 builds, 10-pass warm-up; run 2 (ab_3, ab_4):
# base vs sleep 16, ABAB / BABA after a 2 s warm-up.
export TMPDIR=/tmp
O=gpurun_out/r04zs; mkdir -p $O
B=build/abl/nsh_stream
timeout -k 10 200 python tools/probe/stream_ab.py ${B}_base.so ${B}_sl16.so ${B}_base.so ${B}_sl16.so > $O/ab_3.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe/stream_ab.py ${B}_sl16.so ${B}_base.so ${B}_sl16.so ${B}_base.so > $O/ab_4.log 2>&1 || exit 1
