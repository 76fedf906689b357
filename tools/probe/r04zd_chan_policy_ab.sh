#!/bin/bash
# round 4: the channelizer's (and fft1024's) cache policy on its frame loads / stores (nt = 2, default
# = 0), one TU built four ways, both orders
export TMPDIR=/tmp
O=gpurun_out/r04zd; mkdir -p $O
P=build/abl/nsh_fft_
timeout -k 10 200 python tools/probe/chan_libs_ab.py ${P}l2s2.so ${P}l0s2.so ${P}l2s0.so ${P}l0s0.so > $O/chan_1.log 2>&1 &&
timeout -k 10 200 python tools/probe/chan_libs_ab.py ${P}l0s0.so ${P}l2s0.so ${P}l0s2.so ${P}l2s2.so > $O/chan_2.log 2>&1 &&
KIND=fft timeout -k 10 200 python tools/probe/chan_libs_ab.py ${P}l2s2.so ${P}l0s2.so ${P}l2s0.so ${P}l0s0.so > $O/fft_1.log 2>&1
