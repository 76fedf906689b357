#!/bin/bash
# round 4: k_fir_exact12's duration against the number of queued chunks (rocprof kernel trace):
# every 256th / 64th / 16th chunk exact
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
for k in 256 64 16; do
  INPUT=spike$k ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s$k -o run --output-format csv -- python3 tools/probe/lib_abn.py newsched_amd/lib/libnsh_hip.so > $O/s$k.log 2>&1 || exit 1
done
