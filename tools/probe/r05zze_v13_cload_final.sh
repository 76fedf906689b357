#!/bin/bash
# round 5: the whole-line chunk loads as the default (in-tree build): decimator + C++ runtime tests,
# and k_fir_mfma11 (D = 2, its plane layout padded alongside) c0 vs c1nt both orders.
export TMPDIR=/tmp
O=gpurun_out/r05zze; mkdir -p $O
L=build/abl/nsh_fir_mfma
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_cpp_runtime.py -x -q -k "decim or fir or runtime or cpp" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo "tests ok" &&
DECIM=2 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c0.so ${L}_c1nt.so > $O/d2_a.log 2>&1 &&
DECIM=2 ROUNDS=12 timeout -k 10 200 python tools/probe/lib_abn.py ${L}_c1nt.so ${L}_c0.so > $O/d2_b.log 2>&1
echo "rc=$?"
