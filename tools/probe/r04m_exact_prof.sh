export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
INPUT=spike1 ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s1 -o run --output-format csv -- python3 tools/probe/lib_abn.py build/abl/x5.so > $O/s1.log 2>&1 &&
INPUT=spike64 ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s64 -o run --output-format csv -- python3 tools/probe/lib_abn.py build/abl/x5.so > $O/s64.log 2>&1 &&
ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s0 -o run --output-format csv -- python3 tools/probe/lib_abn.py build/abl/x5.so > $O/s0.log 2>&1
