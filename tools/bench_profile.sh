set -o pipefail
O=gpurun_out/r01i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/rocprof.err && echo "rocprof ok"
