set -o pipefail
mkdir -p gpurun_out/r01b
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01b/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py > gpurun_out/r01b/bench.json 2> gpurun_out/r01b/bench.err && echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01b/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r01b/bench_under_rocprof.json 2> gpurun_out/r01b/rocprof.err && echo "rocprof ok" &&
tools/pmc_fir.sh gpurun_out/r01b/pmc && python3 tools/pmc_summary.py gpurun_out/r01b/pmc $((1<<25)) gpurun_out/r01b/pmc_fir.json > /dev/null && echo "pmc ok"
