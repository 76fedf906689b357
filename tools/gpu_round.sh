#!/bin/bash
# One GPU-box pass over everything the round's numbers come from. Usage: tools/gpu_round.sh TAG
# (run via gpurun). Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/rocprof.err && echo "rocprof ok" &&
tools/pmc_fir.sh $O/pmc && python3 tools/pmc_summary.py $O/pmc $((1<<25)) $O/pmc_fir.json > /dev/null && echo "pmc ok" &&
tools/pmc_fir.sh $O/pmc_casc --algo casc && python3 tools/pmc_summary.py $O/pmc_casc $((1<<25)) $O/pmc_casc.json > /dev/null && echo "pmc casc ok" &&
tools/pmc_fir.sh $O/pmc_mul4 --algo mul4 --log2n 26 && tools/pmc_fir.sh $O/pmc_chan --algo chan --log2n 26 &&
tools/pmc_fir.sh $O/pmc_d2 --algo mfma --decim 2 --log2n 26 && tools/pmc_fir.sh $O/pmc_d4 --algo mfma --decim 4 --log2n 26 &&
for L in mul4 chan d2 d4; do python3 tools/pmc_summary.py $O/pmc_$L $((1<<26)) $O/pmc_$L.json > /dev/null || exit 1; done &&
python3 - $O <<'PY' && echo "pmc legs ok" &&
import json, sys
o = sys.argv[1]; merged = {"_source": "profiles/pmc_legs.json (tools/gpu_round.sh: pmc_{mul4,chan,d2,d4}, 2^26 inputs per launch)"}
for l in ("mul4", "chan", "d2", "d4"):
    for k, v in json.load(open("%s/pmc_%s.json" % (o, l))).items():
        if k != "k_copy_v4":
            merged[k] = v
json.dump(merged, open(o + "/pmc_legs.json", "w"), indent=1)
PY
timeout -k 10 120 python tools/pfft_bench.py > $O/pfft_bench.json 2> $O/pfft_bench.err && echo "pfft bench ok" &&
timeout -k 10 400 build/tools/bench_configs 28 30 > $O/configs.jsonl 2> $O/configs.err && echo "configs ok" &&
# the exact-fp32 form's clock by the PMC method, beside bench.py's in-process sampler (clock_mhz)
[ "${CLOCK:-1}" = 1 ] && tools/pmc_clock.sh $O/clock_f32 --algo f32 > /dev/null && tools/pmc_clock.sh $O/clock_fir --algo mfma > /dev/null && echo "clock ok"
