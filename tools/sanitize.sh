#!/usr/bin/env bash
# Host-side ASan + UBSan pass over the C++ runtime (CPU only; GPU sanitizers are not
# available on the MI355X pool). Builds libnewsched.so and the CPU-side C++ tests with
# -fsanitize=address,undefined into $OUT (default /tmp/nsh_asan), links the normal
# libnsh_hip.so (its host code is not instrumented; no GPU is touched by these cases),
# and runs the scheduler, tag and 2-process remote-edge cases. Exit status != 0 on any
# sanitizer report.
#   tools/sanitize.sh            # build + run
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-/tmp/nsh_asan}
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
FLAGS="-O1 -g -std=c++17 -fPIC -pthread $SAN -Iinclude -Inewsched_amd/runtime/include \
 -Inewsched_amd/schedulers/include -Inewsched_amd/blocklib/include"
make -s newsched_amd/lib/libnsh_hip.so
objs=()
for f in newsched_amd/runtime/lib/*.cpp newsched_amd/schedulers/lib/*.cpp \
         newsched_amd/blocklib/lib/*.cpp newsched_amd/capi/*.cpp; do
    o="$OUT/$(echo "${f%.cpp}" | tr / _).o"
    objs+=("$o")
    [ "$o" -nt "$f" ] || g++ $FLAGS -c "$f" -o "$o" &
    while [ "$(jobs -rp | wc -l)" -ge 8 ]; do wait -n; done
done
wait
g++ -shared $SAN -pthread -o "$OUT/libnewsched.so" "${objs[@]}" -Lnewsched_amd/lib -lnsh_hip \
    -Wl,-rpath,"$PWD/newsched_amd/lib"
for t in qa_scheduler_mt qa_tags qa_remote_edge qa_fusion; do
    g++ $FLAGS -Itests/cpp -o "$OUT/$t" "tests/cpp/$t.cpp" -L"$OUT" -lnewsched \
        -Lnewsched_amd/lib -lnsh_hip -Wl,-rpath,"$OUT:$PWD/newsched_amd/lib" &
done
wait
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1
rc=0
timeout -k 5 600 "$OUT/qa_scheduler_mt" >"$OUT/sched.log" 2>&1 || { echo "qa_scheduler_mt FAILED"; rc=1; }
timeout -k 5 300 "$OUT/qa_tags" SchedulerMTTags >"$OUT/tags.log" 2>&1 || { echo "qa_tags FAILED"; rc=1; }
timeout -k 5 120 "$OUT/qa_fusion" >"$OUT/fusion.log" 2>&1 || { echo "qa_fusion FAILED"; rc=1; }
port=$((30000 + RANDOM % 20000))
for c in RemoteCpu.ChainRestart RemoteCpu.TwoCrossingsBothWays RemoteCpu.ReaderFinishesFirst; do
    QA_RANK=0 QA_PORT=$port timeout -k 5 120 "$OUT/qa_remote_edge" "$c" >"$OUT/remote0.log" 2>&1 &
    p0=$!
    QA_RANK=1 QA_PORT=$port timeout -k 5 120 "$OUT/qa_remote_edge" "$c" >"$OUT/remote1.log" 2>&1 || { echo "$c rank1 FAILED"; rc=1; }
    wait $p0 || { echo "$c rank0 FAILED"; rc=1; }
    cat "$OUT/remote0.log" "$OUT/remote1.log" >>"$OUT/remote.log"
done
if grep -lE "ERROR: (Address|Leak)Sanitizer|runtime error:" "$OUT"/*.log; then rc=1; fi
echo "sanitize: rc=$rc (logs in $OUT)"
exit $rc
