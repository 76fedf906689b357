set -o pipefail
mkdir -p gpurun_out/grid2
for g in 2 8 2 16 4 32; do NSH_FIR_WG_PER_CU=$g LOG2N=28 VARIANTS=0 ROUNDS=10 timeout -k 10 100 python -u tools/fir_variants.py > gpurun_out/grid2/g$g.log 2>&1 || exit 1; grep median gpurun_out/grid2/g$g.log | sed "s/^/wg_per_cu=$g /"; done
