set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcd
for d in 2 4; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/pmcd/d${d}p1 -o run --output-format csv -- python3 tools/fir_one.py --decim $d --log2n 28 --reps 5 > gpurun_out/pmcd/d${d}p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcd/d${d}p2 -o run --output-format csv -- python3 tools/fir_one.py --decim $d --log2n 28 --reps 5 > gpurun_out/pmcd/d${d}p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcd/d${d}kt -o run --output-format csv -- python3 tools/fir_one.py --decim $d --log2n 28 --reps 5 > gpurun_out/pmcd/d${d}kt.log 2>&1
done
