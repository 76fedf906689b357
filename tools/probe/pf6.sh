set -o pipefail
O=gpurun_out/pf6; mkdir -p $O; export TMPDIR=/tmp
(cd build/abl && timeout -k 10 300 python ../../tools/probe/pfft_ab.py pfft_new2.so pfft_b1.so pfft_b4.so pfft_b8.so pfft_b2.so > ../../$O/ab.log 2>&1) || echo "ab failed"
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 tools/fir_one.py --algo casc --log2n 25 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; break; }
done
echo pmc done
