# PMC passes over any command: bash tools/pmc_any.sh <tag> <kernel-regex> <python script + args...>
set -e
R=$GRAFT_REPO_ROOT; T=$1; KR=$2; shift 2
O=$R/gpurun_out/pmc_$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE TA_BUSY_avr TA_ADDR_STALL_CYCLES_sum" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --kernel-include-regex "$KR" --output-format csv -d $O/p$i -o p$i -- python3 "$@" > $O/p$i.log 2>&1
done
