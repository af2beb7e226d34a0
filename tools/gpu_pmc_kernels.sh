#!/bin/bash
# PMC passes (instruction mix, wave state, fetch / write bytes) over any
# probe program, summarised for the kernels whose name contains $FILTER.
#   FILTER=lrn TAG=lrn PROBE="tools/bench_lrn.py 2048" tools/gpu_pmc_kernels.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-k}
for pass in ${PASSES:-A B F W M}; do
  case $pass in
    A) ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES" ;;
    B) ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" ;;
    F) ctr="FETCH_SIZE" ;;
    W) ctr="WRITE_SIZE" ;;
    M) ctr="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16" ;;
    L) ctr="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" ;;
    D) ctr="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" ;;
    X) ctr="SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" ;;
  esac
  tools/gpu_step.sh 200 gpurun_out/pmc_${T}_$pass.log timeout -s KILL 150 \
    rocprofv3 --kernel-trace --pmc $ctr -d "$R/gpurun_out/pmc_${T}_$pass" \
    -o run --output-format csv -- python3 $PROBE || exit 1
done
python3 tools/pmc_kernels_summary.py "$T" "$FILTER"
exit 0
