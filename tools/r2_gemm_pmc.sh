#!/bin/bash
# Prefill GEMM counters (LLaMA-7B 4096x4096x512 and 4096->11008) -> gpurun_out/gpmc*/summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
for shape in "4096 4096" "4096 11008"; do
  set -- $shape
  export K=$1 M=$2
  SETS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS|FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_SALU" \
    bash tools/gemm_pmc.sh > gpurun_out/gpmc_${K}_${M}.txt 2>&1 || exit 1
  mv gpurun_out/gpmc gpurun_out/gpmc_raw_${K}_${M}
done
