#!/bin/bash
# Two PMC passes of SQ stall / LDS / L2 counters over the detector alone (tools/pmc_table.py TAG 2).
# Usage (gpurun): bash tools/pmc_sq.sh TAG [run_detector.py args]
TAG=$1; shift
exec_args="$*"
bash tools/pmc_detector.sh $TAG \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
