#!/bin/bash
# PMC passes of the config-4 wide kernels (k_wide_runs_and, k_wide_runs_xor): one bench run per
# counter set and workload, under gpurun_out/pmc_c4/<workload>/p<i>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
      "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_TAG_STALL_sum"
      "FETCH_SIZE"
      "TD_TD_BUSY_sum TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum")
for wl in ${PMC_WORKLOADS:-wide_and_runs wide_xor_runs}; do
  scripts/pmc_run.sh "pmc_c4/$wl" "python3 bench.py --workload $wl --secondary none --steps 2 --warmup 1 --no-cpu-baseline" "${SETS[@]}" || exit $?
done
