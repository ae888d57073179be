#!/bin/bash
# naive_xor (config 4, k_wide_runs_xor) counters, VERDICT r05 #3: one rocprofv3 --pmc pass per counter set over
# the product library, then the pass-duplication study builds (RBG_XOR_DUP=1 marks + check x2, 2 toggles x3,
# 3 flushes x2; abvar/xdup*) timed by kernel trace.  Output under gpurun_out/r6xor/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6xor
mkdir -p $O
export TMPDIR=/tmp
CMD="python3 bench.py --workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline"
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_REQ_sum TCC_BUSY_avr GRBM_GUI_ACTIVE"
      "FETCH_SIZE"
      "WRITE_SIZE")
libs=("base" "${@}")
O=${PMC_OUT:-$O}
for v in "${libs[@]}"; do
  if [ "$v" = base ]; then unset RBGPU_LIB; else export RBGPU_LIB=$PWD/abvar/$v/librbgpu.so; fi
  i=0
  nsets=${#SETS[@]}
  if [ "$v" != base ]; then nsets=2; fi  # the study builds: instruction / LDS counters and the kernel time
  for set in "${SETS[@]:0:$nsets}"; do
    i=$((i+1))
    mkdir -p $O/$v
    echo "=== $v pass $i: $set"
    timeout -s KILL 100 rocprofv3 --pmc $set --output-format csv -d $O/$v/p$i -o run -- $CMD > $O/$v/p$i.log 2>&1
    rc=$?
    echo "exit=$rc"
    if [ $rc -ne 0 ]; then tail -5 $O/$v/p$i.log; exit $rc; fi
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v/stats -o run -- $CMD > $O/$v/stats.log 2>&1 || exit 1
done
