#!/bin/bash
# Kernel-trace profiles of library variants on one bench workload:
#   scripts/profab.sh <name> ...   (abvar/<name>/librbgpu.so; "main" = the in-tree library)
# PROFAB_WORKLOAD picks the workload (default: the config-2 headline).  Summarise with
# scripts/prof_summary.py gpurun_out/profab/<name>/p_results.db.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/profab
export HSA_ENABLE_IPC_MODE_LEGACY=0
W=${PROFAB_WORKLOAD:-pairwise_and}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib=$GRAFT_REPO_ROOT/abvar/$v/librbgpu.so; [ "$v" = main ] && lib=$GRAFT_REPO_ROOT/roaringbitmap_amd/librbgpu.so
  RBGPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profab/$v -o p -- \
    python $GRAFT_REPO_ROOT/bench.py --workload $W --secondary none --steps 5 --warmup 2 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/profab/$v.json 2>&1 || exit 1
done
