#!/bin/bash
# The GPU suite on the in-tree library, then an A/B of the opt-in spin-wait scheduling
# (RBGPU_SCHEDULE_SPIN=1) on the config-2 bench and a kernel-trace profile of the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/host
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/host/tests2.txt 2>&1 || { tail -30 gpurun_out/host/tests2.txt; exit 1; }
tail -2 gpurun_out/host/tests2.txt
bash scripts/ab_env.sh off - spin RBGPU_SCHEDULE_SPIN=1 off2 - spin2 RBGPU_SCHEDULE_SPIN=1 || exit 1
bash scripts/profab.sh main
timeout -k 10 120 python -u scripts/host_overhead.py > gpurun_out/host/overhead_off.txt 2>&1 && \
RBGPU_SCHEDULE_SPIN=1 timeout -k 10 120 python -u scripts/host_overhead.py > gpurun_out/host/overhead_spin.txt 2>&1
cat gpurun_out/host/overhead_off.txt gpurun_out/host/overhead_spin.txt
