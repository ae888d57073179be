#!/bin/bash
# Timing study of the config-4 XOR kernel: k_wide_runs_xor time per variant library (rocprofv3 stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/xab
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset RBGPU_LIB; else export RBGPU_LIB=$PWD/scratch/$v/librbgpu.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xab/$v -o run -- python3 bench.py --workload wide_xor_runs --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xab/$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/xab/$v/run_kernel_stats.csv')):
    if 'wide_runs_xor' in r['Name'] or 'k_wide_reduce' in r['Name']: print('$v', r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e6, 3), 'ms')
"
done
