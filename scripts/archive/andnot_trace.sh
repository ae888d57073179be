#!/bin/bash
# Kernel traces of the pairwise ANDNOT workload in separate processes (run-to-run bimodality study).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ant/r$i -o run -- python3 bench.py --workload pairwise_andnot --steps 3 --warmup 1 --no-cpu-baseline --secondary none > gpurun_out/ant/r$i.json 2>gpurun_out/ant/r$i.err || exit 1
  echo "run $i done"
done
