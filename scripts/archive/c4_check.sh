#!/bin/bash
# Config-4 kernels after a change: the wide GPU tests (run-list fast paths), then the two config-4 bench
# lines and a kernel-trace profile of them.  Every GPU step has its own limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/c4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_wide.py tests/test_gpu_configs.py \
  > gpurun_out/c4/tests.txt 2>&1 || { tail -30 gpurun_out/c4/tests.txt; exit 1; }
tail -3 gpurun_out/c4/tests.txt
for w in wide_and_runs wide_xor_runs; do
  timeout -k 10 180 python -u bench.py --workload $w --secondary none --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/c4/$w.json 2> gpurun_out/c4/$w.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c4/$w.json').read().splitlines()[-1]);print('$w',d['ms_per_step'],d['roofline'].get('kernel_ms'),d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c4/prof -o c4 -- \
  python $GRAFT_REPO_ROOT/bench.py --workload wide_and_runs --secondary wide_xor_runs --steps 5 --warmup 2 \
  --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c4/prof.json 2>&1
cd $GRAFT_REPO_ROOT && PMC_WORKLOADS=pairwise_or timeout -k 10 400 scripts/pmc_c4.sh > gpurun_out/c4/pmc_or.log 2>&1
