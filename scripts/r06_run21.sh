#!/bin/bash
# Full GPU suite on the product tree, then BSI RANGE step time: relaxed hand-off (product) vs system release (bsirel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6bsi; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
for r in 1 2 3; do
  for v in base bsirel; do
    if [ "$v" = base ]; then unset RBGPU_LIB; else export RBGPU_LIB=$PWD/abvar/$v/librbgpu.so; fi
    timeout -k 10 200 python3 bench.py --workload bsi_range --secondary none --steps 50 --warmup 5 --no-cpu-baseline > $o/$v.$r.json 2> $o/$v.$r.err || { echo "BENCH FAILED $v"; tail -5 $o/$v.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$o/$v.$r.json').read().strip().splitlines()[-1]); print('$v r$r', d['ms_per_step'], d['roofline'].get('kernel_ms'))"
  done
done | tee $o/summary.txt
