#!/bin/bash
# naive_xor records by 256-key x 32-member tiles (abvar/rquad) vs the 128 x 64 tiles: wide parity tests under the
# variant, then config-4 XOR setup (records build) interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6rquad; mkdir -p $o
RBGPU_LIB=$PWD/abvar/rquad/librbgpu.so timeout -k 10 900 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $o/gputests.txt; exit 1; }
tail -1 $o/gputests.txt
for r in 1 2 3; do
  for v in base rquad; do
    if [ "$v" = base ]; then unset RBGPU_LIB; else export RBGPU_LIB=$PWD/abvar/$v/librbgpu.so; fi
    timeout -k 10 300 python3 bench.py --workload wide_xor_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline > $o/$v.$r.json 2> $o/$v.$r.err || { echo "BENCH FAILED $v"; tail -5 $o/$v.$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o/$v.$r.json').read().strip().splitlines()[-1])
print('$v r$r', 'step', d['ms_per_step'], 'setup', d['setup']['ms'], 'krec', d['setup']['parts'].get('krec',{}).get('ms'), 'with', d.get('ms_per_step_with_setup'), 'card', d.get('result_cardinality'))"
  done
done | tee $o/summary.txt
