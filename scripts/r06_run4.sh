#!/bin/bash
# The compaction tail (call-tail parity, headline A/B against RBGPU_NO_CALL_TAIL=1), workShyAnd on the SoA without
# the type load (parity, A/B against the packed records), then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_steps.sh \
  "tailtests:300:python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_async.py tests/test_gpu_pairwise.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "tailab:300:for i in 1 2 3; do RBGPU_NO_CALL_TAIL=1 python bench.py --secondary none --no-cpu-baseline --steps 20 > gpurun_out/r6tail_off_\$i.json && python bench.py --secondary none --no-cpu-baseline --steps 20 > gpurun_out/r6tail_on_\$i.json || exit 1; done" \
  "andab:400:scripts/r06_ab.sh r6andab2 2 'wide_runs_and|pack_records' '--workload wide_and_runs --secondary none --steps 3 --warmup 1 --no-cpu-baseline' base asoa0" \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
