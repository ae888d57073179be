#!/bin/bash
# Round artifacts on the GPU box: GPU tests, the default bench line, its rocprofv3 kernel stats,
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE) that feed profiles/<round>/traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/art
export TMPDIR=/tmp
P="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
scripts/gpu_steps.sh \
  "gputests:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench:300:python bench.py > gpurun_out/art/bench.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/art/stats -o run -- python3 bench.py > gpurun_out/art/bench_under_rocprof.json" \
  "pmc_fetch:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/art/pmc/p1 -o run -- $P" \
  "pmc_write:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/art/pmc/p2 -o run -- $P" \
  "pmc_tcc:240:timeout -s KILL 200 rocprofv3 --pmc TCC_BUSY_avr TCC_REQ_sum TCC_HIT_sum --output-format csv -d gpurun_out/art/pmc/p3 -o run -- $P --secondary none"
