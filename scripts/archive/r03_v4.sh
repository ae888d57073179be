#!/bin/bash
# Round-3 final-tree artifacts (profiles/r03/v4): smoke, GPU suite, the default bench line, the same
# under rocprofv3 --stats (CSV), a kernel trace of the headline for the union span and a step
# timeline, and the FETCH_SIZE / WRITE_SIZE passes for traffic.json.  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/v4
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
scripts/gpu_steps.sh \
  "v4_smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "v4_gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "v4_bench:400:python bench.py > gpurun_out/v4/bench_default.json" \
  "v4_stats:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v4/stats -o run -- python3 bench.py > gpurun_out/v4/bench_under_rocprof.json" \
  "v4_trace:240:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/v4/trace -o run -- python3 bench.py --secondary none --steps 10 --no-cpu-baseline > gpurun_out/v4/bench_under_trace.json" \
  "v4_pmc_fetch:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v4/pmc/p1 -o run -- $P" \
  "v4_pmc_write:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v4/pmc/p2 -o run -- $P"
