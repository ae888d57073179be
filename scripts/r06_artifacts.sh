#!/bin/bash
# Round-6 artifacts on the GPU box: GPU suite, smoke, the default bench line, its rocprofv3 kernel stats, and
# the PMC passes (FETCH_SIZE, WRITE_SIZE: traffic.json; TCC busy / requests / hits of the headline).
# usage: scripts/r06_artifacts.sh [outdir under gpurun_out, default r6art]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r6art}
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
scripts/gpu_steps.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.txt 2>&1; r=\$?; tail -3 $O/gputests.txt; exit \$r" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
  "bench:400:python bench.py > $O/bench_default.json" \
  "stats:400:timeout -k 10 380 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.json" \
  "pmc_fetch:300:timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/p1 -o run -- $P" \
  "pmc_write:300:timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/p2 -o run -- $P" \
  "pmc_tcc:240:timeout -s KILL 200 rocprofv3 --pmc TCC_BUSY_avr TCC_REQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc/p3 -o run -- $P --secondary none"
