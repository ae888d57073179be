#!/bin/bash
# RBG_PIPELINE A/B: the async tests on the pipelined build, then the async headline line
# of the in-tree library ("main") and of abvar/pipe, interleaved, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5pipe
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
RBGPU_LIB=abvar/pipe/librbgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -v --timeout 120 --timeout-method thread > $O/async_tests_pipe.txt 2>&1 || { tail -30 $O/async_tests_pipe.txt; exit 1; }
tail -1 $O/async_tests_pipe.txt
for round in 1 2; do
  for v in main pipe; do
    lib=abvar/$v/librbgpu.so; [ "$v" = main ] && lib=roaringbitmap_amd/librbgpu.so
    RBGPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --secondary pairwise_async --steps 30 > $O/${v}_$round.json || exit 1
    python -c "import json;d=json.loads(open('$O/${v}_$round.json').read().splitlines()[-1]);s=d['secondary']['pairwise_and_async'];print('$v', $round, 'sync', d['ms_per_step'], d['config']['roofline_pct_whole_step'], 'async', s['ms_per_step'], s['roofline_pct_whole_step'])"
  done
done
