#!/bin/bash
# Round-end check of the final tree on one GPU: smoke(), the GPU suite, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 || { tail -20 gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gputests.txt 2>&1 || { tail -30 gpurun_out/final/gputests.txt; exit 1; }
tail -1 gpurun_out/final/gputests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python - <<'PY'
import json
l=json.loads([x for x in open('gpurun_out/final/bench.json') if x.startswith('{')][-1])
print('HEAD', l['value'], l['ms_per_step'], l['roofline']['frac'], l.get('step_ms'), l['config']['roofline_pct_whole_step'])
for k,v in l['secondary'].items():
    print(k, v.get('value'), v.get('ms_per_step'), v.get('roofline',{}).get('frac'))
PY
