#!/bin/bash
# Process-to-process spread of the config-2 headline on one box: the headline alone in separate
# processes, then the default bench (all secondary lines, CPU baselines) and the headline alone again.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/procvar
export HSA_ENABLE_IPC_MODE_LEGACY=0
show() { python -c "import json;d=json.loads([x for x in open('$1') if x.startswith('{')][-1]);r=d['roofline'];print('$2',d['ms_per_step'],r['kernel_ms'],r['frac'],d['config']['roofline_pct_whole_step'])"; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline > gpurun_out/procvar/h$i.json 2>/dev/null || exit 1
  show gpurun_out/procvar/h$i.json head$i
done
timeout -k 10 500 python -u bench.py > gpurun_out/procvar/default.json 2>/dev/null || exit 1
show gpurun_out/procvar/default.json default
timeout -k 10 200 python -u bench.py --secondary none > gpurun_out/procvar/h3.json 2>/dev/null || exit 1
show gpurun_out/procvar/h3.json head3_cpu
timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline > gpurun_out/procvar/h4.json 2>/dev/null || exit 1
show gpurun_out/procvar/h4.json head4
