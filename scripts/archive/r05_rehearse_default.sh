#!/bin/bash
# The driver's N=2 scaling command (default bench, every secondary line) rehearsed on a one-GPU box: two
# ranks on device 0, collectives over gloo (RBGPU_DIST_BACKEND=gloo RBGPU_SAME_DEVICE=1).  Not scaling
# evidence (both ranks share one GPU): it checks that every line's N>1 path runs end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5n2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 20; done ) &
HB=$!
RBGPU_DIST_BACKEND=gloo RBGPU_SAME_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err
rc=$?
kill $HB
echo "rc=$rc"
tail -5 $O/bench_n2.err
python3 - $O/bench_n2.json <<'PY'
import json, sys
ls = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
d = ls[-1]
print("HEAD", d.get("n_gpus"), d.get("value"), d.get("ms_per_step"), d["config"].get("parallelism"))
for k, v in d.get("secondary_summary", {}).items():
    print(k, v)
PY
exit $rc
