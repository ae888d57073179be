#!/bin/bash
# N>1 rehearsal on a one-GPU box: every bench workload at N=1 and at N=2 (two ranks on device 0,
# collectives over gloo: RBGPU_DIST_BACKEND=gloo RBGPU_SAME_DEVICE=1).  Checks that the sharded
# paths run end to end and that the strong-scaling workloads (config 3/4/5: the same data split by
# key range) report the same global result as N=1.  Times are NOT scaling evidence (both ranks
# share one GPU).  Output: gpurun_out/n2/<workload>_n<N>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/n2
export HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --secondary none"
for w in ${REHEARSE_WORKLOADS:-pairwise_and wide_or wide_and_runs wide_xor_runs bsi_range}; do
  timeout -k 10 300 python bench.py --workload $w $ARGS > gpurun_out/n2/${w}_n1.json 2> gpurun_out/n2/${w}_n1.err || { echo "$w n1 failed"; exit 1; }
  RBGPU_DIST_BACKEND=gloo RBGPU_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload $w $ARGS \
    > gpurun_out/n2/${w}_n2.json 2> gpurun_out/n2/${w}_n2.err || { echo "$w n2 failed"; exit 1; }
  echo "$w done"
done
python scripts/rehearse_summary.py gpurun_out/n2
