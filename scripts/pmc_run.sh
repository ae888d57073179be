#!/bin/bash
# PMC passes over one command, one rocprofv3 run per counter set (each set within the gfx950 block
# limits: <= 8 SQ_, <= 4 TCC_ with FETCH_SIZE = 3 and WRITE_SIZE = 2, so those two get passes of
# their own).  A pass that fails or times out ends the script.
# usage: scripts/pmc_run.sh <outdir under gpurun_out> "<command after --, no env/shell hops>" "<set>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out="gpurun_out/$1"; shift
cmd="$1"; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -s KILL "${PMC_TIMEOUT:-100}" rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- $cmd > "$out/p$i.log" 2>&1
  rc=$?
  echo "exit=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
done
