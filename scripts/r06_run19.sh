#!/bin/bash
# Phase study of the early-slot-word small kernel (census AND / OR).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r6early3; mkdir -p $o
for op in AND OR; do
  RBGPU_LIB=$PWD/abvar/sstudy/librbgpu.so timeout -k 10 120 python3 scripts/micro/small_study.py $op > $o/study_$op.txt 2>&1 || { echo "STUDY FAILED"; tail -20 $o/study_$op.txt; exit 1; }
done
cat $o/study_AND.txt $o/study_OR.txt
