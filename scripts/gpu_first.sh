#!/bin/bash
# why bench.py's first IPE step (817 ms) differs from ipe_bench's (465 ms)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --no-fit --no-qpca --no-hard --no-mnist --no-pipeline"
timeout -k 10 400 python -u bench.py $A --no-share8 > gpurun_out/first_noshare.log 2>&1
rc=$?; echo "noshare rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py $A > gpurun_out/first_share.log 2>&1
rc=$?; echo "share rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ipe_early.sh
