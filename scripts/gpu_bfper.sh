#!/bin/bash
# headline step time against the bounds filter's rows per thread (SQ_BF_PER)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 --steps 30 --warmup 10"
for per in 0 8 16 64 4; do
  SQ_BF_PER=$per timeout -k 10 200 python -u $B > gpurun_out/bfper_$per.log 2>&1
  rc=$?; echo "per=$per rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/bfper_$per.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"
done
