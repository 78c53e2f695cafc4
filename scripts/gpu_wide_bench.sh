#!/bin/bash
# IPE steps at wide rows: the ipe16 screen (values pass) vs the fp32 kernel
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "1000000 784 1024" "2000000 1000 256"; do
  set -- $cfg
  for u in 1 0; do
    SQ_IPE16=$u timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows $1 --d $2 --k $3 --steps 6 > gpurun_out/wb_${1}_${2}_${3}_$u.log 2>&1
    rc=$?; echo "rows=$1 d=$2 k=$3 ipe16=$u rc=$rc"; [ $rc -eq 0 ] || exit $rc
    tail -1 gpurun_out/wb_${1}_${2}_${3}_$u.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([s['ms'] for s in d['steps']], d['ms_per_step'])"
  done
done
