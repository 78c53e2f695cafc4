#!/bin/bash
# IPE step time vs the launch-group size (balanced groups)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for c in 4194304 8388608 16777216; do
  SQ_IPE16_CHUNK=$c timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/chunk_$c.log 2>&1
  rc=$?; echo "chunk=$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/chunk_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([s['ms'] for s in d['steps']], d['ms_per_step'])"
done
