#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_estep_precision_gpu.py tests/test_dmeans_pinned_gpu.py tests/test_failure_pruning_gpu.py \
  tests/test_kmeans_gpu.py > gpurun_out/ovf2_tests.log 2>&1 || { tail -30 gpurun_out/ovf2_tests.log; exit 1; }
tail -2 gpurun_out/ovf2_tests.log
for v in 1 0; do
  SQ_OVF2=$v timeout -k 10 300 python benchmarks/hard_bench.py > gpurun_out/hard_ovf2_$v.json 2>/dev/null || exit 1
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d["hard_ms_per_step"],3), round(d["hard_first_iter_ms"],3))' gpurun_out/hard_ovf2_$v.json $v
done
