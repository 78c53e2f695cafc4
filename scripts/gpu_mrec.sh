#!/bin/bash
# gap records: GPU tests, headline bench with records on / off, profile
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_multi_records_gpu.py tests/test_failure_pruning_gpu.py \
  tests/test_estep_precision_gpu.py > gpurun_out/mrec_tests.log 2>&1 || { tail -40 gpurun_out/mrec_tests.log; exit 1; }
tail -3 gpurun_out/mrec_tests.log
for v in 1 0 1; do
  SQ_MULTI_RECORDS=$v timeout -k 10 200 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard \
    --no-mnist --no-pipeline > gpurun_out/mrec_bench_$v.json 2> gpurun_out/mrec_bench_$v.err || exit 1
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); e=d["extra"]; print(sys.argv[2], round(d["ms_per_step"],4), e.get("phase_ms"), e.get("multi_rows_last"), e.get("gap_rows_last"), e.get("inertia_last"))' gpurun_out/mrec_bench_$v.json $v
done
bash scripts/prof_headline.sh
