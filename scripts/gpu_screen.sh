#!/bin/bash
# fp32 screen resolving wide bands: estep GPU tests, then the headline bench
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_multi_records_gpu.py tests/test_failure_pruning_gpu.py tests/test_estep_precision_gpu.py \
  tests/test_dmeans_pinned_gpu.py tests/test_runtime_gpu.py tests/test_distributed_gpu.py \
  > gpurun_out/screen_tests.log 2>&1 || { tail -30 gpurun_out/screen_tests.log; exit 1; }
tail -2 gpurun_out/screen_tests.log
timeout -k 10 200 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist \
  --no-pipeline > gpurun_out/screen_bench.json 2> gpurun_out/screen_bench.err || exit 1
python -c 'import json; d=json.load(open("gpurun_out/screen_bench.json")); e=d["extra"]; print(round(d["ms_per_step"],4), e.get("phase_ms"), e.get("multi_rows_last"), e.get("multi_fp64_rows_last"), e.get("share8_ms_per_step"), e.get("inertia_last"))'
bash scripts/prof_headline.sh
