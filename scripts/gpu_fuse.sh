#!/bin/bash
# Lloyd-step M-step changes: GPU tests touching the M-step / finalize,
# then the headline + share8 bench (ms per step) and a share8 kernel timeline
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_delta_lists_gpu.py \
  tests/test_mstep_incremental_gpu.py tests/test_kmeans_gpu.py tests/test_multi_records_gpu.py \
  tests/test_pipeline_gpu.py tests/test_runtime_gpu.py tests/test_failure_pruning_gpu.py \
  > gpurun_out/fuse_tests.log 2>&1 || { tail -30 gpurun_out/fuse_tests.log; exit 1; }
tail -1 gpurun_out/fuse_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
    > gpurun_out/fuse_b$i.json 2>gpurun_out/fuse_b$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fuse_b$i.json')); e=d['extra']; print(round(d['ms_per_step'],4), round(e['first_iter_ms'],3), round(e['share8_ms_per_step'],4))"
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_s8 -o r -- \
  python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
  --steps 3 --warmup 3 > gpurun_out/fuse_prof.log 2>&1 || exit 1
python3 scripts/prof_timeline.py /tmp/p_s8 --marker bounds_filter --last 3 > gpurun_out/fuse_timeline.md
python3 scripts/prof_timeline.py /tmp/p_s8 --marker bounds_filter --first 3 --last 1 > gpurun_out/fuse_timeline_head.md
rm -rf /tmp/p_s8
echo done
