#!/bin/bash
# validation + headline/hard/share8 measurements (screen grid variants)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash scripts/gpu_screen.sh || exit 1
timeout -k 10 300 python benchmarks/hard_bench.py --unpruned > gpurun_out/hard5.json 2>/dev/null || exit 1
cat gpurun_out/hard5.json
for g in 512 2048; do
  SQ_SCREEN_GRID=$g timeout -k 10 200 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard \
    --no-mnist --no-pipeline > gpurun_out/grid_$g.json 2>/dev/null || exit 1
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d["ms_per_step"],4), round(d["extra"]["share8_ms_per_step"],4))' gpurun_out/grid_$g.json $g
done
