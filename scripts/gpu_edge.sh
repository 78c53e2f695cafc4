#!/bin/bash
# dense-row band decisions certified against the fp32-faithful error bound:
# the E-step precision tests, the overflow diagnostic, the hard regime
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_estep_wide_gpu.py tests/test_estep_overflow_gpu.py tests/test_estep_precision_gpu.py \
  tests/test_delta_lists_gpu.py tests/test_multi_records_gpu.py > gpurun_out/edge_tests.log 2>&1 \
  || { tail -30 gpurun_out/edge_tests.log; exit 1; }
tail -1 gpurun_out/edge_tests.log
timeout -k 10 200 python benchmarks/ovf2_diag.py 2>&1 | grep -v amdgpu.ids | head -3
timeout -k 10 300 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-mnist --no-pipeline --no-share8 \
  > gpurun_out/edge_b.json 2>gpurun_out/edge_b.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/edge_b.json')); e=d['extra']; print(round(d['ms_per_step'],4), {k: e[k] for k in e if k.startswith('hard_')})"
