export TMPDIR=/tmp
B="python bench.py --warmup 5 --no-fit --no-qpca --no-mnist --ipe-steps 0"
scripts/gpu_steps.sh \
 "etests|600|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_estep_precision_gpu.py tests/test_estep_wide_gpu.py tests/test_mstep_incremental_gpu.py tests/test_kmeans_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py" \
 "ab|500|for v in 1 0 1 0; do echo half \$v; SQ_SCREEN_HALF=\$v $B | grep -o '\"ms_per_step\": [0-9.]*\|\"multi_fp64_rows_last\": [0-9]*\|\"inertia_last\": [0-9.]*\|\"hard_ms_per_step\": [0-9.]*'; done" \
 "tl10M|300|rm -rf /tmp/tl && rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- python3 bench.py --steps 20 --warmup 5 --no-fit --no-qpca --ipe-steps 0 --no-hard --no-mnist > gpurun_out/tl10_bench.log 2>&1 && python3 scripts/prof_timeline.py /tmp/tl --marker bounds_filter --last 3 > gpurun_out/timeline_10M.md"
