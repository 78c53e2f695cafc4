export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "etests|600|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_estep_precision_gpu.py tests/test_mstep_incremental_gpu.py tests/test_kmeans_gpu.py tests/test_distributed_gpu.py tests/test_device_estimators_gpu.py" \
 "smoke|180|python -c \"import __graft_entry__ as g; g.smoke()\"" \
 "ab|400|for r in 1250000 10000000; do python bench.py --rows \$r --warmup 5 --no-fit --no-qpca --no-mnist --ipe-steps 0 --no-hard | grep -o '\"ms_per_step\": [0-9.]*\|\"rows_per_gpu\": [0-9]*'; done" \
 "tl1p25|300|rm -rf /tmp/tl && rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- python3 bench.py --rows 1250000 --steps 20 --warmup 5 --no-fit --no-qpca --ipe-steps 0 --no-hard --no-mnist > gpurun_out/tl1p25_bench.log 2>&1 && python3 scripts/prof_timeline.py /tmp/tl --marker bounds_filter --last 40 > gpurun_out/timeline_1p25M.md"
