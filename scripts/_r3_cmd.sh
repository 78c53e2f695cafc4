export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "gputest|700|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "smoke|180|python -c \"import __graft_entry__ as g; g.smoke()\"" \
 "bench|400|python bench.py --warmup 5" \
 "tl1p25|300|rm -rf /tmp/tl && rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- python3 bench.py --rows 1250000 --steps 20 --warmup 5 --no-fit --no-qpca --ipe-steps 0 --no-hard --no-mnist > gpurun_out/tl1p25_bench.log 2>&1 && python3 scripts/prof_timeline.py /tmp/tl --marker bounds_filter --last 3 > gpurun_out/timeline_1p25M.md" \
 "chunk|300|for c in 128 512 4096; do echo chunk \$c; SQ_CHUNK_MB=\$c python benchmarks/tsgemm_bench.py --reps 4 2>&1 | grep -i 'cholqr2\|sigma'; done"
