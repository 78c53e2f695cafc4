export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "gputest|700|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "smoke|180|python -c \"import __graft_entry__ as g; g.smoke()\"" \
 "bench|400|python bench.py --warmup 5"
