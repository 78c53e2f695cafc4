export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "ptest|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py"
