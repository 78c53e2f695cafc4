set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/gpu_all.log | tail -8
exit $rc
