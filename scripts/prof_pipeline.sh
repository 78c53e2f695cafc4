#!/bin/bash
# BASELINE config 5 (qPCA -> q-means, 50M x 128): stage + q-means phase
# seconds, then a kernel trace of the same run
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 240 python3 benchmarks/pipeline_bench.py > gpurun_out/pipe.json 2> gpurun_out/pipe.err || exit 1
cat gpurun_out/pipe.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_pipe -o r -- \
  python3 benchmarks/pipeline_bench.py > gpurun_out/prof_pipe.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_pipe -name '*.db') --top 40 > gpurun_out/prof_pipe.md
rm -rf /tmp/p_pipe
echo done
