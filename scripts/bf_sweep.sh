#!/bin/bash
# bounds-filter rows-per-thread sweep: kernel averages at 1.25M (share8) and 10M rows
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for per in 4 8 16; do
  SQ_BF_PER=$per timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/p_bf$per -o r -- \
    python3 bench.py --rows 1250000 --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 \
    --steps 20 --warmup 5 > gpurun_out/bf_$per.log 2>&1 || exit 1
  echo "1.25M PER=$per"; python3 scripts/pmc_summary.py $(find /tmp/p_bf$per -name '*.db') --top 40 | grep bounds_filter
  rm -rf /tmp/p_bf$per
done
for per in 16 20 32 64; do
  SQ_BF_PER=$per timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/p_bg$per -o r -- \
    python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 \
    --steps 20 --warmup 5 > gpurun_out/bg_$per.log 2>&1 || exit 1
  echo "10M PER=$per"; python3 scripts/pmc_summary.py $(find /tmp/p_bg$per -name '*.db') --top 40 | grep bounds_filter
  rm -rf /tmp/p_bg$per
done
