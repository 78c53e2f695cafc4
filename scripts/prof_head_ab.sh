#!/bin/bash
# steady-state headline kernel timeline (the last iterations of a 25-step
# run), A/B of an environment toggle: bash scripts/prof_head_ab.sh VAR "a b"
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
var=$1
for v in $2; do
  env "$var=$v" timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_h_$v -o r -- \
    python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 \
    --steps 5 --warmup 20 > gpurun_out/prof_h_$v.log 2>&1 || exit 1
  python3 scripts/prof_timeline.py /tmp/p_h_$v --marker bounds_filter --last 2 > gpurun_out/prof_h_$v.md
  rm -rf /tmp/p_h_$v
done
echo done
