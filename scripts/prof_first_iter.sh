#!/bin/bash
# headline first iterations (full filter sweep, then the first filtered
# list-mode sweeps); A/B of the list-mode row sets via SQ_LIST_RS
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rs in 0 2 auto; do
  if [ "$rs" = auto ]; then unset SQ_LIST_RS; else export SQ_LIST_RS=$rs; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_fi_$rs -o r -- \
    python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 \
    --steps 3 --warmup 0 > gpurun_out/prof_fi_$rs.log 2>&1 || exit 1
  python3 scripts/prof_timeline.py /tmp/p_fi_$rs --marker estep_x64 --first 0 --last 3 --seq-all > gpurun_out/prof_fi_$rs.md
  rm -rf /tmp/p_fi_$rs
done
echo done
