#!/bin/bash
# A/B of native variants on the headline bench (Lloyd steps only) at two
# shard sizes: usage scripts/ab_bench.sh "cur" gpu_variants/_C_x.so ...
# ("cur" = the in-tree extension); stops at the first crash.
for rows in 1250000 10000000; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset SQ_NATIVE_VARIANT; else export SQ_NATIVE_VARIANT=$v; fi
    out=$(timeout -k 10 150 python bench.py --rows $rows --no-fit --no-qpca --ipe-steps 0 2>/dev/null)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v rows=$rows rc=$rc"; exit $rc; fi
    echo "$v rows=$rows $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["extra"]["phase_ms"], d["extra"]["inertia_last"])')"
  done
done
