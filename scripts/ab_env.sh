#!/bin/bash
# A/B of an environment toggle on the headline bench (same box, alternated):
#   bash scripts/ab_env.sh VAR "v1 v2 v1 v2"
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
var=$1; vals=$2
for v in $vals; do
  env "$var=$v" timeout -k 10 200 python bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard \
    --no-mnist --no-pipeline > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); e=d['extra']; print('$var=$v', round(d['ms_per_step'],4), round(e['first_iter_ms'],3), round(e['share8_ms_per_step'],4))"
done
