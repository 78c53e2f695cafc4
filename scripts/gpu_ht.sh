#!/bin/bash
# IPE step vs the far band's hazard target (SQ_IPE16_HT)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for ht in 2e-4 4e-4 9e-4 2e-3; do
  SQ_IPE16_HT=$ht timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/ht_$ht.log 2>&1
  rc=$?; echo "ht $ht rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
