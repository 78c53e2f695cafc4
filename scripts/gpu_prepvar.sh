#!/bin/bash
# ipe16 prep time by part: one kernel trace per timing-only variant library
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for v in d0 d16 d32 d48; do
  SQ_NATIVE_VARIANT=$PWD/benchmarks/_ipev/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/pv_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_summary.py $(find /tmp/p_$v -name '*.db') --top 8 > gpurun_out/pv_$v.md
  rm -rf /tmp/p_$v
done
echo done
