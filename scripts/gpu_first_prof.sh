#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/ipe_first_step_profile.py > gpurun_out/fsp.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
