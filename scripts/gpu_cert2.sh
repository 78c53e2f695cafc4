#!/bin/bash
# ipe16: law tests, 10M IPE bench, kernel timeline, two PMC passes at 4M rows
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ipe16_gpu.py > gpurun_out/cert_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/cert_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_cert -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 2 > gpurun_out/cert_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_cert -name '*.db') --top 20 > gpurun_out/cert_prof.md
python3 scripts/prof_timeline.py /tmp/p_cert --marker ipe16_prep --last 2 --seq-all > gpurun_out/cert_timeline.md
rm -rf /tmp/p_cert
S=scripts/pmc_summary.py
A="benchmarks/ipe_bench.py --rows 4000000 --steps 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d /tmp/p_i16a -o r -- python3 $A > gpurun_out/pmc_i16a.log 2>&1
rc=$?; echo "pmc a rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $S $(find /tmp/p_i16a -name '*.db') --match ipe16 --top 6 > gpurun_out/pmc_i16a.md
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD \
  -d /tmp/p_i16b -o r -- python3 $A > gpurun_out/pmc_i16b.log 2>&1
rc=$?; echo "pmc b rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $S $(find /tmp/p_i16b -name '*.db') --match ipe16 --top 6 > gpurun_out/pmc_i16b.md
rm -rf /tmp/p_i16a /tmp/p_i16b
echo done
