#!/bin/bash
# Session profile pass: (1) PMC of the certified E-step full sweep (x64 filter,
# every row), (2) kernel timeline of the 1.25M-row shard (the N=8 per-GPU
# share of the 10M headline).  Every rocprofv3 run under its own time limit;
# stops at the first failing step.  DBs live in /tmp, summaries in gpurun_out.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-10000000}
for pass in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  tag=$(echo $pass | cut -c1-12 | tr ' ' _)
  rm -rf /tmp/pmc_$tag
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $pass -d /tmp/pmc_$tag -o r \
    -- python3 benchmarks/estep_micro.py --prec x64 --iters 2 --n $N > gpurun_out/pmc_$tag.log 2>&1
  python3 scripts/pmc_summary.py $(find /tmp/pmc_$tag -name '*.db') --match estep_x64 >> gpurun_out/pmc_x64.md
done
if [ -z "$NO_TIMELINE" ]; then
  rm -rf /tmp/tl
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl \
    -- python3 bench.py --rows 1250000 --steps 20 --warmup 5 --no-fit --no-qpca --ipe-steps 0 \
       --no-hard --no-mnist > gpurun_out/tl_bench.log 2>&1
  python3 scripts/prof_timeline.py /tmp/tl --marker bounds_filter --last 6 > gpurun_out/timeline_1p25M.md
  python3 scripts/prof_summary.py /tmp/tl --top 30 >> gpurun_out/timeline_1p25M.md 2>&1 || true
fi
