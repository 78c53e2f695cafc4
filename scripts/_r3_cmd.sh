export TMPDIR=/tmp
B="python3 bench.py --steps 6 --warmup 5 --no-fit --no-qpca --ipe-steps 0 --no-hard --no-mnist"
R="recheck_fast|bounds_filter|recheck_rows|delta_scatter"
scripts/gpu_steps.sh \
 "tlb1|200|rm -rf /tmp/p1 && timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex '$R' --pmc TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS GRBM_GUI_ACTIVE -d /tmp/p1 -o p1 -- $B > gpurun_out/tlb1_bench.log 2>&1 && python3 scripts/pmc_summary.py \$(find /tmp/p1 -name '*.db') --top 6 > gpurun_out/tlb1.md" \
 "tlb2|200|rm -rf /tmp/p2 && timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex '$R' --pmc TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_UTCL1_THRASHING_STALL TCP_PENDING_STALL_CYCLES TA_BUSY_avr TD_TD_BUSY -d /tmp/p2 -o p2 -- $B > gpurun_out/tlb2_bench.log 2>&1 && python3 scripts/pmc_summary.py \$(find /tmp/p2 -name '*.db') --top 6 > gpurun_out/tlb2.md"
scripts/gpu_steps.sh \
 "il|300|for v in 0 1 0 1; do echo il \$v; SQ_SCREEN_IL=\$v python bench.py --warmup 5 --no-fit --no-qpca --no-mnist --ipe-steps 0 --no-hard | grep -o '\"ms_per_step\": [0-9.]*'; done" \
 "ilprof|200|rm -rf /tmp/p3 && SQ_SCREEN_IL=1 timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex 'recheck_fast' --pmc TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS GRBM_GUI_ACTIVE -d /tmp/p3 -o p3 -- $B > gpurun_out/il_bench.log 2>&1 && python3 scripts/pmc_summary.py \$(find /tmp/p3 -name '*.db') --top 6 > gpurun_out/tlb_il.md"
