export TMPDIR=/tmp
export PYTHONPATH=$PWD
scripts/gpu_steps.sh \
 "chunk|400|for c in 128 512 4096; do echo chunk \$c; SQ_CHUNK_MB=\$c timeout -k 10 120 python benchmarks/tsgemm_bench.py --reps 4 | grep -i 'cholqr2\|xw_tri\|gram'; done"
