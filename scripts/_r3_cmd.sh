export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "stamps|200|SQ_NATIVE_VARIANT=sq_learn_amd/_variants/_C_stamp.so python benchmarks/estep_micro.py --prec x64 --iters 3 --stamps --bounds" \
 "tl10M|300|rm -rf /tmp/tl && rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- python3 bench.py --steps 20 --warmup 5 --no-fit --no-qpca --ipe-steps 0 --no-hard --no-mnist > gpurun_out/tl10_bench.log 2>&1 && python3 scripts/prof_timeline.py /tmp/tl --marker bounds_filter --last 4 > gpurun_out/timeline_10M.md"
