set -e
export TMPDIR=/tmp
for v in cur ${AB_VARIANTS}; do
  if [ $v = cur ]; then unset SQ_NATIVE_VARIANT; else export SQ_NATIVE_VARIANT=sq_learn_amd/_variants/_C_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --kernel-include-regex recheck -d gpurun_out/ab_$v -o run -- python3 bench.py --steps 20 --warmup 3 --ipe-steps 0 --no-fit --no-qpca > gpurun_out/ab_$v.log 2>&1
  echo "== $v" >> gpurun_out/ab_screen.txt
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log >> gpurun_out/ab_screen.txt
  python3 scripts/kern_avg.py gpurun_out/ab_$v/run_results.db recheck >> gpurun_out/ab_screen.txt
  rm -rf gpurun_out/ab_$v
done
