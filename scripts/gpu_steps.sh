#!/bin/bash
# Run GPU steps in order; stop at the first step that crashed (signal, abort,
# segfault, timeout).  Test failures (exit 1) do not stop later steps.
# usage: scripts/gpu_steps.sh "name1|timeout1|cmd1" "name2|timeout2|cmd2" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (timeout $to): $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" >> gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then
    echo "step $name ended with rc=$rc: stopping" >> gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
