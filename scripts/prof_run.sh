#!/bin/bash
# rocprofv3 into a scratch dir OUTSIDE gpurun_out (the DBs are large), then a
# markdown summary into gpurun_out/<name>.md.
# usage: scripts/prof_run.sh NAME "rocprofv3 options" [--filter S] -- cmd args...
name=$1; shift
opts=$1; shift
filt=""
if [ "$1" == "--filter" ]; then filt="--filter $2"; shift 2; fi
[ "$1" == "--" ] && shift
export TMPDIR=/tmp
out=/tmp/prof_$name
rm -rf "$out"
mkdir -p gpurun_out
rocprofv3 $opts -d "$out" -o out -- "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
python3 scripts/prof_summary.py "$out" --top 40 $filt > "gpurun_out/$name.md" 2>&1
rm -rf "$out"
exit $rc
