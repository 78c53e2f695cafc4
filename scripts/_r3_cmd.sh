export TMPDIR=/tmp
rm -f gpurun_out/pmc_x64.md
NO_TIMELINE=1 timeout -k 10 400 scripts/prof_r3.sh
