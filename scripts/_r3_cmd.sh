export TMPDIR=/tmp
scripts/gpu_steps.sh \
 "ab|500|for v in cur nw8 cur nw8; do echo \$v; if [ \$v = nw8 ]; then export SQ_NATIVE_VARIANT=sq_learn_amd/_variants/_C_nw8.so; else unset SQ_NATIVE_VARIANT; fi; timeout -k 10 100 python benchmarks/estep_micro.py --prec x64 --iters 5 | grep x64; done"
