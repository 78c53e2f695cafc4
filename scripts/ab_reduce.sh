#!/bin/bash
# A/B: current extension vs build/variants/_C_oldseg.so on the reduce micro-benchmark
for rep in 1 2; do
  for v in cur old; do
    if [ $v = old ]; then export SQ_NATIVE_VARIANT=build/variants/_C_oldseg.so; else unset SQ_NATIVE_VARIANT; fi
    echo -n "$v d=256: "; timeout -k 10 120 python benchmarks/estep_micro.py --what reduce --iters 20 2>&1 | grep reduce || exit 1
    echo -n "$v d=32 : "; timeout -k 10 120 python benchmarks/estep_micro.py --what reduce --d 32 --k 256 --iters 20 2>&1 | grep reduce || exit 1
  done
done
