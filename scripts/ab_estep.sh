#!/bin/bash
# A/B of E-step variants: current extension vs build/variants/_C_<name>.so;
# names of the form env:VAR=VAL run the current extension with an env setting
names="$@"
what=${AB_WHAT:-estep}   # estep | reduce ; AB_ARGS: extra micro-benchmark flags
for rep in 1 2; do
  for v in cur $names; do
    unset SQ_NATIVE_VARIANT SQ_ESTEP_ROWS SQ_ESTEP_NW SQ_SEG_HALF SQ_SEG_RANGE
    case $v in
      cur) ;;
      env:*) export "${v#env:}" ;;
      *) export SQ_NATIVE_VARIANT=sq_learn_amd/_variants/_C_$v.so ;;
    esac
    echo -n "$v: "; timeout -k 10 120 python benchmarks/estep_micro.py --what $what --iters 20 $AB_ARGS 2>&1 | grep $what || exit 1
  done
done
