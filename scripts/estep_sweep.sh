#!/bin/bash
# E-step kernel ablations: SQ_ESTEP_DBG bit1 = no centroid staging after
# tile 1, bit2 = no top-2 epilogue (results invalid; timing only).
for nw in 4 8; do
  for dbg in 0 2 4 6; do
    echo -n "nw=$nw dbg=$dbg  "
    SQ_ESTEP_DBG=$dbg SQ_ESTEP_NW=$nw \
      timeout -k 10 120 python benchmarks/estep_micro.py --what estep --iters 10 2>&1 | grep estep || exit 1
  done
done
