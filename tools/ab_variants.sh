#!/bin/bash
# A/B timing of dev library variants (make -C csrc dev DEVTAG=<tag> DEVFLAGS=...): each variant's
# N2 loop twice, interleaved.  usage: tools/ab_variants.sh tag1 tag2 ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab.txt
: > $out
for rep in 1 2; do
  for t in "$@"; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20) || { echo "$t FAILED" >> $out; exit 1; }
    echo "$t rep$rep $r" | tee -a $out
  done
done
