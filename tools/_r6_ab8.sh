#!/bin/bash
# fused-kernel geometry: 256-thread blocks (variants/blk256) and no kernarg reload (variants/karg0) vs in-tree
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u tools/ab_variants.py base= blk256=variants/blk256 karg0=variants/karg0 --rounds 4 --iters 50 \
  > gpurun_out/r6_s30_ab_geom.jsonl 2>&1 || exit $?
echo done
