#!/bin/bash
# A/B: LDS transpose swizzle (in-tree) vs plain layout (variants/kx0) vs 3-wave headline (variants/occ3)
cd "$(dirname "$0")/.."
timeout -k 10 420 python -u tools/ab_variants.py swz= kx0=variants/kx0 occ3=variants/occ3 --rounds 4 --iters 50 \
  > gpurun_out/r6_s10_ab_256.jsonl 2>&1 || exit $?
timeout -k 10 420 python -u tools/ab_variants.py swz= kx0=variants/kx0 --rounds 3 --iters 30 --acl wild \
  > gpurun_out/r6_s10_ab_wild.jsonl 2>&1 || exit $?
echo done
