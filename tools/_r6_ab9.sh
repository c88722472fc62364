#!/bin/bash
# fused-kernel grid: at most 2 workgroups per CU (variants/pc2: the resident count at 4 waves / SIMD) vs in-tree
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/ab_variants.py base= pc2=variants/pc2 --rounds 4 --iters 50 > gpurun_out/r6_s34_ab_grid.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py base= pc2=variants/pc2 --rounds 2 --iters 30 --acl wild > gpurun_out/r6_s34_ab_grid_wild.jsonl 2>&1 || exit $?
echo done
