#!/bin/bash
# ClassBench-style ACL: batched prefilter-tile loop + source-first placement (variants/pt2src) vs in-tree
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u tools/ab_variants.py base= ptsrc=variants/ptsrc pt2src=variants/pt2src --rounds 3 --iters 30 --acl wild \
  > gpurun_out/r6_s21_acl_ab_wild.jsonl 2>&1 || exit $?
echo done
