#!/bin/bash
# ClassBench-style ACL: prefilter tiles (variants/pt), + source-first rule placement (variants/ptsrc) vs in-tree
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u tools/ab_variants.py base= pt=variants/pt ptsrc=variants/ptsrc --rounds 3 --iters 30 --acl wild \
  > gpurun_out/r6_s20_acl_ab_wild.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py base= ptsrc=variants/ptsrc --rounds 2 --iters 30 \
  > gpurun_out/r6_s20_acl_ab_256.jsonl 2>&1 || exit $?
echo done
