#!/bin/bash
# flow-bucket loads as raw buffer loads: cache policy 0 / 1 (sc0) / 16 (sc1) vs the flat default; then the ClassBench set
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u tools/ab_variants.py base= aux0=variants/aux0 aux1=variants/aux1 aux16=variants/aux16 --rounds 3 --iters 50 \
  > gpurun_out/r6_s27_ab_probe_aux.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py base= aux0=variants/aux0 --rounds 3 --iters 30 --acl wild \
  > gpurun_out/r6_s27_ab_probe_aux_wild.jsonl 2>&1 || exit $?
echo done
