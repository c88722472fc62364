#!/bin/bash
# flow-bucket loads as raw buffer loads: default (flat) vs cache-policy 0 vs 2 (nt)
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u tools/ab_variants.py base= aux0=variants/aux0 aux2=variants/aux2 --rounds 4 --iters 50 \
  > gpurun_out/r6_s26_ab_probe_aux.jsonl 2>&1 || exit $?
echo done
