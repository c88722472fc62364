#!/bin/bash
# A/B: fused-kernel self stamp (in-tree) vs the same build with a stamp kernel per batch vs the r6-s9 build
cd "$(dirname "$0")/.."
timeout -k 10 420 python -u tools/ab_variants.py self= kern=:kernel old=variants/kx0:kernel --rounds 4 --iters 50 \
  > gpurun_out/r6_s11_ab_stamp.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r6_s11_bench.json 2> gpurun_out/r6_s11_bench.err || exit $?
echo done
