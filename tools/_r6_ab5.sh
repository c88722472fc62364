#!/bin/bash
# workgroup-start latency stamp (default now) vs a stamp kernel per batch, same build; then the bench
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/ab_variants.py wg= kern=:kernel --rounds 4 --iters 50 > gpurun_out/r6_s23_ab_wgstamp.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r6_s23_bench_nolive.json 2> gpurun_out/r6_s23_bench_nolive.err || exit $?
echo done
