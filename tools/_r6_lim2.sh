#!/bin/bash
# limiter on the final build (buffer-load bucket fetch)
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/limiter.py --rounds 5 --iters 20 > gpurun_out/r6_s35_limiter.json 2> gpurun_out/r6_s35_limiter.err || exit $?
echo done
