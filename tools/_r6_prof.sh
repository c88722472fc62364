#!/bin/bash
# kernel trace + stats of the bench's timed region and variants (no live block)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof -o bench -- python3 bench.py --steps 20 --warmup 5 --no-live \
  > gpurun_out/r6_prof_bench.json 2> gpurun_out/r6_prof_bench.err || exit $?
echo done
