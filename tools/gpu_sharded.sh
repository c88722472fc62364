#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --force-sharded --chunks 1 --steps 30 > gpurun_out/bench_sh1.log 2>&1 && echo "sh1 ok" && \
timeout -k 10 400 python bench.py --force-sharded --chunks 4 --steps 30 > gpurun_out/bench_sh4.log 2>&1 && echo "sh4 ok" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sh -o sh --output-format csv -- python3 bench.py --force-sharded --chunks 4 --steps 10 --warmup 2 --no-lowlat --rotate 1 > gpurun_out/prof_sh.log 2>&1 && echo "prof ok"
rc=$?
tail -1 gpurun_out/bench_sh1.log; tail -1 gpurun_out/bench_sh4.log
exit $rc
