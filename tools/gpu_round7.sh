#!/bin/bash
# GPU session (round 1, session 4): gpu tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.log 2>&1 && echo "bench ok" && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r7 -o run -- python3 bench.py --steps 20 > gpurun_out/prof_r7.log 2>&1 && echo "prof ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench1.log | cut -c1-600
exit $rc
