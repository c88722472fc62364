#!/bin/bash
# GPU tests + device-resident bench + host-resident (pinned/SDMA) bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && \
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.log 2>&1 && echo "bench ok" && \
timeout -k 10 400 python bench.py --steps 50 --io host > gpurun_out/bench1_host.log 2>&1 && echo "bench host ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench1.log | cut -c1-250; tail -1 gpurun_out/bench1_host.log
exit $rc
