#!/bin/bash
# One GPU session: gpu tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# usage: tools/gpu_session.sh <tag> [bench steps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-run}
steps=${2:-100}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 400 python bench.py --steps ${steps} > gpurun_out/${tag}_bench.log 2>&1 && echo "bench ok" && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 20 > gpurun_out/${tag}_prof.log 2>&1 && echo "prof ok"
rc=$?
tail -3 gpurun_out/${tag}_pytest_gpu.log; tail -2 gpurun_out/${tag}_smoke.log; tail -1 gpurun_out/${tag}_bench.log | cut -c1-900
exit $rc
