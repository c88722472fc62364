#!/bin/bash
# One GPU session: tests, smoke, bench, kernel-trace profile.  Each GPU step has its own limit;
# steps are chained with && so the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python bench.py > gpurun_out/bench1.log 2>&1 && echo "bench ok" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-lowlat > gpurun_out/prof.log 2>&1 && echo "prof ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log | tail -2; tail -2 gpurun_out/bench1.log
exit $rc
