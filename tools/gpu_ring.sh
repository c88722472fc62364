#!/bin/bash
# GPU session: persistent ring kernel tests (each under its own time limit), then the full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_ring_gpu.py -x -v -s --timeout 100 --timeout-method thread > gpurun_out/ring_tests.log 2>&1 && echo "ring tests ok" && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "gpu suite ok"
rc=$?
grep -E "PASS|FAIL|ERROR|ring p50|Error|error" gpurun_out/ring_tests.log | head -30; tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
