#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_ring_gpu.py tests/test_dataplane_gpu.py -x -v -s --timeout 100 --timeout-method thread > gpurun_out/ring_tests.log 2>&1 && echo "tests ok" && \
timeout -k 10 300 python -u tools/ring_probe.py > gpurun_out/ring_probe.log 2>&1 && echo "probe ok"
rc=$?
grep -E "FAIL|ERROR|ring p50|Error|passed|failed" gpurun_out/ring_tests.log | head -20; grep -v amdgpu.ids gpurun_out/ring_probe.log
exit $rc
