#!/bin/bash
# GPU session: tests (incl. replicated REMOTE kernel), replicated cost probe, 1-GPU bench, profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && \
timeout -k 10 400 python tools/replicated_probe.py > gpurun_out/replicated_probe.log 2>&1 && echo "probe ok" && \
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.log 2>&1 && echo "bench ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/replicated_probe.log | grep -v amdgpu.ids; tail -1 gpurun_out/bench1.log | cut -c1-300
exit $rc
