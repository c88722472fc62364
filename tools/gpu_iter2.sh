#!/bin/bash
# Kernel iteration: GPU tests (bit-exact vs the oracle) -> interleaved ablation -> 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && \
timeout -k 10 400 python tools/ablate.py > gpurun_out/ablate.log 2>&1 && echo "ablate ok" && \
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.log 2>&1 && echo "bench ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; grep -v amdgpu.ids gpurun_out/ablate.log; tail -1 gpurun_out/bench1.log | cut -c1-300
exit $rc
