#!/bin/bash
# GPU session: replicated cost probe, 1-GPU bench, rocprofv3 kernel stats of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/replicated_probe.py > gpurun_out/replicated_probe.log 2>&1 && echo "probe ok" && \
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.log 2>&1 && echo "bench ok" && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4 -o run -- python3 bench.py --steps 20 > gpurun_out/prof_r4.log 2>&1 && echo "prof ok"
rc=$?
grep -v amdgpu.ids gpurun_out/replicated_probe.log; tail -1 gpurun_out/bench1.log | cut -c1-400
exit $rc
