#!/bin/bash
# the GPU suite, then the split-chain hand-off probe
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r6_suite_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/live_bench.py --device cuda:0 --duration 0.5 --split acl,nat,l2fwd@1 --idle-only \
  > gpurun_out/r6_xfer_idle.json 2> gpurun_out/r6_xfer_idle.err || exit $?
echo done
