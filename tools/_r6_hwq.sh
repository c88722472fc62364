#!/bin/bash
# the full GPU suite with the ring streams at the highest priority (NFDP_RING_STREAM=prio)
cd "$(dirname "$0")/.."
NFDP_RING_STREAM=prio timeout -k 10 560 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r6_s18_pytest_gpu_prio.log 2>&1
echo "prio rc=$?"
