#!/bin/bash
# split-chain hand-off timing: gpu test of the cross-plane path, then the unloaded probe with inbox timing
cd "$(dirname "$0")/.."
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_native_io_mq.py \
  -k split > gpurun_out/r6_xfer_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/live_bench.py --device cuda:0 --duration 0.5 --split acl,nat,l2fwd@1 --idle-only \
  > gpurun_out/r6_xfer_idle.json 2> gpurun_out/r6_xfer_idle.err || exit $?
echo done
