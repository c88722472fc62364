#!/bin/bash
cd "$(dirname "$0")/.."
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_native_io_mq.py -k split > gpurun_out/r6_xfer_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/live_bench.py --device cuda:0 --duration 0.5 --split acl,nat,l2fwd@1 --idle-only > gpurun_out/r6_xfer_idle.json 2> gpurun_out/r6_xfer_idle.err || exit $?
timeout -k 10 150 python -u tools/live_bench.py --device cuda:0 --duration 1.0 --trials 3 --split acl,nat,l2fwd@1 > gpurun_out/r6_xfer_full.json 2> gpurun_out/r6_xfer_full.err || exit $?
echo done
