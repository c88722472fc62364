#!/bin/bash
# live split-chain check: gpu tests of the cross-plane path, then the bench-scale live run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_native_io_mq.py tests/test_hop_pipeline_gpu.py > gpurun_out/r6_split_tests.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/live_bench.py --device cuda:0 --duration 0.5 --split acl,nat,l2fwd@1 \
  > gpurun_out/r6_split_live.json 2> gpurun_out/r6_split_live.err || exit $?
if [ "$1" = "bench" ]; then
  timeout -k 10 520 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_s6_bench.json 2> gpurun_out/r6_s6_bench.err || exit $?
fi
echo done
