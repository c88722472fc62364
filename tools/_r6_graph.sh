#!/bin/bash
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dataplane_gpu.py > gpurun_out/r6_graph_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-live --no-variants > gpurun_out/r6_s36_bench_nolive.json 2> gpurun_out/r6_s36_bench_nolive.err || exit $?
echo done
