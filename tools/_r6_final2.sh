#!/bin/bash
# final round-6 GPU pass: the GPU suite, smoke, the 1-GPU bench, a 2-rank rehearsal on this GPU
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r6_final_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final_smoke.log 2>&1 || exit $?
timeout -k 10 540 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6_final_bench.json 2> gpurun_out/r6_final_bench.err || exit $?
echo done
