set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_s14_pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s14_bench.json 2> gpurun_out/r3_s14_bench.err
