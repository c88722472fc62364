set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_io.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_s3_pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/live_bench.py --device cuda --duration 1.0 > gpurun_out/r3_s3_live_gpu.json 2> gpurun_out/r3_s3_live_gpu.err && \
timeout -k 10 200 python -u tools/live_bench.py --device cuda --duration 1.0 --tx-workers 4 --threads 6 > gpurun_out/r3_s3_live_gpu_w4.json 2>> gpurun_out/r3_s3_live_gpu.err && \
timeout -k 10 200 python -u tools/live_bench.py --device cpu --duration 1.0 > gpurun_out/r3_s3_live_cpu.json 2> gpurun_out/r3_s3_live_cpu.err
