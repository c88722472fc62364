set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r3_s7_ring.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rss_steer_list or rehearsal" > gpurun_out/r3_s7_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/rss_probe.py > gpurun_out/r3_s7_rss_probe.jsonl 2> gpurun_out/r3_s7_rss_probe.err
