set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_l3_tunnels.py tests/test_dataplane_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_s11_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/rss_probe.py > gpurun_out/r3_s11_rss_probe.jsonl 2> gpurun_out/r3_s11_rss_probe.err && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s11_bench.json 2> gpurun_out/r3_s11_bench.err
