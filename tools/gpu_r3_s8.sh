set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rss" > gpurun_out/r3_s8_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/rss_probe.py > gpurun_out/r3_s8_rss_probe.jsonl 2> gpurun_out/r3_s8_rss_probe.err && \
NFDP_EXT_DIR=variants/b256w3 timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_s8_pytest_b256w3.log 2>&1 && \
PASSES=1 bash tools/gpu_abn.sh variants/b256w3 variants/b256w2 && cp gpurun_out/abn_results.txt gpurun_out/r3_s8_abn.txt
