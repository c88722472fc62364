set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg/v6_variant_dbg.py > gpurun_out/r3_s19_v6dbg.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_rss_streams_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_s19_rss_streams.log 2>&1 && \
timeout -k 10 300 python -u tools/rss_probe.py > gpurun_out/r3_s19_rss_probe.jsonl 2> gpurun_out/r3_s19_rss_probe.err
