set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rss or acl_wild" > gpurun_out/r3_s10_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/rss_probe.py > gpurun_out/r3_s10_rss_probe.jsonl 2> gpurun_out/r3_s10_rss_probe.err
