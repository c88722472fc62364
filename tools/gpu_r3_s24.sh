set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_l3_tunnels.py tests/test_overlay_sfc.py tests/test_ipv6_flows.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s24_tun.log 2>&1 && \
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s24_bench.json 2> gpurun_out/r3_s24_bench.err
