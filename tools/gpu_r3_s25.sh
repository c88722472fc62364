set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_l3_tunnels.py tests/test_overlay_sfc.py tests/test_dataplane_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s25_tun.log 2>&1 && \
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 --no-live --no-lowlat > gpurun_out/r3_s25_bench.json 2> gpurun_out/r3_s25_bench.err
