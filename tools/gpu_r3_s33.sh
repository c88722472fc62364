set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 --no-live --no-lowlat > gpurun_out/r3_s33_bench.json 2> gpurun_out/r3_s33_bench.err
