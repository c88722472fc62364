set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_s6_bench.json 2> gpurun_out/r3_s6_bench.err
