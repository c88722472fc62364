set -o pipefail
mkdir -p gpurun_out
for w in 2 4 8; do
timeout -k 10 200 python -u tools/live_bench.py --device cuda --duration 1.0 --tx-workers $w --threads 6 > gpurun_out/r3_s5_live_gpu_w$w.json 2>> gpurun_out/r3_s5_live_gpu.err || exit 1
done
timeout -k 10 200 python -u tools/live_bench.py --device cpu --duration 1.0 --tx-workers 4 --threads 6 > gpurun_out/r3_s5_live_cpu_w4.json 2>> gpurun_out/r3_s5_live_gpu.err
