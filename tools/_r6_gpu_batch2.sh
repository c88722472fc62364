#!/bin/bash
# round-6 GPU batch: counter names, limiter A/B, ring A/B, N=8 rehearsal on one GPU
cd "$(dirname "$0")/.."
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stop: rc $rc"; exit $rc; fi; }
timeout -k 5 60 rocprofv3 -L > gpurun_out/r6_s8_counters.txt 2>&1; ok $?
timeout -k 10 300 python -u tools/limiter.py --rounds 5 --iters 20 > gpurun_out/r6_s8_limiter.json 2> gpurun_out/r6_s8_limiter.err; ok $?
timeout -k 10 300 python -u tools/ring_ab.py --trials 5 > gpurun_out/r6_s8_ring_ab.json 2> gpurun_out/r6_s8_ring_ab.err; ok $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --rehearse --steps 5 --warmup 2 > gpurun_out/r6_s8_rehearse8.json 2> gpurun_out/r6_s8_rehearse8.err; ok $?
echo done
