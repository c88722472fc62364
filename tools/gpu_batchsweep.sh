#!/bin/bash
# Batch-size sweep of the 1-GPU bench: throughput vs p50 latency at that throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for b in 1048576 2097152 4194304 8388608; do
  timeout -k 10 200 python bench.py --steps 50 --batch $b --no-lowlat > gpurun_out/sweep_$b.log 2>&1 || exit 1
  tail -1 gpurun_out/sweep_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'], d['p50_latency_us'], d['p99_latency_us'])"
done
