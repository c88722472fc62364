#!/bin/bash
# Rehearsal of the multi-GPU bench path on a 1-GPU box (every rank on cuda:0, gloo exchanges:
# correctness, not a measurement), then a 1-GPU bench.  usage: tools/gpu_rehearse.sh <tag> [ranks]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-rh}
n=${2:-4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --gpus $n --steps 5 --warmup 2 --rehearse > gpurun_out/${tag}_n${n}.log 2>&1 && echo "rehearse n=$n ok" && \
timeout -k 10 400 python bench.py --steps 100 > gpurun_out/${tag}_bench.log 2>&1 && echo "bench ok"
rc=$?
grep '"metric"' gpurun_out/${tag}_n${n}.log | cut -c1-1500; tail -1 gpurun_out/${tag}_bench.log | cut -c1-1500
exit $rc
