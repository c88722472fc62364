#!/bin/bash
# ESP kernels: in-tree build vs variant dirs ($@), interleaved, two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
  for v in "" "$@"; do
    echo "variant=${v:-in-tree} pass=$pass" | tee -a gpurun_out/esp_ab.txt
    NFDP_EXT_DIR="$v" timeout -k 10 200 python tools/esp_bench.py --sizes 64,1400 --n 262144 2>&1 | grep frame_bytes | tee -a gpurun_out/esp_ab.txt || exit 1
  done
done
