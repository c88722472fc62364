#!/bin/bash
# Same-box A/B of the ESP kernels: a build variant (NFDP_EXT_DIR=$1) vs the in-tree module, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
  for v in "$1" "${2:-}"; do
    echo "variant=${v:-default} pass=$pass" | tee -a gpurun_out/esp_ab.txt
    NFDP_EXT_DIR="$v" timeout -k 10 200 python tools/esp_bench.py --sizes 64,1400 --n 262144 2>&1 | grep frame_bytes | tee -a gpurun_out/esp_ab.txt || exit 1
  done
done
