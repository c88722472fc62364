#!/bin/bash
# Same-box interleaved A/B of several build variants (NFDP_EXT_DIR dirs given as arguments)
# against the in-tree module: V1, default, V2, default, ... then the same order again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in $(seq 1 "${PASSES:-2}"); do
  for V in "$@"; do
    for v in "$V" ""; do
      echo "variant=${v:-default} pass=$pass" | tee -a gpurun_out/abn_results.txt
      NFDP_EXT_DIR="$v" timeout -k 10 200 python tools/ablate.py --rounds 3 > gpurun_out/abn_run.log 2>&1 || exit 1
      grep -E "ACL256|aclOff|ACL1024|Wild" gpurun_out/abn_run.log | tee -a gpurun_out/abn_results.txt
    done
  done
done
