#!/bin/bash
# Same-box A/B of a build variant (NFDP_EXT_DIR=$1) against the in-tree module: GPU tests under
# the variant, then interleaved ablation runs (variant, default, variant, default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="$1"
NFDP_EXT_DIR="$V" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 && tail -1 gpurun_out/pytest_ab.log && \
for v in "$V" "" "$V" ""; do
  echo "variant=$v"
  NFDP_EXT_DIR="$v" timeout -k 10 200 python tools/ablate.py --rounds 5 > gpurun_out/ab_run.log 2>&1 || exit 1
  grep -E "lds\+mfmaACL256|lds\+aclOff|mfma\+mfmaACL1024" gpurun_out/ab_run.log
done
