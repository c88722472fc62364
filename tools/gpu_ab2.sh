#!/bin/bash
# Same-box A/B of a build variant (NFDP_EXT_DIR=$1) against the in-tree module: interleaved
# ablation runs only (variant, default, variant, default) — for experiment builds that are not
# feature-complete (no test run under the variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="$1"
for v in "$V" "" "$V" ""; do
  echo "variant=$v"
  NFDP_EXT_DIR="$v" timeout -k 10 200 python tools/ablate.py --rounds 5 > gpurun_out/ab2_run.log 2>&1 || exit 1
  cat gpurun_out/ab2_run.log
done
