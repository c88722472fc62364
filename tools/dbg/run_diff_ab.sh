#!/bin/bash
# A/B the big-batch mismatch between a variant build ($1) and the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$1" ""; do
  echo "variant=${v:-default}"
  NFDP_EXT_DIR="$v" timeout -k 10 200 python -u tools/dbg/bigbatch_diff.py 2>&1 | grep "rows differ" || exit 1
done
