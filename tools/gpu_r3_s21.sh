set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dbg/v6_bigbatch_dbg.py > gpurun_out/r3_s21_v6big.log 2>&1
