set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ipv6_flows.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_s22_v6.log 2>&1 && \
timeout -k 10 400 python -u tools/dbg/v6_bench_seq_dbg.py > gpurun_out/r3_s22_v6seq.log 2>&1
