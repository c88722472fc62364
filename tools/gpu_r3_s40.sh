set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ipv6_flows.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_s40_pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s40_bench.json 2> gpurun_out/r3_s40_bench.err && \
cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/gpurun_out/r3_s40_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --variant-steps 3 --no-lowlat --no-live --rotate 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_s40_pmc.log 2>&1
