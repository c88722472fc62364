set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ipv6_flows.py tests/test_overlay_sfc.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_s23_v6.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s23_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s23_bench.json 2> gpurun_out/r3_s23_bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s23_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-live > $GRAFT_REPO_ROOT/gpurun_out/r3_s23_prof.log 2>&1
