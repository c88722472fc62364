set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_s17_pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s17_bench.json 2> gpurun_out/r3_s17_bench.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s17_prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-live --no-variants > $GRAFT_REPO_ROOT/gpurun_out/r3_s17_prof.log 2>&1
