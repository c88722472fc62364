set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s37_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_s37_smoke.log 2>&1 && \
timeout -k 10 800 python -u bench.py --steps 20 --warmup 5 --no-live > gpurun_out/r3_s37_bench.json 2> gpurun_out/r3_s37_bench.err
