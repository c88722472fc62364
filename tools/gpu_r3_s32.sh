set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/vxlan_probe.py egress > gpurun_out/r3_s32_egress.log 2>&1 && \
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s32_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_s32_smoke.log 2>&1 && \
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_s32_bench.json 2> gpurun_out/r3_s32_bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s32_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-live > $GRAFT_REPO_ROOT/gpurun_out/r3_s32_prof.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/gpurun_out/r3_s32_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-lowlat --no-variants --no-live --rotate 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_s32_pmc.log 2>&1
