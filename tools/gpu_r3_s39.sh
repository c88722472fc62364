set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_overlay_sfc.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_s39_pytest.log 2>&1  && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s39_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/vxlan_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r3_s39_probe.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/gpurun_out/r3_s39_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/vxlan_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r3_s39_pmc.log 2>&1
