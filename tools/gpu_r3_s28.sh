set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_l3_tunnels.py tests/test_overlay_sfc.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s28_tun.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s28_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/vxlan_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r3_s28_prof.log 2>&1
