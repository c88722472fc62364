set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_overlay_sfc.py tests/test_frames.py tests/test_l3_tunnels.py tests/test_independent_l2.py tests/test_ring_gpu.py tests/test_livepath_engines.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s30_side.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s30_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/vxlan_probe.py egress > $GRAFT_REPO_ROOT/gpurun_out/r3_s30_prof.log 2>&1
