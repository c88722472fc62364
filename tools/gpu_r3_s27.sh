set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s27_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/vxlan_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r3_s27_prof.log 2>&1
