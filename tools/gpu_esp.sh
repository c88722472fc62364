#!/bin/bash
# ESP engine on the GPU: its tests, the throughput sweep, and a rocprofv3 kernel-stats pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-esp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ipsec.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 && echo "esp tests ok" && \
timeout -k 10 300 python -u tools/esp_bench.py --n 262144 > gpurun_out/${tag}_bench.log 2>&1 && echo "esp bench ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 tools/esp_bench.py --n 65536 --steps 5 > gpurun_out/${tag}_prof.log 2>&1 && echo "esp prof ok"
rc=$?
tail -3 gpurun_out/${tag}_pytest.log; cat gpurun_out/${tag}_bench.log | cut -c1-600
exit $rc
