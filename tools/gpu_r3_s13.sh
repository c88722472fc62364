set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/abn_results.txt
PASSES=1 bash tools/gpu_abn.sh variants/noflowctr && cp gpurun_out/abn_results.txt gpurun_out/r3_s13_abn.txt && \
timeout -k 10 400 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_s13_pytest.log 2>&1
