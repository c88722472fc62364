set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_overlay_sfc.py tests/test_frames.py tests/test_l3_tunnels.py tests/test_independent_l2.py tests/test_ring_gpu.py tests/test_livepath_engines.py tests/test_dataplane_gpu.py tests/test_native_io.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_s34_side.log 2>&1
