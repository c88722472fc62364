"""dpu-operator on MI355X: control plane (Python) + HIP/CDNA4 data plane (native extensions).

The package leaves the HIP runtime's settings to its operator (GPU_MAX_HW_QUEUES included): the
resident ring grids and the streams around them are built to run within HIP's default queue
count (tests/test_ring_gpu.py runs the live paths with GPU_MAX_HW_QUEUES=4 set explicitly).
"""
