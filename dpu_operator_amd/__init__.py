import os as _os

# Persistent ring kernels hold their HIP stream's hardware queue for good.  HIP maps streams
# round-robin onto GPU_MAX_HW_QUEUES queues per device (4 by default), so a stream sharing a ring's
# queue (the default stream's copies, a learn or staging stream, a second plane's ring on the same
# GPU) would wait behind the resident grid forever.  Enough queues for every ring, its side streams
# and the default stream; effective when set before HIP starts (any entry point importing this
# package first: bench.py, the VSP, the tests' conftest).  A lower value from the environment
# (e.g. HIP's default written out as 4) is raised too: fewer queues can deadlock the live path.
try:
    _hwq = int(_os.environ.get("GPU_MAX_HW_QUEUES", "0"))
except ValueError:
    _hwq = 0
if _hwq < 16:
    _os.environ["GPU_MAX_HW_QUEUES"] = "16"
