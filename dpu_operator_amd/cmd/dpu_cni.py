"""`dpu-cni` — the CNI plugin binary (reference dpu-cni/dpu-cni.go:17-42)."""
import sys

from ..cni.shim import main

if __name__ == "__main__":
    sys.exit(main())
