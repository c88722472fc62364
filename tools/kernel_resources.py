"""Per-instance register / spill / scratch / occupancy table of the data-plane kernels (gfx950),
from the compiler's resource remarks: the guard for the hot kernels' register budget (see
docs/DATAPLANE.md "Register budget").

python tools/kernel_resources.py [--max-vgpr-spill N]   (exit 1 if a fused / ring instance spills more)
"""
import argparse
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
FIELDS = ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill")


def remarks(src: Path) -> list[dict]:
    sys.path.insert(0, str(REPO))
    from dpu_operator_amd.native.build import parse_resource_remarks

    cmd = [CLANG, "--offload-arch=gfx950", "-x", "hip", "-munsafe-fp-atomics", "-O3", "-std=c++17",
           "-I", str(REPO / "csrc/nfdp"), "--cuda-device-only", "-c", str(src), "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    return parse_resource_remarks(subprocess.run(cmd, capture_output=True, text=True).stderr)


def demangle(n: str) -> str:
    try:
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-vgpr-spill", type=int, default=32)
    a = ap.parse_args()
    bad = 0
    print(f"{'kernel':70s} {'VGPR':>5s} {'occ':>4s} {'scr':>5s} {'sSpill':>6s} {'vSpill':>6s}")
    for src in ("kernels.hip", "ring.hip"):
        for r in remarks(REPO / "csrc/nfdp" / src):
            if not any(k in r["name"] for k in ("fused_kernel", "ring_kernel")):
                continue
            name = demangle(r["name"]).replace("(nfdp::FusedArgs)", "").replace("(nfdp::RingArgs)", "")
            print(f"{name[:70]:70s} {r.get('VGPRs', 0):5d} {r.get('Occupancy [waves/SIMD]', 0):4d} "
                  f"{r.get('ScratchSize [bytes/lane]', 0):5d} {r.get('SGPRs Spill', 0):6d} {r.get('VGPRs Spill', 0):6d}")
            bad += r.get("VGPRs Spill", 0) > a.max_vgpr_spill
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
