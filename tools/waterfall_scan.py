"""Find buffer-descriptor "waterfall" loops in the device assembly of the data-plane kernels.

A buffer descriptor (make_buffer_rsrc) whose base or size the compiler cannot prove wave-uniform is
legal, but every access through it compiles to a loop over the lanes' distinct descriptors:
v_readfirstlane x4 -> v_cmp_eq_u64 x2 -> s_and_saveexec -> the access -> repeat.  In the r6 inbox
resume pass that loop cost 17 us per pass.  This compiles the sources to assembly and counts the
idiom per kernel (device.h wave_ptr / wave_u32 are the fix).

python tools/waterfall_scan.py [ring.hip kernels.hip ...]   (exit 1 if any kernel has one)
"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
FN = re.compile(r"^(_Z[^:\s]+):")


def scan_asm(text: str) -> collections.Counter:
    hits: collections.Counter = collections.Counter()
    cur, win = None, collections.deque(maxlen=12)
    for ln in text.splitlines():
        m = FN.match(ln)
        if m:
            cur = m.group(1)
            win.clear()
            continue
        s = ln.strip()
        if not s or s.startswith((".", ";")):
            continue
        win.append(s)
        if cur and s.startswith("s_and_saveexec_b64") and \
                sum(x.startswith("v_readfirstlane_b32") for x in win) >= 2 and \
                any(x.startswith("v_cmp_eq_u64") for x in win):
            hits[cur] += 1
    return hits


def compile_asm(src: Path) -> str:
    with tempfile.NamedTemporaryFile(suffix=".s") as f:
        subprocess.run([CLANG, "--offload-arch=gfx950", "-x", "hip", "-munsafe-fp-atomics", "-O3", "-std=c++17",
                        "-I", str(REPO / "csrc/nfdp"), "--cuda-device-only", "-S", str(src), "-o", f.name],
                       check=True, capture_output=True)
        return Path(f.name).read_text()


def main() -> int:
    srcs = sys.argv[1:] or ["ring.hip"]
    bad = 0
    for s in srcs:
        hits = scan_asm(compile_asm(REPO / "csrc/nfdp" / s))
        for k, v in hits.most_common():
            print(f"{s}: {v} waterfall loop(s) in {k}")
            bad += 1
    if not bad:
        print("no waterfall loops")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
