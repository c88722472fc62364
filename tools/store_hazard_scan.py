"""Find gfx950 buffer stores of more than 8 bytes whose data VGPRs the next instruction overwrites.

On gfx950 that sequence corrupted frame data (r5 s8): a raw buffer store (dwordx4, SGPR soffset)
directly followed by `v_lshlrev_b32 v2, 2, ...` writing its first data VGPR stored the NEW value
for some lanes - 4 frames of 64K, in the last chunk pass of the wave's coalesced frame store
(device.h wave_frames_store).  LLVM's hazard recognizer inserts the wait state for such stores only
when their soffset is not a register; device.h store_b128 guards every 16-B buffer store.

Input: `hipcc --cuda-device-only -S` assembly or `llvm-objdump -d` of a gfx950 code object.
Usage: python tools/store_hazard_scan.py FILE [...]   (exit status 1 when a site is found)
"""
import re
import sys

_STORE = re.compile(r"^(buffer_store_(?:dwordx3|dwordx4|b96|b128))\s+v\[(\d+):(\d+)\]")
_DST = re.compile(r"^(v_[a-z0-9_]+)\s+(?:v\[(\d+):(\d+)\]|v(\d+))[,\s]")
_FN = re.compile(r"^(?:[0-9a-f]+ )?<?(_Z\w+)>?:")


def _insns(text: str):
    fn = None
    for ln in text.splitlines():
        m = _FN.match(ln.strip())
        if m:
            fn = m.group(1)
            continue
        s = ln.split("//")[0].split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        yield fn, s


def scan_text(text: str) -> list[tuple[str, str, str]]:
    hits = []
    prev = None
    for fn, ins in _insns(text):
        if prev is not None:
            pfn, lo, hi, pins = prev
            d = _DST.match(ins + " ")
            if d and not d.group(1).startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_cmpx")):
                a, b = (int(d.group(2)), int(d.group(3))) if d.group(2) else (int(d.group(4)), int(d.group(4)))
                if a <= hi and b >= lo:
                    hits.append((pfn, pins, ins))
        m = _STORE.match(ins)
        prev = (fn, int(m.group(2)), int(m.group(3)), ins) if m else None
    return hits


if __name__ == "__main__":
    bad = 0
    for p in sys.argv[1:]:
        for fn, st, nx in scan_text(open(p).read()):
            bad += 1
            print(f"{p}: {fn}\n    {st}\n    {nx}")
    print(f"{bad} hazard site(s)")
    sys.exit(1 if bad else 0)
