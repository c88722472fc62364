"""Static instruction histogram of one kernel in a `hipcc -S -g` listing, attributed to source lines.

python tools/isa_hist.py <file.s> <mangled-kernel-symbol> [top]
Counts VALU / SALU / LDS / VMEM / MFMA instructions per (file:line) from the `.loc` markers, so the
per-packet cost of each pipeline stage can be read without a thread trace.
"""
import collections
import re
import sys


def classify(op: str) -> str:
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "sync"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    files: dict[str, str] = {}
    hist = collections.defaultdict(collections.Counter)
    tot = collections.Counter()
    inside = False
    loc = ("?", 0)
    with open(path) as f:
        for line in f:
            s = line.strip()
            m = re.match(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)
            if m:
                files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
                continue
            if s.startswith(sym + ":"):
                inside = True
                continue
            if not inside:
                continue
            if s.startswith(".Lfunc_end"):
                break
            m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
            if m:
                loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
                continue
            if not s or s.startswith((".", ";")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c = classify(op)
            hist[loc][c] += 1
            tot[c] += 1
    print("totals:", dict(tot))
    rows = sorted(hist.items(), key=lambda kv: -(kv[1]["valu"] + kv[1]["salu"] + kv[1]["lds"] + kv[1]["vmem"]))
    for (fn, ln), c in rows[:top]:
        print(f"{fn}:{ln:<5d} valu={c['valu']:4d} salu={c['salu']:4d} lds={c['lds']:3d} vmem={c['vmem']:3d} "
              f"mfma={c['mfma']:3d} sync={c['sync']:3d}")
    per_file = collections.defaultdict(collections.Counter)
    for (fn, _), c in hist.items():
        per_file[fn].update(c)
    print("per file:")
    for fn, c in sorted(per_file.items(), key=lambda kv: -kv[1]["valu"]):
        print(f"  {fn:20s} {dict(c)}")


if __name__ == "__main__":
    main()
