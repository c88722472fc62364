"""Register-budget guard for the hot kernels (CPU: reads the compiler's resource remarks).

The 4-wave fused instances run at the 128-VGPR cap; spilling more than the budget below moved
header dwords through scratch in the past (docs/DATAPLANE.md "Register budget": a 64-spill
build corrupted ~0.1 % of egress dwords).  The build records `-Rpass-analysis=kernel-resource-
usage` for kernels.hip / ring.hip in dpu_operator_amd/native/_nfdp.resources.json
(native/build.py); without a current record the remarks are produced here (slow: ~2 min).
"""
import json
import subprocess
from pathlib import Path

import pytest

from dpu_operator_amd.native.build import parse_resource_remarks

REPO = Path(__file__).resolve().parent.parent
SRC = REPO / "csrc" / "nfdp"
RECORD = REPO / "dpu_operator_amd" / "native" / "_nfdp.resources.json"

# the headline instance's spilled SGPRs (VGPR lanes: v_writelane / v_readlane): 332 before its table
# bases were read from the kernarg block per iteration (r5, kernels.hip NFDP_KARG_RELOAD); 234 in r6,
# 267 with the flow-bucket loads as buffer loads (their descriptor: +1.6 % / +0.7 % by A/B)
HEADLINE_SGPR_SPILLS = 270

# (source, mangled-name prefix, max spilled VGPRs, min waves / SIMD)
BUDGET = [
    # headline: lds hash + MFMA ACL, 1 GPU; and the MFMA-hash twin
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb0ELb0ELb0ELb0E", 15, 4),
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi2ELi1ELb0ELb0ELb0ELb0ELb0E", 12, 4),
    # early-fetch instances (2 waves / SIMD by design): no spills
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb1ELb0E", 0, 2),
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi2ELi1ELb0ELb1ELb0E", 0, 2),
    # steer-list instance (multi-GPU RSS): within one register of the hot instance
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb0ELb1E", 17, 4),
    # IPv6-capable 1-GPU instances (tables with IPv6 flows / rules): no frame prefetch, so within
    # the headline's budget
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb0ELb0ELb1E", 16, 4),
    ("kernels.hip", "_ZN4nfdp9v6_kernel", 0, 2),
    # split-chain instances (kHopXfer: the SFC hop pipeline across GPUs; spill-free at 3 waves / SIMD
    # they ran 12 % slower) and the hand-off / resume kernels
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb0ELb0ELb0ELb1E", 32, 4),
    ("kernels.hip", "_ZN4nfdp12fused_kernelILi2ELi1ELb0ELb0ELb0ELb0ELb1E", 14, 4),
    ("kernels.hip", "_ZN4nfdp13resume_kernel", 0, 4),
    ("kernels.hip", "_ZN4nfdp15hop_pack_kernel", 0, 8),
    # persistent ring kernels: no spills at all
    ("ring.hip", "_ZN4nfdp11ring_kernel", 0, 2),
    # side pass (replicas, learn events, outer headers): no spills
    ("kernels.hip", "_ZN4nfdp11side_kernel", 0, 3),
]

# kernels whose per-packet work must not touch scratch memory at all: a private array there costs a
# memory round trip per access (r5: the outer-header byte array put ~30 scratch loads / stores per
# packet into the side pass, 378 -> 266 us per 4M overlay-egress packets once built as dwords)
NO_SCRATCH = ["_ZN4nfdp11side_kernel", "_ZN4nfdp9v6_kernel", "_ZN4nfdp13resume_kernel", "_ZN4nfdp15hop_pack_kernel"]


def _rows() -> dict[str, list[dict]]:
    newest = max(p.stat().st_mtime for p in list(SRC.glob("*.h")) + [SRC / "kernels.hip", SRC / "ring.hip"])
    if RECORD.exists() and RECORD.stat().st_mtime >= newest:
        rec = json.loads(RECORD.read_text())
        if not rec.get("flags") and all(s in rec["sources"] for s in ("kernels.hip", "ring.hip")):
            return rec["sources"]
    out = {}
    for src in ("kernels.hip", "ring.hip"):
        cmd = ["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-x", "hip", "-munsafe-fp-atomics", "-O3",
               "-std=c++17", "-I", str(SRC), "--cuda-device-only", "-c", str(SRC / src), "-o", "/dev/null",
               "-Rpass-analysis=kernel-resource-usage"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        except (OSError, subprocess.TimeoutExpired) as e:
            pytest.skip(f"no gfx950 compiler here: {e}")
        out[src] = parse_resource_remarks(r.stderr)
    return out


@pytest.fixture(scope="module")
def rows():
    return _rows()


@pytest.mark.parametrize("src,prefix,max_spill,min_occ", BUDGET)
def test_hot_kernel_register_budget(rows, src, prefix, max_spill, min_occ):
    hits = [r for r in rows[src] if r["name"].startswith(prefix)]
    assert hits, f"{prefix} not found in {src}"
    for r in hits:
        assert r.get("VGPRs Spill", 0) <= max_spill, (r["name"], r)
        assert r.get("Occupancy [waves/SIMD]", 0) >= min_occ, (r["name"], r)
        assert r.get("ScratchSize [bytes/lane]", 0) <= 4 * max_spill + 64, (r["name"], r)


@pytest.mark.parametrize("prefix", NO_SCRATCH)
def test_no_scratch_in_per_packet_passes(rows, prefix):
    hits = [r for r in rows["kernels.hip"] if r["name"].startswith(prefix)]
    assert hits, prefix
    for r in hits:
        assert r.get("ScratchSize [bytes/lane]", 0) == 0, (r["name"], r)


def test_headline_sgpr_spill_budget(rows):
    r = [x for x in rows["kernels.hip"] if x["name"].startswith("_ZN4nfdp12fused_kernelILi1ELi1ELb0ELb0ELb0ELb0ELb0E")]
    assert r and r[0].get("SGPRs Spill", 0) <= HEADLINE_SGPR_SPILLS, r


def test_no_direct_to_lds_loads_in_the_data_plane():
    """No kernel of the data plane uses direct-to-LDS buffer loads (buffer_load ... lds).  ROCm 7.2's
    waitcnt insertion is unreliable for them: tools/lds_dma_probe.hip reads stale LDS in 41 % of its
    reads in a plain double-buffered loop whose second LDS read carries no s_waitcnt vmcnt for the
    DMA that wrote it (profiles/r5_s7_lds_dma_waitcnt_repro.txt) - the root cause of the round-2
    direct-to-LDS prefetch corruption (docs/DATAPLANE.md)."""
    import re

    hits = []
    for f in sorted(SRC.glob("*.h")) + sorted(SRC.glob("*.hip")):
        for i, line in enumerate(f.read_text().splitlines(), 1):
            if re.search(r"buffer_load_lds|global_load_lds|load_to_lds", line) and not line.lstrip().startswith("//"):
                hits.append(f"{f.name}:{i}")
    assert not hits, hits


def test_no_store_data_hazard_in_device_code(tmp_path):
    """No 16-B buffer store whose data VGPRs the next instruction overwrites (gfx950 store-data
    hazard, device.h store_b128; tools/store_hazard_scan.py): scans the built objects' gfx950 code."""
    import shutil
    import sys

    sys.path.insert(0, str(REPO / "tools"))
    from store_hazard_scan import scan_text

    llvm = Path("/opt/rocm/lib/llvm/bin")
    tools = [llvm / t for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    objs = sorted((REPO / "build" / "native" / "_nfdp").glob("*.hip.o"))
    if not all(t.exists() for t in tools) or not objs:
        pytest.skip("no gfx950 toolchain / no built objects")
    scanned = 0
    for o in objs:
        fb, co = tmp_path / (o.stem + ".fatbin"), tmp_path / (o.stem + ".co")
        r = subprocess.run([str(tools[0]), "--dump-section", f".hip_fatbin={fb}", str(o), str(tmp_path / "x.o")],
                           capture_output=True, text=True)
        if r.returncode != 0:   # (an object with no device code)
            continue
        subprocess.run([str(tools[1]), "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        dis = subprocess.run([str(tools[2]), "-d", "--mcpu=gfx950", str(co)], check=True, capture_output=True,
                             text=True).stdout
        hits = scan_text(dis)
        assert not hits, (o.name, hits[:3])
        scanned += 1
    assert scanned >= 3   # kernels / ring / shard at least
    shutil.rmtree(tmp_path, ignore_errors=True)


def test_ring_kernels_have_no_descriptor_waterfall_loops():
    """Buffer descriptors in the ring kernels are wave-uniform (tools/waterfall_scan.py): a
    non-uniform one compiles each access into a loop over the lanes.  Known: the coop instances'
    ACL tiles past the LDS copy (> 64 tiles) build their two descriptors from the LDS copy of the
    table set - one loop pair on that path.  The split-chain hand-off path had 26 more before its
    peer records moved into the kernargs (r6)."""
    import importlib.util
    import shutil

    if not shutil.which("/opt/rocm/lib/llvm/bin/clang++"):
        pytest.skip("no ROCm clang")
    spec = importlib.util.spec_from_file_location("waterfall_scan", REPO / "tools" / "waterfall_scan.py")
    ws = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ws)
    hits = ws.scan_asm(ws.compile_asm(REPO / "csrc" / "nfdp" / "ring.hip"))
    assert all(v <= 2 for v in hits.values()), hits
