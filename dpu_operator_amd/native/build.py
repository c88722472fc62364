"""In-tree build of the native extensions (gfx950 only).

Two modules, both built with the ROCm toolchain and placed next to this file so they travel with
the repository snapshot to the GPU box:

* ``_nfdp``  — HIP/CDNA4 data-plane kernels + host control structures (hipcc, ``-x hip``,
  ``--offload-arch=gfx950``).
* ``_agent`` — C++ host<->device control mailbox and control-plane agent (g++/hipcc host code).

Incremental by content: an object is rebuilt when the hash of its source, the local headers it
includes (transitively) and its compile flags differs from the one recorded next to it.

Provenance: every module carries a digest of the exact sources it was built from (``source_digest``:
sources + their local headers + experiment flags), compiled into a marker string
(``DPUSRCDIGEST:<hex>``).  The loader (``native/__init__.py``) reads the marker out of the ``.so``
before importing it and refuses a binary whose digest is not the one of the sources in the tree,
so a stale extension cannot pass a GPU test silently.
Usage: ``python -m dpu_operator_amd.native.build [-v] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
# Experiment variants: NFDP_BUILD_OUT=<dir> puts the module (and its objects) there instead of
# next to this file; load it with NFDP_EXT_DIR=<dir> (see __init__.py).
VARIANT_OUT = os.environ.get("NFDP_BUILD_OUT")
if VARIANT_OUT:
    BUILD = BUILD / ("variant-" + Path(VARIANT_OUT).name)
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = "gfx950"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _includes() -> list[str]:
    import pybind11

    return ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"]]


MODULES = {
    "_nfdp": {
        "dir": CSRC / "nfdp",
        "sources": ["kernels.hip", "shard.hip", "pktio.hip", "ring.hip", "ipsec.hip", "host.cpp", "shard_cpu.cpp",
                    "ipsec_cpu.cpp", "iox.cpp", "iox_xdp.cpp", "iox_gpu.cpp", "bindings.cpp"],
        "hip": True,
    },
    "_agent": {
        "dir": CSRC / "agent",
        "sources": ["mbox.cpp", "ctrl_net.cpp", "config.cpp", "agent.cpp", "plugin_server.cpp", "soc.cpp", "bindings.cpp"],
        "hip": False,
    },
}

# Standalone native executables (no Python): the node control agent daemon.
EXES = {
    "dpu-cp-agent": {
        "dir": CSRC / "agent",
        "module": "_agent",
        "sources": ["mbox.cpp", "ctrl_net.cpp", "config.cpp", "agent.cpp", "plugin_server.cpp", "soc.cpp", "agent_main.cpp"],
    },
    # The CNI plugin kubelet execs on the host: static, no Python / package needed there.
    "dpu-cni": {
        "dir": CSRC / "cni",
        "module": "_cni",
        "sources": ["dpu_cni.cpp"],
        "ldflags": ["-static"],
    },
}


def _newest_header(d: Path) -> float:
    ts = [p.stat().st_mtime for p in d.glob("*.h")]
    return max(ts) if ts else 0.0


def _deps(src: Path) -> list[Path]:
    """Local headers `src` includes (transitively, `#include "x.h"` lines), sorted."""
    import re

    seen, todo = set(), [src]
    while todo:
        f = todo.pop()
        try:
            text = f.read_text(errors="replace")
        except OSError:
            continue
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
            h = (f.parent / m.group(1)).resolve()
            if h in seen or not h.exists():
                continue
            seen.add(h)
            todo.append(h)
    return sorted(seen)


def _hash_files(files, extra: str = "") -> str:
    import hashlib

    h = hashlib.sha256()
    for f in files:
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    h.update(extra.encode())
    return h.hexdigest()


def _hip_flags() -> str:
    return os.environ.get("NFDP_HIPCC_FLAGS", "").strip()


def source_digest(name: str) -> str:
    """Digest of everything a module is compiled from: its sources, the local headers they
    include and the experiment flags (hip modules).  Embedded in the module at link time."""
    spec = MODULES[name]
    d: Path = spec["dir"]
    files = set()
    for s in spec["sources"]:
        files.add((d / s).resolve())
        files.update(_deps(d / s))
    return _hash_files(sorted(files), _hip_flags() if spec["hip"] else "")


DIGEST_MARKER = b"DPUSRCDIGEST:"


def embedded_digest(so: Path) -> str | None:
    """The source digest compiled into a built module (None: no marker, a pre-provenance build)."""
    try:
        data = Path(so).read_bytes()
    except OSError:
        return None
    i = data.find(DIGEST_MARKER)
    if i < 0:
        return None
    return data[i + len(DIGEST_MARKER): i + len(DIGEST_MARKER) + 64].decode("ascii", "replace")


def _digest_object(name: str, digest: str, verbose: bool) -> Path:
    """A one-symbol object carrying the digest marker, linked into the module."""
    src = BUILD / name / "src_digest.cpp"
    obj = BUILD / name / "src_digest.cpp.o"
    text = (f'extern "C" __attribute__((visibility("default"), used)) const char dpu_{name.strip("_")}_src_digest[] = '
            f'"{DIGEST_MARKER.decode()}{digest}";\n')
    src.parent.mkdir(parents=True, exist_ok=True)
    if not obj.exists() or not src.exists() or src.read_text() != text:
        src.write_text(text)
        cmd = [shutil.which("g++") or "g++", "-fPIC", "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, capture_output=True)
    return obj


# HIP sources whose kernels' register / spill / occupancy figures are recorded at build time
# (compiler resource remarks -> <module>.resources.json next to the module; the spill guard test
# tests/test_kernel_resources.py and tools/kernel_resources.py read them)
RESOURCE_SOURCES = ("kernels.hip", "ring.hip")
RESOURCE_FIELDS = ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
                   "LDS Size [bytes/block]")


def parse_resource_remarks(text: str) -> list[dict]:
    """Rows {name, VGPRs, ..., VGPRs Spill} from `-Rpass-analysis=kernel-resource-usage` output."""
    import re

    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+)", line)
        if m and cur is not None and m.group(1).strip() in RESOURCE_FIELDS:
            cur[m.group(1).strip()] = int(m.group(2))
    return rows


def _compile(src: Path, obj: Path, hip: bool, verbose: bool) -> None:
    obj.parent.mkdir(parents=True, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", *_includes(), "-I", str(src.parent)]
    remarks = hip and src.name in RESOURCE_SOURCES
    if hip:
        extra = os.environ.get("NFDP_HIPCC_FLAGS", "").split()  # build-time experiments (-D...)
        cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common, *extra, "-c", str(src),
               "-o", str(obj)]
        if remarks:
            cmd.append("-Rpass-analysis=kernel-resource-usage")
    else:
        cxx = shutil.which("g++") or "g++"
        extra = [f for f in os.environ.get("NFDP_HIPCC_FLAGS", "").split() if f.startswith("-D")]   # (same experiments)
        cmd = [cxx, *common, *extra, "-pthread", "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    err = r.stderr
    if remarks:
        import json

        obj.with_suffix(".resources.json").write_text(json.dumps(parse_resource_remarks(err)))
        err = "\n".join(ln for ln in err.splitlines() if "kernel-resource-usage" not in ln)
    if verbose and err.strip():
        print(err, file=sys.stderr)


def _obj_hash(src: Path, hip: bool) -> str:
    return _hash_files([src.resolve(), *_deps(src)], ("hip:" + _hip_flags()) if hip else ("cxx:" + _hip_flags()))


def _stale(src: Path, obj: Path, hip: bool, force: bool) -> str | None:
    """None when `obj` was built from exactly this content, else the hash to record after building."""
    h = _obj_hash(src, hip)
    stamp = obj.with_name(obj.name + ".hash")
    if force or not obj.exists() or not stamp.exists() or stamp.read_text() != h:
        return h
    return None


def build_module(name: str, force: bool = False, verbose: bool = False) -> Path:
    spec = MODULES[name]
    d: Path = spec["dir"]
    out = (Path(VARIANT_OUT) if VARIANT_OUT else HERE) / f"{name}{EXT}"
    out.parent.mkdir(parents=True, exist_ok=True)
    objs = []
    jobs = []
    for s in spec["sources"]:
        src = d / s
        obj = BUILD / name / (s + ".o")
        objs.append(obj)
        h = _stale(src, obj, spec["hip"], force)
        if h is not None:
            jobs.append((src, obj, h))

    def run(j):
        _compile(j[0], j[1], spec["hip"], verbose)
        j[1].with_name(j[1].name + ".hash").write_text(j[2])

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 4)) as ex:
            list(ex.map(run, jobs))
    digest = source_digest(name)
    objs.append(_digest_object(name, digest, verbose))
    if force or jobs or not out.exists() or embedded_digest(out) != digest:
        if spec["hip"]:
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out)]
        else:
            cmd = [shutil.which("g++") or "g++", "-shared", "-fPIC", "-pthread", *map(str, objs), "-o", str(out)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {name}\n{r.stdout}\n{r.stderr}")
        if spec["hip"]:
            _write_resources(name, out, [BUILD / name / (s + ".resources.json") for s in spec["sources"]
                                         if s in RESOURCE_SOURCES])
    return out


def _write_resources(name: str, out: Path, parts: list[Path]) -> None:
    import json

    rows = {}
    for p in parts:
        if p.exists():
            rows[p.name.replace(".resources.json", "")] = json.loads(p.read_text())
    res = out.parent / f"{name}.resources.json"
    res.write_text(json.dumps({"flags": os.environ.get("NFDP_HIPCC_FLAGS", "").strip(), "sources": rows}, indent=0))


def build_exe(name: str, force: bool = False, verbose: bool = False) -> Path:
    """Link a standalone executable into dpu_operator_amd/native/bin/ (objects shared with the module)."""
    spec = EXES[name]
    d: Path = spec["dir"]
    objs, jobs = [], []
    for s in spec["sources"]:
        src = d / s
        obj = BUILD / spec["module"] / (s + ".o")
        objs.append(obj)
        h = _stale(src, obj, False, force)
        if h is not None:
            jobs.append((src, obj, h))
    for src, obj, h in jobs:
        _compile(src, obj, False, verbose)
        obj.with_name(obj.name + ".hash").write_text(h)
    out = HERE / "bin" / name
    out.parent.mkdir(exist_ok=True)
    if force or jobs or not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [shutil.which("g++") or "g++", "-pthread", *map(str, objs), *spec.get("ldflags", []), "-o", str(out)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {name}\n{r.stdout}\n{r.stderr}")
    return out


AGENT_CORE = ["mbox.cpp", "ctrl_net.cpp", "config.cpp", "agent.cpp", "plugin_server.cpp", "soc.cpp"]
SANITIZERS = {"tsan": ["-fsanitize=thread"], "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]}


# host-only sanitizer targets: sources and extra flags.  The I/O engine and its oracle backend are
# plain C++ (the GPU backend lives in iox_gpu.cpp), compiled against the HIP headers only.
SANITIZE_TARGETS = {
    "agent": {"dir": CSRC / "agent", "sources": AGENT_CORE + ["stress_main.cpp"], "flags": []},
    "iox": {"dir": CSRC / "nfdp", "sources": ["iox_stress.cpp", "iox.cpp", "host.cpp"],
            "flags": ["-D__HIP_PLATFORM_AMD__", "-I", str(ROCM / "include")]},
}


def build_sanitized(kind: str, verbose: bool = False, target: str = "agent") -> Path:
    """Host-only sanitizer build of a stress driver: the agent (csrc/agent/stress_main.cpp) or the
    native I/O engine (csrc/nfdp/iox_stress.cpp).  GPU sanitizers are unavailable on the MI355X
    pool; both are pure host code."""
    spec = SANITIZE_TARGETS[target]
    d = spec["dir"]
    out = BUILD / "sanitize" / f"{target}-stress-{kind}"
    out.parent.mkdir(parents=True, exist_ok=True)
    srcs = [d / s for s in spec["sources"]]
    newest = max(max(s.stat().st_mtime for s in srcs), _newest_header(d))
    if out.exists() and out.stat().st_mtime >= newest:
        return out
    cmd = [shutil.which("g++") or "g++", "-std=c++17", "-O1", "-g", "-pthread", *SANITIZERS[kind], *spec["flags"],
           "-I", str(d), *map(str, srcs), "-o", str(out)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"sanitizer build failed ({kind})\n{r.stdout}\n{r.stderr}")
    return out


def build_all(force: bool = False, verbose: bool = False) -> list[Path]:
    outs = []
    for name, spec in MODULES.items():
        if not (spec["dir"]).exists():
            continue
        if not all((spec["dir"] / s).exists() for s in spec["sources"]):
            continue
        outs.append(build_module(name, force=force, verbose=verbose))
    for name in EXES:
        outs.append(build_exe(name, force=force, verbose=verbose))
    return outs


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    for p in build_all(force=a.force, verbose=a.verbose):
        print(p)


if __name__ == "__main__":
    main()
