"""In-tree build of the native extensions (gfx950 only).

Two modules, both built with the ROCm toolchain and placed next to this file so they travel with
the repository snapshot to the GPU box:

* ``_nfdp``  — HIP/CDNA4 data-plane kernels + host control structures (hipcc, ``-x hip``,
  ``--offload-arch=gfx950``).
* ``_agent`` — C++ host<->device control mailbox and control-plane agent (g++/hipcc host code).

Incremental: an object is rebuilt when its source or any header in its directory is newer.
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
                    "ipsec_cpu.cpp", "iox.cpp", "iox_gpu.cpp", "bindings.cpp"],
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


def _newest_dep(src: Path) -> float:
    """mtime of the newest local header `src` includes (transitively, `#include "x.h"` lines):
    a header edit rebuilds only the sources that see it."""
    import re

    seen, todo, newest = set(), [src], 0.0
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
            newest = max(newest, h.stat().st_mtime)
            todo.append(h)
    return newest


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
        cmd = [cxx, *common, "-pthread", "-c", str(src), "-o", str(obj)]
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


def _flags_changed(name: str, hip: bool) -> bool:
    """True when the experiment flags differ from the ones the objects were built with (the
    stamp is rewritten), so an NFDP_HIPCC_FLAGS build never survives into a default build."""
    flags = os.environ.get("NFDP_HIPCC_FLAGS", "").strip() if hip else ""
    stamp = BUILD / name / "flags.stamp"
    old = stamp.read_text() if stamp.exists() else None
    if old == flags:
        return False
    stamp.parent.mkdir(parents=True, exist_ok=True)
    stamp.write_text(flags)
    return True


def build_module(name: str, force: bool = False, verbose: bool = False) -> Path:
    spec = MODULES[name]
    d: Path = spec["dir"]
    out = (Path(VARIANT_OUT) if VARIANT_OUT else HERE) / f"{name}{EXT}"
    out.parent.mkdir(parents=True, exist_ok=True)
    force = _flags_changed(name, spec["hip"]) or force
    objs = []
    jobs = []
    for s in spec["sources"]:
        src = d / s
        obj = BUILD / name / (s + ".o")
        objs.append(obj)
        stale = force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, _newest_dep(src))
        if stale:
            jobs.append((src, obj))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 4)) as ex:
            list(ex.map(lambda j: _compile(j[0], j[1], spec["hip"], verbose), jobs))
    newest_obj = max(o.stat().st_mtime for o in objs)
    if force or jobs or not out.exists() or out.stat().st_mtime < newest_obj:
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
    hdr = _newest_header(d)
    objs, jobs = [], []
    for s in spec["sources"]:
        src = d / s
        obj = BUILD / spec["module"] / (s + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr):
            jobs.append((src, obj))
    for src, obj in jobs:
        _compile(src, obj, False, verbose)
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
