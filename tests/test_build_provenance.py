"""Build provenance (native/build.py source_digest, native/__init__.py _check_provenance): every
module carries the digest of the sources it was built from, and the loader refuses a binary whose
digest differs from the sources in the tree, so a stale `.so` cannot pass a GPU test silently."""
import shutil
from pathlib import Path

import pytest

from dpu_operator_amd import native
from dpu_operator_amd.native import build as B


@pytest.mark.parametrize("name", ["_nfdp", "_agent"])
def test_built_modules_carry_the_digest_of_the_tree(name):
    so = Path(native.__file__).parent / f"{name}{B.EXT}"
    assert so.exists()
    assert B.embedded_digest(so) == B.source_digest(name)
    p = native.provenance()[name]
    assert p["built"] == p["sources"]


def test_digest_follows_every_input(tmp_path, monkeypatch):
    """A byte changed in a source, in a header it includes or in the experiment flags moves the
    digest; a header nobody includes does not."""
    d = tmp_path / "src"
    d.mkdir()
    (d / "a.cpp").write_text('#include "a.h"\nint f() { return A; }\n')
    (d / "a.h").write_text('#include "b.h"\n#define A B\n')
    (d / "b.h").write_text("#define B 1\n")
    (d / "unused.h").write_text("#define U 1\n")
    monkeypatch.setitem(B.MODULES, "_probe", {"dir": d, "sources": ["a.cpp"], "hip": True})
    monkeypatch.delenv("NFDP_HIPCC_FLAGS", raising=False)
    d0 = B.source_digest("_probe")
    (d / "unused.h").write_text("#define U 2\n")
    assert B.source_digest("_probe") == d0
    (d / "b.h").write_text("#define B 2\n")          # transitive include
    d1 = B.source_digest("_probe")
    assert d1 != d0
    monkeypatch.setenv("NFDP_HIPCC_FLAGS", "-DX=1")
    assert B.source_digest("_probe") != d1


def test_loader_refuses_a_stale_extension(tmp_path, monkeypatch):
    """A module whose embedded digest is not the tree's is refused when building is not allowed
    (the GPU box at round end runs without building)."""
    so = Path(native.__file__).parent / f"_agent{B.EXT}"
    fake_here = tmp_path / "native"
    fake_here.mkdir()
    stale = fake_here / so.name
    data = so.read_bytes()
    i = data.find(B.DIGEST_MARKER) + len(B.DIGEST_MARKER)
    stale.write_bytes(data[:i] + b"0" * 64 + data[i + 64:])
    assert B.embedded_digest(stale) == "0" * 64
    monkeypatch.setattr(native, "_HERE", fake_here)
    with pytest.raises(native.StaleExtensionError):
        native._check_provenance("_agent", autobuild=False)
    shutil.copy(so, stale)                          # the real build passes
    native._check_provenance("_agent", autobuild=False)
