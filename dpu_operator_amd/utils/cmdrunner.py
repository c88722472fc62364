"""Testable command execution (the reference shells out with exec.Command everywhere and notes
the tech debt, vspnetutils.go:64; here every external command goes through a Runner).

`HostRunner` runs real commands, optionally inside `chroot /host` (the VSP pods mount the node's
root at /host); `FakeRunner` records argv lists and answers from a table of canned results.
"""
from __future__ import annotations

import subprocess
from dataclasses import dataclass, field


class CommandError(RuntimeError):
    def __init__(self, argv: list[str], rc: int, out: str):
        super().__init__(f"command {' '.join(argv)!r} failed with exit code {rc}: {out.strip()[:400]}")
        self.argv, self.rc, self.out = argv, rc, out


class Runner:
    def run(self, argv: list[str], check: bool = True, host: bool = False, timeout: float = 60.0) -> str: ...


class HostRunner(Runner):
    def __init__(self, host_root: str = "/host"):
        self.host_root = host_root

    def run(self, argv, check=True, host=False, timeout=60.0):
        full = (["chroot", self.host_root] if host else []) + list(argv)
        r = subprocess.run(full, capture_output=True, text=True, timeout=timeout)
        out = (r.stdout or "") + (r.stderr or "")
        if check and r.returncode != 0:
            raise CommandError(full, r.returncode, out)
        return out


@dataclass
class FakeRunner(Runner):
    """Records commands; `responses` maps an argv prefix (tuple) -> (rc, output)."""
    responses: dict[tuple, tuple[int, str]] = field(default_factory=dict)
    calls: list[list[str]] = field(default_factory=list)

    def run(self, argv, check=True, host=False, timeout=60.0):
        full = (["chroot", "/host"] if host else []) + list(argv)
        self.calls.append(full)
        rc, out = 0, ""
        best = -1
        for prefix, resp in self.responses.items():
            if tuple(full[: len(prefix)]) == prefix and len(prefix) > best:
                best, (rc, out) = len(prefix), resp
        if check and rc != 0:
            raise CommandError(full, rc, out)
        return out

    def commands(self, head: str | None = None) -> list[str]:
        cmds = [" ".join(c) for c in self.calls]
        return [c for c in cmds if head is None or c.startswith(head)]
