"""Write-ahead journal with snapshot compaction (checkpoint/resume of control-plane state).

The reference keeps all VSP state in memory and loses it on restart (SURVEY §5 "Checkpoint /
resume": only the CNI NetConf cache survives).  Components here append one JSON record per
mutation (fsync'd before the RPC returns), periodically compact to a snapshot, and replay the
snapshot + tail on start.  A torn last line (crash mid-append) is ignored.
Files: <dir>/<name>.jsonl (log), <dir>/<name>.snap.json (snapshot, atomically replaced).

Every record carries a monotonically increasing ``seq``; a snapshot stores the last ``seq`` it
covers (``_journal_seq``).  Compaction replaces the snapshot first and truncates the log second,
so a crash between the two leaves records the new snapshot already contains: ``load`` skips
every record at or below the snapshot's sequence number instead of replaying it twice (replay is
not idempotent, e.g. NF creation appends).
"""
from __future__ import annotations

import json
import os
import threading


class Journal:
    def __init__(self, directory: str, name: str = "state", compact_every: int = 1000):
        os.makedirs(directory, mode=0o700, exist_ok=True)
        self.log_path = os.path.join(directory, f"{name}.jsonl")
        self.snap_path = os.path.join(directory, f"{name}.snap.json")
        self.compact_every = compact_every
        self._lock = threading.Lock()
        self._n = 0
        snap, recs = self._read()
        self._seq = max([int((snap or {}).get("_journal_seq", 0))] + [int(r.get("seq", 0)) for r in recs])

    @property
    def seq(self) -> int:
        """Sequence number of the last appended record."""
        return self._seq

    def append(self, rec: dict) -> None:
        with self._lock:
            self._seq += 1
            line = json.dumps(dict(rec, seq=self._seq), separators=(",", ":")) + "\n"
            with open(self.log_path, "a") as f:
                f.write(line)
                f.flush()
                os.fsync(f.fileno())
            self._n += 1

    def needs_compaction(self) -> bool:
        return self._n >= self.compact_every

    def compact(self, state: dict) -> None:
        tmp = self.snap_path + ".tmp"
        with self._lock:
            with open(tmp, "w") as f:
                json.dump(dict(state, _journal_seq=self._seq), f)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, self.snap_path)
            with open(self.log_path, "w") as f:
                f.flush()
                os.fsync(f.fileno())
            self._n = 0

    def load(self) -> tuple[dict | None, list[dict]]:
        """-> (snapshot or None, log records newer than the snapshot)."""
        snap, recs = self._read()
        floor = int((snap or {}).get("_journal_seq", 0))
        return snap, [r for r in recs if int(r.get("seq", floor + 1)) > floor]

    def _read(self) -> tuple[dict | None, list[dict]]:
        snap = None
        if os.path.exists(self.snap_path):
            with open(self.snap_path) as f:
                snap = json.load(f)
        recs: list[dict] = []
        if os.path.exists(self.log_path):
            with open(self.log_path) as f:
                for line in f:
                    if not line.strip():
                        continue
                    try:
                        recs.append(json.loads(line))
                    except ValueError:
                        break  # torn tail: everything before it is durable
        return snap, recs

    def reset(self) -> None:
        with self._lock:
            for p in (self.log_path, self.snap_path):
                try:
                    os.unlink(p)
                except FileNotFoundError:
                    pass
            self._n = 0
